"""High-level MCMC facade — drop-in for mlx_mcmc/inference/mcmc.py:10-246.

``MCMC(log_prob_fn).run(...)`` dispatches ``method='hmc'`` / ``'nuts'`` to
the MI355X kernels exactly as the reference's branches do (mcmc.py:83-133):
``key`` is built from ``random_seed``, extra kwargs go to the sampler,
samples are stored as NumPy arrays in ``.samples`` and the rate in
``.acceptance_rate``.  ``summary`` / ``print_summary`` follow mcmc.py:191-246,
computed on the device from the kept [C, S, D] sample buffer
(diagnostics.summarize: per-series moments and exact order statistics);
``diagnostics()`` adds per-element ESS and split R-hat.

``method='metropolis'`` (the reference default) follows mcmc.py:135-189: a
warmup run of ``metropolis_hastings`` with ``random_seed``, then a sampling
run from its last draw with ``random_seed + 1`` (both on the GPU, k_mh in
csrc/mh.h).  Unknown methods raise ``ValueError`` (mcmc.py:138).
"""
from __future__ import annotations

import numpy as np

from .. import diagnostics as _diag
from .. import random as _random
from ..kernels.hmc import hmc
from ..kernels.metropolis import metropolis_hastings
from ..kernels.nuts import nuts


class MCMC:
    """High-level MCMC inference interface."""

    def __init__(self, log_prob_fn):
        self.log_prob_fn = log_prob_fn
        self.samples = None
        self.acceptance_rate = None
        self.info = None

    def run(self, initial_params, num_samples=1000, num_warmup=1000, method='metropolis',
            proposal_scale=0.1, random_seed=0, verbose=True, **kwargs):
        if method in ('hmc', 'nuts'):
            if verbose:
                print(f"\n{'=' * 70}")
                print(f"MLX-MCMC: {method.upper()} Sampling")
                print(f"{'=' * 70}\n")
            sampler = hmc if method == 'hmc' else nuts
            kwargs = dict(kwargs)
            kwargs['return_info'] = True
            kwargs.setdefault('keep_on_device', True)
            samples, accept_rate, info = sampler(
                self.log_prob_fn, initial_params, num_samples=num_samples,
                num_warmup=num_warmup, key=_random.key(random_seed), **kwargs)
            self.samples = {k: np.array(v) for k, v in samples.items()}
            self.acceptance_rate = accept_rate
            self.info = info
            if verbose:
                print(f"\n{'=' * 70}")
                print("Sampling complete!")
                print(f"{'=' * 70}\n")
            return self.samples
        if method != 'metropolis':
            raise ValueError(f"Unknown sampling method: {method}")
        sampler = metropolis_hastings
        if verbose:
            print(f"\n{'=' * 70}")
            print(f"MLX-MCMC: {method.upper()} Sampling")
            print(f"{'=' * 70}\n")
        kwargs = dict(kwargs)
        kwargs['return_info'] = True
        kwargs.setdefault('keep_on_device', True)
        # warmup phase (mcmc.py:145-165): a sampler run whose last draw starts sampling
        if num_warmup > 0:
            if verbose:
                print(f"Warmup phase: {num_warmup} samples")
            wkw = dict(kwargs)
            wkw['keep_on_device'] = False
            warmup_samples, warmup_accept, winfo = sampler(
                self.log_prob_fn, initial_params, num_samples=num_warmup,
                proposal_scale=proposal_scale, random_seed=random_seed, verbose=verbose, **wkw)
            if verbose:
                print(f"Warmup acceptance rate: {float(np.mean(warmup_accept)):.2%}\n")
            if np.ndim(warmup_accept) == 0:
                final_warmup = {k: v[-1] for k, v in warmup_samples.items()}
            else:  # several chains: each continues from its own last draw
                C = len(warmup_accept)
                final_warmup = initial_params
                kwargs['initial_positions'] = np.concatenate(
                    [np.asarray(warmup_samples[n])[:, -1].reshape(C, -1)
                     for n in winfo.layout.names], axis=1)
        else:
            final_warmup = initial_params
        # sampling phase (mcmc.py:167-178)
        if verbose:
            print(f"Sampling phase: {num_samples} samples")
        samples, self.acceptance_rate, self.info = sampler(
            self.log_prob_fn, final_warmup, num_samples=num_samples,
            proposal_scale=proposal_scale,
            random_seed=random_seed + 1 if num_warmup > 0 else random_seed,
            verbose=verbose, **kwargs)
        if verbose:
            print(f"Sampling acceptance rate: {float(np.mean(self.acceptance_rate)):.2%}")
            print(f"\n{'=' * 70}")
            print("Sampling complete!")
            print(f"{'=' * 70}\n")
        self.samples = {k: np.array(v) for k, v in samples.items()}
        return self.samples

    def summary(self, credible_interval=0.95):
        """Per parameter: mean, std, median and the central credible interval
        over every chain, draw and element (mcmc.py:191-227)."""
        if self.samples is None:
            raise ValueError("Must run sampling first. Call run() method.")
        dev = getattr(self.info, "device_samples", None)
        if dev is not None:
            return _diag.summarize(dev, self.info.layout, credible_interval)
        return _diag.summarize(self.samples, None, credible_interval)

    def diagnostics(self, max_lag=100):
        """Per parameter: ESS per chain (examples/06_nuts_comparison.py:22-41
        rule), ESS summed over chains and split R-hat, shaped like the
        parameter (chain axis first for the per-chain ESS)."""
        if self.samples is None:
            raise ValueError("Must run sampling first. Call run() method.")
        dev = getattr(self.info, "device_samples", None)
        if dev is None:
            raise ValueError("diagnostics need the device samples (keep_on_device=True)")
        d = _diag.chain_diagnostics(dev, max_lag=max_lag, group=False)
        lay = self.info.layout
        out = {}
        C = d["ess"].shape[0]
        for name, shape, off in zip(lay.names, lay.shapes, lay.offsets):
            n = int(np.prod(shape)) if shape else 1
            out[name] = {"ess": d["ess"][:, off:off + n].reshape((C,) + tuple(shape)),
                         "ess_sum": d["ess_sum"][off:off + n].reshape(shape),
                         "r_hat": d["rhat"][off:off + n].reshape(shape)}
        return out

    def print_summary(self, credible_interval=0.95):
        summary = self.summary(credible_interval)
        print("\nPosterior Summary:")
        print("=" * 80)
        print(f"{'Parameter':<15} {'Mean':<10} {'Std':<10} {'Median':<10} "
              f"{f'{int(credible_interval * 100)}% CI':<20}")
        print("-" * 80)
        for name, st in summary.items():
            vals = list(st.values())
            ci = f"[{vals[3]:.3f}, {vals[4]:.3f}]"
            print(f"{name:<15} {st['mean']:<10.3f} {st['std']:<10.3f} {st['median']:<10.3f} "
                  f"{ci:<20}")
        print("=" * 80)
