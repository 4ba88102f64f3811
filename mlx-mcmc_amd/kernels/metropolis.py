"""Random-walk Metropolis-Hastings on MI355X — drop-in for
mlx_mcmc/kernels/metropolis.py:6-101.

Same signature, defaults, return value and progress output as the
reference's ``metropolis_hastings()``; every iteration (Gaussian random-walk
proposal, forward log density, accept/reject, sample store) runs in the
persistent HIP kernel ``k_mh`` (csrc/mh.h), one chain group per chain.

Additions (keyword-only), as for ``hmc()``: ``num_chains`` runs independent
chains in one launch (samples gain a leading chain axis), ``chain_offset``
selects the RNG streams, ``initial_positions`` gives each chain its own start
([num_chains, D] flat), ``return_info`` also returns a ``RunInfo``.  Samples
are arrays ``[num_samples, *shape]`` (the reference's lists of floats, which
``MCMC.run`` converts with ``np.array``, mcmc.py:187); vector-valued
parameters are supported (the reference's ``float()`` store rejects them).
"""
from __future__ import annotations

import time
from typing import Optional

import numpy as np

from .. import _engine, _trace
from ..random import _as_key
from ._driver import RunInfo


def metropolis_hastings(log_prob_fn, initial_params, num_samples=1000, proposal_scale=0.1,
                        random_seed=0, verbose=False, *, num_chains=1, chain_offset=0,
                        initial_positions=None, return_info=False, return_trace=False,
                        keep_on_device=False, progress_every: Optional[int] = None):
    """Metropolis-Hastings MCMC sampler with a Gaussian random-walk proposal
    θ' = θ + ε, ε ~ N(0, proposal_scale² I).

    Returns ``(samples, acceptance_rate)``: ``samples`` maps each parameter
    name to an array ``[num_samples, *shape]`` (``[num_chains, num_samples,
    *shape]`` when ``num_chains > 1``); ``acceptance_rate`` is the fraction of
    accepted proposals (an array over chains when ``num_chains > 1``).
    """
    import torch

    num_samples = int(num_samples)
    if num_samples < 0:
        raise ValueError("num_samples must be non-negative")
    k = _as_key(random_seed)
    # (a large regression's affine terms as expression terms: the sliced MH
    # kernel instead of the tape, _trace.mh_program)
    program = _trace.mh_program(_trace.compile_model(log_prob_fn, initial_params))
    layout = program.layout
    C = int(num_chains)
    if C < 1:
        raise ValueError("num_chains must be >= 1")
    if initial_positions is None:
        q0 = layout.flatten(initial_params)
    else:
        q0 = np.asarray(initial_positions, np.float32).reshape(C, layout.size)
    chains = _engine.ChainSet(program, C, q0, proposal_scale)
    samples = torch.empty((C, max(num_samples, 1), layout.size), dtype=torch.float32,
                          device=chains.device)
    trace = (_engine.make_trace(C, 0, max(num_samples, 1), chains.device)
             if return_trace else None)
    cfg = dict(chain_offset=chain_offset, num_warmup=0, num_samples=num_samples,
               sample_begin=0, sample_capacity=num_samples, seed=k.seed)
    out = print if verbose else (lambda *a: None)
    every = progress_every or 500
    out(f"Running {num_samples} Metropolis-Hastings iterations...")
    t0 = time.perf_counter()
    it = 0
    while it < num_samples:
        nxt = min(num_samples, it + every) if verbose else num_samples
        chains.run_mh(proposal_scale=proposal_scale, samples=samples, trace=trace,
                      iter_begin=it, iter_count=nxt - it, **cfg)
        it = nxt
        if verbose and it % every == 0:  # metropolis.py:95-97
            s = chains.scalars()
            rate = float(np.mean(s["n_accept"])) / it
            out(f"  Iteration {it}/{num_samples} (accept rate: {rate:.2%})")
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    s = chains.scalars()
    if num_samples == 0:
        raise ZeroDivisionError("division by zero")  # metropolis.py:99
    accept = s["n_accept"] / num_samples
    flat = samples[:, :num_samples, :]
    info = RunInfo(
        algorithm="metropolis", num_chains=C, num_warmup=0, num_samples=num_samples,
        step_size=np.full(C, float(proposal_scale)), warmup_accept_rate=np.full(C, np.nan),
        accept_rate=accept, n_grad=np.zeros(C, np.int64), warmup_seconds=0.0,
        sampling_seconds=t1 - t0, trace=trace.numpy() if trace is not None else None,
        device_samples=flat if keep_on_device else None, layout=layout)
    info.extra["logp"] = s["logp"].copy()
    per_name = layout.unflatten(flat.cpu().numpy())  # name -> [C, S, *shape]
    if C == 1:
        per_name = {n: v[0] for n, v in per_name.items()}
        rate = float(accept[0])
    else:
        rate = accept
    if return_info:
        return per_name, rate, info
    return per_name, rate
