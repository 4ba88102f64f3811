"""Shared host driver behind ``hmc()`` and ``nuts()``.

The iteration loop of the reference (mlx_mcmc/kernels/hmc.py:155-198,
nuts.py:287-356) runs inside the HIP kernels; the host only launches
chunks of iterations (at the reference's progress-print boundaries), prints
the same progress lines, and converts the device samples to the reference's
return types.
"""
from __future__ import annotations

import time
import warnings
from dataclasses import dataclass, field
from typing import Dict, Optional

import numpy as np

from .. import _engine, _lib, _trace
from ..random import _as_key


@dataclass
class RunInfo:
    """Everything a run measured, beyond the reference's (samples, rate)."""
    algorithm: str
    num_chains: int
    num_warmup: int
    num_samples: int
    step_size: np.ndarray            # final epsilon per chain
    warmup_accept_rate: np.ndarray   # per chain
    accept_rate: np.ndarray          # per chain (sampling phase)
    n_grad: np.ndarray               # gradient evaluations per chain
    warmup_seconds: float
    sampling_seconds: float
    mean_tree_depth: Optional[np.ndarray] = None
    n_divergent: Optional[np.ndarray] = None
    trace: Optional[dict] = None
    device_samples: object = None    # torch tensor [C, S, D] when kept on device
    layout: object = None
    extra: Dict = field(default_factory=dict)


# csrc/api.hip kLrAutoMinElements: the automatic plan slices programs of at
# least this many elements (and the lane-resident kernel is what pays for it)
_LANES_WARN_ELEMENTS = 2048


def _chunks(begin: int, end: int, every: int):
    """Split [begin, end) at multiples of `every` counted from `begin`."""
    it = begin
    while it < end:
        nxt = min(end, it + every) if every > 0 else end
        yield it, nxt
        it = nxt


def run_sampler(algorithm: str, log_prob_fn, initial_params, *, num_samples: int,
                num_warmup: int, step_size: float, target_accept: float,
                adapt_step_size: bool, key, num_leapfrog_steps: int = 10,
                max_tree_depth: int = 10, num_chains: int = 1, chain_offset: int = 0,
                slice_mode: str = "reference", progress: bool = True,
                progress_every: Optional[int] = None, return_trace: bool = False,
                keep_on_device: bool = False, initial_positions=None, num_slices: int = 0,
                slice_kernel: str = "auto"):
    import torch

    if algorithm not in ("hmc", "nuts"):
        raise ValueError(algorithm)
    if num_samples < 0 or num_warmup < 0:
        raise ValueError("num_samples and num_warmup must be non-negative")
    k = _as_key(key)
    program = _trace.compile_model(log_prob_fn, initial_params, slices=num_slices,
                                   slice_kernel=slice_kernel)
    if algorithm == "nuts" and num_slices == 0 and slice_kernel == "auto":
        # a large regression's affine terms as expression terms: the sliced
        # NUTS kernel instead of the tape (_trace.nuts_program)
        program = _trace.nuts_program(program, max_tree_depth)
    layout = program.layout
    note = program.kernel_note
    # no warning where the user cannot act on it: no lane-resident kernel
    # exists for affine locs or expression terms, so that note is
    # structural
    if (algorithm == "hmc" and note and num_slices == 0 and slice_kernel == "auto"
            and program.program_elements >= _LANES_WARN_ELEMENTS
            and program.model.n_affines == 0 and program.model.n_exprs == 0):
        # a layout the lane-resident kernel declines runs
        # on a 2-4x slower kernel; say so instead of degrading silently
        warnings.warn(f"{note}; running on the {program.slice_kernel} kernel", RuntimeWarning,
                      stacklevel=3)
    C = int(num_chains)
    if C < 1:
        raise ValueError("num_chains must be >= 1")
    if initial_positions is None:
        q0 = layout.flatten(initial_params)
    else:
        q0 = np.asarray(initial_positions, np.float32).reshape(C, layout.size)
    chains = _engine.ChainSet(program, C, q0, step_size)
    total = num_warmup + num_samples
    samples = torch.empty((C, max(num_samples, 1), layout.size), dtype=torch.float32,
                          device=chains.device)
    trace = (_engine.make_trace(C, 0, max(total, 1), chains.device) if return_trace else None)
    cfg = dict(chain_offset=chain_offset, num_warmup=num_warmup, num_samples=num_samples,
               sample_begin=0, sample_capacity=num_samples, seed=k.seed, step_size=step_size,
               target_accept=target_accept, adapt_step_size=adapt_step_size)
    if algorithm == "hmc":
        cfg["num_leapfrog_steps"] = num_leapfrog_steps
        launch = chains.run_hmc
        every = progress_every or 500
    else:
        cfg["max_tree_depth"] = max_tree_depth
        cfg["slice_mode"] = {"reference": 0, "exact": 1}[slice_mode]
        launch = chains.run_nuts
        every = progress_every or 250
    out = (lambda *a: print(*a)) if progress else (lambda *a: None)

    stats = chains.scalars

    # ---- warmup --------------------------------------------------------------
    if algorithm == "hmc":
        out(f"Warmup phase: {num_warmup} samples")
    else:
        out(f"NUTS warmup: {num_warmup} samples")
    t0 = time.perf_counter()
    for a, b in _chunks(0, num_warmup, every if progress else 0):
        launch(samples=samples, trace=trace, iter_begin=a, iter_count=b - a, **cfg)
        if progress and b % every == 0:
            s = stats()
            rate = float(np.mean(s["n_accept"] / np.maximum(s["n_total"], 1)))
            eps = float(np.mean(s["step_size"]))
            if algorithm == "hmc":
                out(f"  Iteration {b}/{num_warmup} (accept rate: {100 * rate:.2f}%, "
                    f"step_size: {eps:.4f})")
            else:
                depth = float(np.mean(s["depth_sum"])) / b
                out(f"  Iteration {b}/{num_warmup} (accept: {100 * rate:.1f}%, "
                    f"avg_depth: {depth:.1f}, step_size: {eps:.4f})")
    torch.cuda.synchronize()
    chains.check_status()
    t1 = time.perf_counter()
    s = stats()
    if num_warmup == 0:
        # the reference divides by the warmup count right here (hmc.py:175,
        # nuts.py:328-329): num_warmup=0 raises
        raise ZeroDivisionError("division by zero")

    # ---- sampling ------------------------------------------------------------
    if algorithm == "nuts" and adapt_step_size:
        out(f"Warmup complete. Using step_size: {float(np.mean(s['step_size_bar'])):.4f}")
    if algorithm == "hmc":
        wr = float(np.mean(s["n_accept"] / np.maximum(s["n_total"], 1)))
        out(f"Warmup acceptance rate: {100 * wr:.2f}% "
            f"(final step_size: {float(np.mean(s['step_size'])):.4f})")
        out(f"\nSampling phase: {num_samples} samples")
    else:
        wr = float(np.mean(s["n_accept"] / np.maximum(s["n_total"], 1)))
        wd = float(np.mean(s["depth_sum"])) / max(num_warmup, 1)
        out(f"Warmup statistics: accept_rate: {100 * wr:.2f}%, avg_tree_depth: {wd:.2f}")
        out(f"\nNUTS sampling: {num_samples} samples")
    for a, b in _chunks(num_warmup, total, every if progress else 0):
        launch(samples=samples, trace=trace, iter_begin=a, iter_count=b - a, **cfg)
        if progress and (b - num_warmup) % 500 == 0:
            s2 = stats()
            if algorithm == "hmc":
                rate = float(np.mean(s2["n_accept"] / np.maximum(s2["n_total"], 1)))
                out(f"  Iteration {b - num_warmup}/{num_samples} "
                    f"(accept rate: {100 * rate:.2f}%)")
            else:
                depth = float(np.mean(s2["depth_sum"])) / (b - num_warmup)
                out(f"  Iteration {b - num_warmup}/{num_samples} (avg_depth: {depth:.2f})")
    torch.cuda.synchronize()
    chains.check_status()
    t2 = time.perf_counter()
    s = stats()
    n_tot = s["n_total"].astype(np.int64)
    if num_samples == 0:
        raise ZeroDivisionError("division by zero")  # hmc.py:197 / nuts.py:341
    accept = s["n_accept"] / n_tot
    warm_accept = s["warmup_accept"] / np.maximum(s["warmup_total"], 1)
    if algorithm == "hmc":
        out(f"Sampling acceptance rate: {100 * float(np.mean(accept)):.2f}%")
    else:
        out("\nSampling complete!")
        out(f"Final statistics: accept_rate: {100 * float(np.mean(accept)):.2f}%, "
            f"avg_tree_depth: {float(np.mean(s['depth_sum'])) / num_samples:.2f}")

    flat = samples[:, :num_samples, :]
    info = RunInfo(
        algorithm=algorithm, num_chains=C, num_warmup=num_warmup, num_samples=num_samples,
        step_size=s["step_size"].copy(), warmup_accept_rate=warm_accept,
        accept_rate=accept, n_grad=s["n_grad"].copy(), warmup_seconds=t1 - t0,
        sampling_seconds=t2 - t1,
        mean_tree_depth=(s["depth_sum"] / num_samples if algorithm == "nuts" else None),
        n_divergent=(s["n_divergent"].copy() if algorithm == "nuts" else None),
        trace=trace.numpy() if trace is not None else None,
        device_samples=flat if keep_on_device else None, layout=layout)
    info.extra["kernel"] = (program.nuts_kernel(max_tree_depth) if algorithm == "nuts"
                            else program.slice_kernel)
    if note and algorithm == "hmc":
        info.extra["kernel_note"] = note
    host = flat.cpu().numpy()
    per_name = layout.unflatten(host)  # name -> [C, S, *shape]
    if C == 1:
        per_name = {n: v[0] for n, v in per_name.items()}
        rate = float(accept[0])
    else:
        rate = accept
    return per_name, rate, info
