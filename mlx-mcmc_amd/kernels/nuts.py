"""No-U-Turn Sampler on MI355X — drop-in for mlx_mcmc/kernels/nuts.py:16-358.

Same signature, defaults, return value and progress output as the
reference's ``nuts()`` (slice NUTS, Hoffman & Gelman 2014 Alg. 3, dual
averaging).  Tree building runs iteratively inside a persistent HIP kernel:
``k_nuts_lr`` (csrc/nuts_lanes.h, one chain per wave, lane-resident state)
when the model plans as one lane-resident slice, else ``k_nuts`` (csrc/nuts.h,
one chain per chain group on the gradient tape), or ``k_nuts_sl``
(csrc/nuts_sliced.h) when it plans as several fast-form data slices.

``nuts_kernel``: "auto" runs the lane-resident kernel ``k_nuts_lr``
(csrc/nuts_lanes.h: chain state in registers, tree arena in LDS) when the
model plans as one lane-resident slice, the sliced kernel ``k_nuts_sl``
(csrc/nuts_sliced.h: one wave per chain and data slice, one record exchange
per leaf) when it plans as several fast-form slices (the README "Large"
row), else ``k_nuts``; "tape" keeps ``k_nuts``.  ``num_slices``: data slices
per chain (0: the automatic plan, as ``hmc()``).

``slice_mode="reference"`` (default) reproduces the reference's float32
slice variable: u = f32 exp(log u) rounds to the smallest denormal (log u =
~-103.28, SURVEY Q7's ~-103.3) down to ln 2^-150 ~ -103.97 and to 0 below it,
which switches the slice test off (log u = -inf)
(nuts.py:236-237); ``"exact"`` keeps log u in double precision.
Keyword-only additions as for ``hmc()``.
"""
from __future__ import annotations

from ._driver import run_sampler

DELTA_MAX = 1000.0  # nuts.py:13 (the kernel uses the same constant)


def nuts(log_prob_fn, initial_params, num_samples=1000, num_warmup=1000, step_size=0.1,
         max_tree_depth=10, adapt_step_size=True, target_accept=0.65, key=None, *,
         num_chains=1, chain_offset=0, slice_mode="reference", progress=True,
         return_info=False, return_trace=False, keep_on_device=False,
         initial_positions=None, nuts_kernel="auto", num_slices=0):
    """No-U-Turn Sampler (NUTS) for efficient HMC sampling.

    Returns ``(samples, acceptance_rate)`` like the reference, where the rate
    is the fraction of sampling iterations whose mean acceptance statistic
    exceeds 0.5 (nuts.py:347).
    """
    if nuts_kernel not in ("auto", "tape"):
        raise ValueError(f"nuts_kernel must be 'auto' or 'tape', not {nuts_kernel!r}")
    samples, rate, info = run_sampler(
        "nuts", log_prob_fn, initial_params, num_samples=num_samples, num_warmup=num_warmup,
        step_size=step_size, target_accept=target_accept, adapt_step_size=adapt_step_size,
        key=key, max_tree_depth=max_tree_depth, num_chains=num_chains,
        chain_offset=chain_offset, slice_mode=slice_mode, progress=progress,
        return_trace=return_trace, keep_on_device=keep_on_device,
        initial_positions=initial_positions,
        num_slices=1 if nuts_kernel == "tape" else int(num_slices))
    if return_info:
        return samples, rate, info
    return samples, rate
