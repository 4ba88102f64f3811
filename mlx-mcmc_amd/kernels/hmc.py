"""Hamiltonian Monte Carlo on MI355X — drop-in for mlx_mcmc/kernels/hmc.py:7-206.

Same signature, defaults, return value and progress output as the
reference's ``hmc()``; the whole iteration loop (momentum draw, L leapfrog
steps with the fused gradient tape, Metropolis accept, step-size adaptation,
sample store) runs in one persistent HIP kernel chosen by the program's plan:
``k_hmc_lf`` (csrc/lanes_fast.h: lane-resident, fast-form programs such as the
hierarchical and isotropic Gaussians), ``k_hmc_lr`` (csrc/lanes.h: other
lane-resident programs), ``k_hmc_sl`` (csrc/sliced.h: the term interpreter
over data slices) or ``k_hmc`` (csrc/hmc.h: the chain-per-workgroup tape,
every other program).

Additions (keyword-only): ``num_chains`` runs independent chains in one
launch (samples gain a leading chain axis), ``chain_offset`` selects the RNG
streams (for sharding chains over GPUs), ``return_info`` also returns a
``RunInfo`` with per-chain step sizes, timings and an optional trace.
``num_slices`` picks the work split of large models (0 automatic, 1 one
chain per workgroup, >= 2 data slices per chain: csrc/sliced.h), and
``slice_kernel`` the kernel of a sliced program ("auto": the lane-resident
csrc/lanes.h when the layout qualifies, "interpreter": csrc/sliced.h,
"lanes"; with ``num_slices=1`` "lanes" runs the unsliced program on the
lane-resident kernel with one slice).
Vector-valued parameters are supported (the reference's ``float()`` store,
hmc.py:192, rejects them — SURVEY Q6).
"""
from __future__ import annotations

from ._driver import run_sampler


def hmc(log_prob_fn, initial_params, num_samples=1000, num_warmup=1000, step_size=0.1,
        num_leapfrog_steps=10, adapt_step_size=True, target_accept=0.8, key=None, *,
        num_chains=1, chain_offset=0, progress=True, return_info=False, return_trace=False,
        keep_on_device=False, initial_positions=None, num_slices=0, slice_kernel="auto"):
    """Hamiltonian Monte Carlo sampler using gradient information.

    Returns ``(samples, acceptance_rate)`` like the reference: ``samples`` maps
    each parameter name to an array of shape ``[num_samples, *shape]`` (or
    ``[num_chains, num_samples, *shape]``), ``acceptance_rate`` is the
    sampling-phase acceptance rate (an array over chains when
    ``num_chains > 1``).
    """
    samples, rate, info = run_sampler(
        "hmc", log_prob_fn, initial_params, num_samples=num_samples, num_warmup=num_warmup,
        step_size=step_size, target_accept=target_accept, adapt_step_size=adapt_step_size,
        key=key, num_leapfrog_steps=num_leapfrog_steps, num_chains=num_chains,
        chain_offset=chain_offset, progress=progress, return_trace=return_trace,
        keep_on_device=keep_on_device, initial_positions=initial_positions,
        num_slices=num_slices, slice_kernel=slice_kernel)
    if return_info:
        return samples, rate, info
    return samples, rate
