"""BASELINE configs[1]'s own kernel against the oracle (VERDICT r2 "Next
round" 3; reference hmc.py:113-170): the isotropic 100-dim Normal runs on
the fast-form lane-resident kernel with the compile-time isotropic form,
k_hmc_lf<..., FORM = LF_DIR>, one slice, one wave per chain pair.

tests/golden/hmc_iso_trace.npz (scripts/gen_golden_iso.py) holds the
oracle's trace for chains 0, 1, 33, 63 of the config's 64-chain launch at
eps0 = 0.9 with the reference's warmup rule acting, where the decisions are
a mix.  As in test_gpu_large_parity.py: decisions identical until a proven
near-tie (tests/_near_tie.py), ratios and H_init within the tie bound, step
sizes bit-identical, stored draws within rtol 1e-4 — on the compile-time
form and on the same kernel reading its form at run time.
"""
import json
import os

import numpy as np
import pytest

import workloads as W
from _near_tie import compare_trace

pytestmark = pytest.mark.gpu

FIXTURE = os.path.join(os.path.dirname(__file__), "golden", "hmc_iso_trace.npz")


@pytest.mark.parametrize("form", ["compile_time", "run_time"])
def test_iso_hmc_trace_matches_oracle(gpu, form):
    import mlx_mcmc_amd as m
    from mlx_mcmc_amd import _lib, _trace

    fx = np.load(FIXTURE, allow_pickle=False)
    cfg = json.loads(str(fx["config"]))
    lp, init = W.iso_normal(W.ns_product())
    prog = _trace.compile_model(lp, init)
    assert prog.slice_kernel == "lanes" and prog.lanes_fast, "config 2 must run k_hmc_lf"
    lib = _lib.load()
    if form == "run_time":
        lib.mc_debug_lanes_forms(0)
    try:
        s, rate, info = m.hmc(lp, init, num_samples=cfg["num_samples"],
                              num_warmup=cfg["num_warmup"], step_size=cfg["step_size"],
                              num_leapfrog_steps=cfg["num_leapfrog_steps"],
                              adapt_step_size=cfg["adapt_step_size"],
                              target_accept=cfg["target_accept"], key=m.random.key(cfg["seed"]),
                              num_chains=64, progress=False, return_info=True,
                              return_trace=True, keep_on_device=True)
    finally:
        lib.mc_debug_lanes_forms(1)
    tr = info.trace
    draws = info.device_samples.cpu().numpy()
    Wm = cfg["num_warmup"]
    seen_acc = seen_rej = 0
    for j, c in enumerate(fx["chains"]):
        ref = {k: fx[k][j] for k in ("accepted", "ratio", "log_u", "step_size", "energy")}
        gpu_c = {"accepted": tr["accepted"][c], "ratio": tr["accept_stat"][c],
                 "step_size": tr["step_size"][c], "energy": tr["energy"][c]}
        same = compare_trace(gpu_c, ref, f"iso {form} chain {c}", verbose=True)
        seen_acc += int(np.sum(ref["accepted"][:same]))
        seen_rej += int(same - np.sum(ref["accepted"][:same]))
        ns = max(0, same - Wm)
        np.testing.assert_allclose(draws[c, :ns], fx["samples"][j, :ns], rtol=1e-4, atol=1e-5,
                                   err_msg=f"iso {form} chain {c}")
    assert seen_acc > 0 and seen_rej > 0, "the compared iterations must mix accepts and rejects"
