"""HMC at the bench's own shape against the oracle (BASELINE configs[2]:
hierarchical Normal, D = 1000, N = 100 K, L = 20; reference hmc.py:113-170).

tests/golden/hmc_large_trace.npz (scripts/gen_golden_large.py) holds the
oracle's trace for global chains 0, 1, 77, 255 of seed 0 at eps0 = 3e-3,
W = 15 (the reference's step-size rule acting at i = 11..14), S = 15: a regime
where chains move and decisions are a mix.  The GPU runs all 256 chains of
the bench's launch through the product API on each kernel — the sliced
lane-resident kernel (the bench kernel, 16 slices), the sliced term
interpreter, and the unsliced k_hmc — and for the fixture's chains:

  * accept decisions identical to the oracle's until the first divergence,
    and a divergence is allowed only at a proven near-tie: the oracle's
    f32 log U lies within TIE of the oracle's log ratio, where TIE bounds the
    two fp32 energy differences' disagreement (below);
  * log ratios -(H_prop - H_init) and H_init within TIE of the oracle's at
    every compared iteration (should an oracle trajectory diverge, the GPU's
    must too: ratio NaN or below -1e3); step sizes bit-identical (f64,
    hmc.py:163-167);
  * stored draws within rtol 1e-4 (atol 1e-5) of the oracle's;
  * the compared prefix holds both accepted and rejected proposals.

TIE: H is a float32 sum of ~100 K terms of magnitude ~1.4e5 (ulp 2^-6); the
GPU sums per slice / per lane, the oracle (torch) in its own order, so each
H may differ by a few ulp of |H|.  TIE = 8 ulp(|H_init|) (tests/_near_tie.py) (0.125 at this
shape) bounds |ratio_gpu - ratio_ref| (asserted, so the bound is checked,
not assumed; measured on MI355X: at most 3 ulp, and chain 77 diverges at
iteration 16 where |log U - ratio| = 0.0093, below one ulp).
"""
import json
import os

import numpy as np
import pytest

import workloads as W
from _near_tie import compare_trace

pytestmark = pytest.mark.gpu

FIXTURE = os.path.join(os.path.dirname(__file__), "golden", "hmc_large_trace.npz")


def _fixture():
    fx = np.load(FIXTURE, allow_pickle=False)
    out = {k: fx[k] for k in fx.files}
    out["config"] = json.loads(str(out["config"]))
    return out


@pytest.mark.parametrize("kernel", ["lanes", "lanes_runtime_form", "interpreter", "unsliced"])
def test_large_hmc_trace_matches_oracle(gpu, kernel):
    """lanes: k_hmc_lf with the compile-time hierarchical form (the bench
    kernel); lanes_runtime_form: the same kernel reading the form at run time
    (mc_debug_lanes_forms(0))."""
    import mlx_mcmc_amd as m
    from mlx_mcmc_amd import _lib

    if kernel == "lanes_runtime_form":
        _lib.load().mc_debug_lanes_forms(0)
        try:
            return _large_trace(m, "lanes")
        finally:
            _lib.load().mc_debug_lanes_forms(1)
    _large_trace(m, kernel)


def _large_trace(m, kernel):
    fx = _fixture()
    cfg = fx["config"]
    lp, init = W.hierarchical(W.ns_product(), *W.SHAPES["large"])
    slices, sk = (1, "auto") if kernel == "unsliced" else (0, kernel)
    s, rate, info = m.hmc(lp, init, num_samples=cfg["num_samples"],
                          num_warmup=cfg["num_warmup"], step_size=cfg["step_size"],
                          num_leapfrog_steps=cfg["num_leapfrog_steps"],
                          adapt_step_size=cfg["adapt_step_size"],
                          target_accept=cfg["target_accept"], key=m.random.key(cfg["seed"]),
                          num_chains=256, progress=False, return_info=True, return_trace=True,
                          keep_on_device=True, num_slices=slices, slice_kernel=sk)
    tr = info.trace
    draws = info.device_samples.cpu().numpy()            # [C, S, D], layout order
    Wm = cfg["num_warmup"]
    seen_acc = seen_rej = 0
    for j, c in enumerate(fx["chains"]):
        ref = {k: fx[k][j] for k in ("accepted", "ratio", "log_u", "step_size", "energy")}
        gpu_c = {"accepted": tr["accepted"][c], "ratio": tr["accept_stat"][c],
                 "step_size": tr["step_size"][c], "energy": tr["energy"][c]}
        same = compare_trace(gpu_c, ref, f"{kernel} chain {c}", verbose=True)
        seen_acc += int(np.sum(ref["accepted"][:same]))
        seen_rej += int(same - np.sum(ref["accepted"][:same]))
        ns = max(0, same - Wm)                 # stored draws before any divergence
        np.testing.assert_allclose(draws[c, :ns], fx["samples"][j, :ns], rtol=1e-4, atol=1e-5,
                                   err_msg=f"{kernel} chain {c}")
    assert seen_acc > 0 and seen_rej > 0, "the compared iterations must mix accepts and rejects"
    # the whole launch moved: no chain froze at this step size
    assert np.all(info.accept_rate > 0)

