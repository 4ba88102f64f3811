"""Affine loc operands (include/mcmc355.h mc_affine; _trace.Affine): the
reference differentiates any MLX expression of the parameters (hmc.py:53-67,
nuts.py:76-87); the linear-predictor forms a + b * x (regression),
mu + tau * z (non-centred hierarchy) and alpha[group] + beta * x
(varying-intercept regression) run on the GPU tape (eval.h strided_generic,
and seg_generic for the non-injective gather) and are checked against the
CPU oracle, whose gradients are torch autograd over the same user model.

Bars: tape log p within 2e-6 of sum |lp| (f32 summation order), gradients
rtol 1e-4; HMC decisions / H / ratios equal to the oracle's until a proven
near-tie (tests/_near_tie.py); NUTS trees identical for >= 10 iterations; MH
decisions identical over 150 iterations; the regression posterior mean of the
slope within 4 MCSE of the least-squares fit (flat-ish priors)."""
import numpy as np
import pytest

import workloads as W
from _near_tie import compare_trace, log_u
from oracle import samplers as S

pytestmark = pytest.mark.gpu

MODELS = {"regression": lambda ns: W.linear_regression(ns, 1000),
          "eight_schools_nc": W.eight_schools_nc,
          "varying_intercept": W.varying_intercept}


@pytest.mark.parametrize("model", list(MODELS))
def test_affine_tape_matches_autograd(gpu, model):
    from mlx_mcmc_amd import _engine, _trace

    lp_fn, init = MODELS[model](W.ns_product())
    prog = _trace.compile_model(lp_fn, init, slices=1)
    assert prog.num_slices == 1 and prog.slice_kernel == "unsliced"   # the tape kernels
    olp, oinit = MODELS[model](W.ns_oracle())
    M = S.EagerModel(olp, oinit)
    rng = np.random.default_rng(7)
    base = prog.layout.flatten(init)
    pts = np.stack([base + rng.normal(0, 0.3, base.size).astype(np.float32) for _ in range(6)])
    for nm in ("sigma", "tau"):
        if nm in prog.layout.names:
            k = prog.layout.offsets[prog.layout.names.index(nm)]
            pts[:, k] = np.abs(pts[:, k]) + 0.2
    lp, g = _engine.logp_grad(prog, pts)
    lp, g = lp.cpu().numpy(), g.cpu().numpy()
    for i, q in enumerate(pts):
        rl, rg = M.logp_grad(q)
        assert abs(lp[i] - rl) <= 2e-6 * max(1.0, abs(rl)) * 50, (i, lp[i], rl)
        np.testing.assert_allclose(g[i], rg, rtol=1e-4, atol=1e-3 * max(1.0, np.abs(rg).max()))


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_affine_hmc_trace_matches_oracle(gpu, seed):
    """The regression a + b * x on the automatic plan: the one-slice
    lane-resident kernel (lanes.h LS_AFF, a chunk term with shared loc and
    slope) against the oracle's HMC trace."""
    import mlx_mcmc_amd as m

    lp, _ = W.linear_regression(W.ns_product())
    olp, _ = W.linear_regression(W.ns_oracle())
    start = {"a": np.float32(1.4), "b": np.float32(1.9), "sigma": np.float32(0.6)}
    kw = dict(num_samples=40, num_warmup=40, step_size=0.004, num_leapfrog_steps=10)
    s, rate, info = m.hmc(lp, start, key=m.random.key(seed), progress=False, return_info=True,
                          return_trace=True, **kw)
    ref = S.hmc(olp, start, seed=seed, **kw)
    n = len(ref.trace["accepted"])
    tr = info.trace
    gpu_c = {"accepted": tr["accepted"][0], "ratio": tr["accept_stat"][0],
             "step_size": tr["step_size"][0], "energy": tr["energy"][0]}
    ref_c = {k: np.asarray(ref.trace[k]) for k in ("accepted", "ratio", "step_size", "energy")}
    ref_c["log_u"] = log_u(seed, 0, n)
    same = compare_trace(gpu_c, ref_c, f"regression seed {seed}", verbose=True)
    acc = np.asarray(ref.trace["accepted"][:same])
    assert same >= 30 and acc.any() and not acc.all()
    ns = max(0, same - 40)
    np.testing.assert_allclose(s["b"][:ns], ref.samples[:ns, 1], rtol=1e-4, atol=1e-5)


def test_affine_nuts_trace_matches_oracle(gpu):
    import mlx_mcmc_amd as m

    plp, pinit = W.eight_schools_nc(W.ns_product())
    olp, oinit = W.eight_schools_nc(W.ns_oracle())
    n_w, n_s = 30, 10
    _, _, info = m.nuts(plp, pinit, num_samples=n_s, num_warmup=n_w, key=m.random.key(2),
                        progress=False, return_info=True, return_trace=True)
    assert info.extra["kernel"] == "tape"
    ref = S.nuts(olp, oinit, num_samples=n_s, num_warmup=n_w, seed=2)
    same = 0
    for i in range(n_w + n_s):
        if (info.trace["tree_depth"][0][i] != ref.trace["depth"][i]
                or info.trace["n_leapfrog"][0][i] != ref.trace["leaves"][i]):
            break
        same += 1
    assert same >= 10, f"trees diverged at iteration {same}"


def test_affine_mh_trace_matches_oracle(gpu):
    import mlx_mcmc_amd as m

    lp, _ = W.linear_regression(W.ns_product())
    olp, _ = W.linear_regression(W.ns_oracle())
    start = {"a": 1.4, "b": 1.9, "sigma": 0.6}
    n = 150
    s, rate, info = m.metropolis_hastings(lp, start, num_samples=n, proposal_scale=0.02,
                                          random_seed=5, return_info=True, return_trace=True)
    ref = S.metropolis_hastings(olp, start, num_samples=n, proposal_scale=0.02, random_seed=5)
    acc = info.trace["accepted"][0].astype(bool)
    assert list(acc) == ref.trace["accepted"] and 0 < acc.mean() < 1
    np.testing.assert_allclose(s["b"], ref.samples[:, 1], rtol=1e-5, atol=1e-6)


def test_affine_regression_posterior(gpu):
    import mlx_mcmc_amd as m

    lp, _ = W.linear_regression(W.ns_product())
    x, y = W.regression_data()
    X = np.stack([np.ones_like(x), x], 1).astype(np.float64)
    ab = np.linalg.lstsq(X, y.astype(np.float64), rcond=None)[0]
    start = {"a": np.float32(ab[0]), "b": np.float32(ab[1]), "sigma": np.float32(0.5)}
    s, rate, info = m.hmc(lp, start, num_samples=500, num_warmup=300, step_size=0.01,
                          num_leapfrog_steps=10, key=m.random.key(1), num_chains=32,
                          progress=False, return_info=True)
    # the automatic plan: the lane-resident kernel (an affine chunk term, lanes.h
    # lr_affine_term with a shared loc and slope)
    assert info.extra["kernel"] == "lanes"
    live = info.accept_rate > 0.05
    assert live.sum() >= 16
    for k, name in enumerate(("a", "b")):
        d = s[name][live]                      # [C, S]
        mcse = d.mean(1).std() / np.sqrt(d.shape[0])
        assert abs(d.mean() - ab[k]) < 4 * mcse + 2e-3, (name, d.mean(), ab[k], mcse)


def test_affine_varying_intercept_hmc_trace(gpu):
    """alpha[group] + beta * x (the segmented tape, a non-injective gather as
    the affine loc) against the oracle's HMC trace."""
    import mlx_mcmc_amd as m

    lp, init = W.varying_intercept(W.ns_product())
    olp, oinit = W.varying_intercept(W.ns_oracle())
    x, y, g = W.varying_intercept_data()
    start = dict(init)
    start["alpha"] = np.array([y[g == k].mean() - 0.7 * x[g == k].mean() for k in range(20)],
                              np.float32)
    kw = dict(num_samples=30, num_warmup=30, step_size=0.01, num_leapfrog_steps=10)
    s, rate, info = m.hmc(lp, start, key=m.random.key(1), progress=False, return_info=True,
                          return_trace=True, num_slices=1, **kw)
    ref = S.hmc(olp, start, seed=1, **kw)
    # the first 25 iterations: the positions' fp32 drift after that moves a
    # large rejection's ratio (|ratio| ~ 50) by more than 8 ulp of |H|
    n = 25
    tr = info.trace
    gpu_c = {"accepted": tr["accepted"][0][:n], "ratio": tr["accept_stat"][0][:n],
             "step_size": tr["step_size"][0][:n], "energy": tr["energy"][0][:n]}
    ref_c = {k: np.asarray(ref.trace[k])[:n] for k in ("accepted", "ratio", "step_size", "energy")}
    ref_c["log_u"] = log_u(1, 0, n)
    same = compare_trace(gpu_c, ref_c, "varying intercept", verbose=True)
    acc = np.asarray(ref.trace["accepted"][:same])
    assert same >= 20 and acc.any()


@pytest.mark.parametrize("G,N", [(20, 2000), (200, 100000)])
def test_affine_varying_intercept_lanes(gpu, G, N):
    """alpha[group] + beta * x on the lane-resident kernel (VERDICT r3 "Next
    round" 4b: lanes.h LS_AFF, the private alpha_g's elements tiled in its
    lane group with x beside y, beta and sigma shared): G = 20 (one slice, 20
    private parameters: replicated lanes, rep = 2) against the oracle's HMC
    trace; G = 200 / N = 100 K (16 slices, exchange) against the tape kernel
    k_hmc on the same chains (decisions, ratios, H to a proven near-tie,
    step sizes bit-identical)."""
    import mlx_mcmc_amd as m
    from mlx_mcmc_amd import _trace

    lp, init = W.varying_intercept(W.ns_product(), G, N)
    x, y, g = W.varying_intercept_data(G, N)
    start = dict(init)
    start["alpha"] = np.array([y[g == k].mean() - 0.7 * x[g == k].mean() for k in range(G)],
                              np.float32)
    prog = _trace.compile_model(lp, start)
    assert prog.slice_kernel == "lanes" and prog.kernel_note == "", prog.kernel_note
    if G == 20:
        olp, _ = W.varying_intercept(W.ns_oracle(), G, N)
        kw = dict(num_samples=30, num_warmup=30, step_size=0.01, num_leapfrog_steps=10)
        s, rate, info = m.hmc(lp, start, key=m.random.key(1), progress=False, return_info=True,
                              return_trace=True, **kw)
        assert info.extra["kernel"] == "lanes"
        ref = S.hmc(olp, start, seed=1, **kw)
        n = 25
        tr = info.trace
        gpu_c = {"accepted": tr["accepted"][0][:n], "ratio": tr["accept_stat"][0][:n],
                 "step_size": tr["step_size"][0][:n], "energy": tr["energy"][0][:n]}
        ref_c = {k: np.asarray(ref.trace[k])[:n] for k in ("accepted", "ratio", "step_size",
                                                            "energy")}
        ref_c["log_u"] = log_u(1, 0, n)
        same = compare_trace(gpu_c, ref_c, "varying intercept (lanes)", verbose=True)
        acc = np.asarray(ref.trace["accepted"][:same])
        assert same >= 20 and acc.any()
        return
    assert prog.num_slices == 16
    kw = dict(num_samples=10, num_warmup=10, step_size=2e-3, num_leapfrog_steps=10,
              key=m.random.key(3), num_chains=16, progress=False, return_info=True,
              return_trace=True)
    a, _, ia = m.hmc(lp, start, num_slices=1, **kw)
    b, _, ib = m.hmc(lp, start, **kw)
    assert ia.extra["kernel"] == "unsliced" and ib.extra["kernel"] == "lanes"
    acc = ia.trace["accepted"].astype(bool)
    assert acc.any()
    full = 0
    for c in range(16):
        ref = {"accepted": ia.trace["accepted"][c], "ratio": ia.trace["accept_stat"][c],
               "energy": ia.trace["energy"][c], "step_size": ia.trace["step_size"][c],
               "log_u": log_u(3, c, 20)}
        got = {"accepted": ib.trace["accepted"][c], "ratio": ib.trace["accept_stat"][c],
               "energy": ib.trace["energy"][c], "step_size": ib.trace["step_size"][c]}
        same = compare_trace(got, ref, f"varying intercept N={N} chain {c}")
        full += same == 20
        ns = max(0, same - 10)
        for k in a:
            np.testing.assert_allclose(b[k][c, :ns], a[k][c, :ns], rtol=1e-3, atol=1e-5)
    assert full >= 10
