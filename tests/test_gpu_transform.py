"""Reparameterised models (include/mcmc355.h mc_transform_kind and
MC_DIST_IDENTITY; _trace.Param.transformed / identity_expr): the reference
differentiates any MLX expression of the parameters (hmc.py:53-67,
nuts.py:76-87); the unconstrained-scale forms `Normal(mu, mx.exp(log_sigma))`
+ `log_sigma`, the non-centred `mu + mx.exp(log_tau) * z` and the
log-transformed positive vector `Normal(m, s).log_prob(mx.log(x)) -
mx.sum(mx.log(x))` run on the GPU tape (eval.h xf_apply / xf_chain) and are
checked against the CPU oracle, whose gradients are torch autograd over the
same user model, and against known answers.  Programs whose transforms act on
broadcast parameters only (the log-scale hierarchical model) also run on the
lane-resident kernels — the fast form k_hmc_lf (lanes_fast.h: the shared
value xf(q) beside q, the identity terms' weights in the holder lane) and the
general k_hmc_lr (lanes.h LrCtx::shxf) — sliced or not, and are checked
against the tape kernel and the oracle there:

  * tape log p within 2e-6 of sum |lp| (f32 summation order), gradients
    rtol 1e-4 (the device's expf / logf are not the CPU's: <= 2 ulp each);
  * HMC decisions / H / ratios equal to the oracle's until a proven near-tie
    (tests/_near_tie.py), NUTS trees identical for >= 10 iterations, MH
    decisions identical over 150 iterations;
  * posterior moments within 1 % (tests/_streaming.py rule): the small
    hierarchical shape's exact (log tau, log sigma, mu, theta) moments
    (oracle/exact.py, tests/golden/posterior_exact.json) and the log-normal
    vector's closed form.
"""
import json
import os

import numpy as np
import pytest

import workloads as W
from _near_tie import compare_trace, log_u
from _streaming import check_within_one_percent, stream_moments
from oracle import samplers as S

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
Z = 4.42

MODELS = {"hier_reparam": lambda ns: W.hierarchical_reparam(ns, *W.SHAPES["small"]),
          "eight_schools_nc_log": W.eight_schools_nc_log,
          "lognormal": W.lognormal}


@pytest.mark.parametrize("model", list(MODELS))
def test_transform_tape_matches_autograd(gpu, model):
    from mlx_mcmc_amd import _engine, _trace

    lp_fn, init = MODELS[model](W.ns_product())
    prog = _trace.compile_model(lp_fn, init)
    olp, oinit = MODELS[model](W.ns_oracle())
    M = S.EagerModel(olp, oinit)
    rng = np.random.default_rng(11)
    base = prog.layout.flatten(init)
    pts = np.stack([base + rng.normal(0, 0.2, base.size).astype(np.float32) for _ in range(6)])
    if model == "lognormal":
        pts = np.abs(pts) + 0.05
    lp, g = _engine.logp_grad(prog, pts)
    lp, g = lp.cpu().numpy(), g.cpu().numpy()
    for i, q in enumerate(pts):
        rl, rg = M.logp_grad(q)
        assert abs(lp[i] - rl) <= 2e-6 * max(1.0, abs(rl)) * 50, (i, lp[i], rl)
        np.testing.assert_allclose(g[i], rg, rtol=1e-4, atol=1e-3 * max(1.0, np.abs(rg).max()))


def test_transform_logp_at_negative_log_argument_is_nan(gpu):
    """mx.log of a negative parameter is NaN in the reference (and the HMC
    proposal that reaches it is rejected, hmc.py:150 NaN comparison)."""
    from mlx_mcmc_amd import _engine, _trace

    lp_fn, init = W.lognormal(W.ns_product())
    prog = _trace.compile_model(lp_fn, init)
    q = prog.layout.flatten(init)[None].copy()
    q[0, 3] = -0.5
    lp, _ = _engine.logp_grad(prog, q)
    assert np.isnan(lp.cpu().numpy()[0])


def test_transform_kernel_selection(gpu):
    """Broadcast-parameter transforms: the lane-resident kernels (the fast form
    included; not the term interpreter, not NUTS lanes); transforms of
    per-element parameters and affine programs: the tape kernels, with the
    reason in the kernel note."""
    from mlx_mcmc_amd import _lib, _trace

    big = _trace.compile_model(*W.hierarchical_reparam(W.ns_product(), *W.SHAPES["large"]))
    assert big.num_slices == 16 and big.slice_kernel == "lanes" and big.lanes_fast
    assert big.kernel_note == ""
    with pytest.raises(_lib.EngineError, match="interpreter"):
        big.set_slice_kernel("interpreter")
    assert big.slice_kernel == "lanes"
    small = _trace.compile_model(*MODELS["hier_reparam"](W.ns_product()))
    assert small.num_slices == 1 and small.slice_kernel == "lanes"
    assert small.nuts_kernel(10) == "tape"
    for name, why in (("eight_schools_nc_log", "affine"), ("lognormal", "transformed")):
        prog = _trace.compile_model(*MODELS[name](W.ns_product()))
        assert prog.slice_kernel == "unsliced" and why in prog.kernel_note, prog.kernel_note


@pytest.mark.parametrize("model,seed,slices", [("hier_reparam", 0, 0), ("hier_reparam", 1, 0),
                                               ("hier_reparam", 0, 1), ("lognormal", 0, 0)])
def test_transform_hmc_trace_matches_oracle(gpu, model, seed, slices):
    """slices = 0: the automatic plan (k_hmc_lr with one slice for the
    log-scale hierarchical model, the tape for the log-normal); 1: the tape."""
    import mlx_mcmc_amd as m

    lp, init = MODELS[model](W.ns_product())
    olp, _ = MODELS[model](W.ns_oracle())
    # fixed step sizes below each model's stability limit (2 x its smallest
    # posterior sd: log sigma 0.022; the log-normal's x_0 0.074, less where
    # x_0 < exp(m_0) curves more), where decisions are mixed
    # and no trajectory diverges; the log-normal's H is a near-zero sum of
    # 40 O(1) terms, so its ties are ulps of their magnitude (h_scale)
    eps, h_scale = {"hier_reparam": (0.025, 0.0), "lognormal": (0.04, 64.0)}[model]
    kw = dict(num_samples=40, num_warmup=40, step_size=eps, num_leapfrog_steps=10,
              adapt_step_size=False)
    s, rate, info = m.hmc(lp, init, key=m.random.key(seed), progress=False, return_info=True,
                          return_trace=True, num_slices=slices, **kw)
    want = "lanes" if (model == "hier_reparam" and slices == 0) else "unsliced"
    assert info.extra["kernel"] == want
    ref = S.hmc(olp, init, seed=seed, **kw)
    n = len(ref.trace["accepted"])
    tr = info.trace
    gpu_c = {"accepted": tr["accepted"][0], "ratio": tr["accept_stat"][0],
             "step_size": tr["step_size"][0], "energy": tr["energy"][0]}
    ref_c = {k: np.asarray(ref.trace[k]) for k in ("accepted", "ratio", "step_size", "energy")}
    ref_c["log_u"] = log_u(seed, 0, n)
    same = compare_trace(gpu_c, ref_c, f"{model} seed {seed}", verbose=True, h_scale=h_scale)
    acc = np.asarray(ref.trace["accepted"][:same])
    assert same >= 30 and acc.any() and not acc.all(), (same, acc.mean())
    k = max(0, same - 40)
    first = np.asarray(s[list(init)[0]]).reshape(kw["num_samples"], -1)  # layout offset 0
    np.testing.assert_allclose(first[:k], ref.samples[:k, :first.shape[1]], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("shape,kernel", [("medium", "fast"), ("large", "fast"),
                                          ("large", "general")])
def test_transform_lanes_match_tape(gpu, shape, kernel):
    """The log-scale hierarchical model sliced onto k_hmc_lf / k_hmc_lr (4 /
    16 slices) against the tape kernel k_hmc on the same chains, with the
    reference's warmup rule acting (mixed decisions): decisions, ratios and
    H_init equal until a proven near-tie (tests/_near_tie.py), step sizes
    bit-identical, draws within rtol 1e-4 before it."""
    import mlx_mcmc_amd as m
    from _near_tie import compare_trace
    from mlx_mcmc_amd import _lib

    lp, init = W.hierarchical_reparam(W.ns_product(), *W.SHAPES[shape])
    kw = dict(num_samples=15, num_warmup=15, step_size=3e-3, num_leapfrog_steps=20,
              key=m.random.key(3), num_chains=16, progress=False, return_info=True,
              return_trace=True)
    a, _, ia = m.hmc(lp, init, num_slices=1, **kw)
    if kernel == "general":
        _lib.load().mc_debug_lanes_fast(0)
    try:
        b, _, ib = m.hmc(lp, init, **kw)
    finally:
        _lib.load().mc_debug_lanes_fast(1)
    assert ia.extra["kernel"] == "unsliced" and ib.extra["kernel"] == "lanes"
    acc = ia.trace["accepted"].astype(bool)
    assert 0 < acc.mean() < 1, "the regime must mix accepts and rejects"
    full = 0
    for c in range(16):
        ref = {"accepted": ia.trace["accepted"][c], "ratio": ia.trace["accept_stat"][c],
               "energy": ia.trace["energy"][c], "step_size": ia.trace["step_size"][c],
               "log_u": log_u(3, c, 30)}
        got = {"accepted": ib.trace["accepted"][c], "ratio": ib.trace["accept_stat"][c],
               "energy": ib.trace["energy"][c], "step_size": ib.trace["step_size"][c]}
        same = compare_trace(got, ref, f"{shape} chain {c}")
        full += same == 30
        ns = max(0, same - 15)
        for k in a:
            np.testing.assert_allclose(b[k][c, :ns], a[k][c, :ns], rtol=1e-4, atol=1e-5)
    print(f"{shape}: {full} of 16 chains agree over all 30 iterations")
    assert full >= 10, "most chains agree over the whole run (the rest to a proven near-tie)"


def test_transform_sliced_zero_leapfrog_steps(gpu):
    """num_leapfrog_steps = 0 (accepted by the reference's hmc(): the proposal
    is the current point, H is unchanged, every log U < 0 accepts) on a
    sliced program with transformed shared parameters: the lane kernels need
    L > 0 and the term interpreter declines transforms, so the run takes the
    chain-per-workgroup tape — it must succeed, not fail with UNSUPPORTED
    (ADVICE r3)."""
    import mlx_mcmc_amd as m
    from mlx_mcmc_amd import _trace

    lp, init = W.hierarchical_reparam(W.ns_product(), *W.SHAPES["large"])
    prog = _trace.compile_model(lp, init)
    assert prog.num_slices == 16 and prog.slice_kernel == "lanes"
    s, rate, info = m.hmc(lp, init, num_samples=4, num_warmup=2, step_size=1e-3,
                          num_leapfrog_steps=0, key=m.random.key(0), num_chains=4,
                          progress=False, return_info=True)
    assert np.all(np.asarray(rate) == 1.0)
    for k, v in init.items():
        want = np.broadcast_to(np.asarray(v, np.float32), np.asarray(s[k]).shape[2:])
        for c in range(4):
            for i in range(4):
                np.testing.assert_array_equal(np.asarray(s[k])[c, i], want)


def test_transform_nuts_trace_matches_oracle(gpu):
    import mlx_mcmc_amd as m

    plp, pinit = W.eight_schools_nc_log(W.ns_product())
    olp, oinit = W.eight_schools_nc_log(W.ns_oracle())
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
    print(f"eight schools (log tau) NUTS: trees identical for {same} of {n_w + n_s} iterations")
    assert same >= 10, f"trees diverged at iteration {same}"


def test_transform_mh_trace_matches_oracle(gpu):
    import mlx_mcmc_amd as m

    lp, init = W.lognormal(W.ns_product())
    olp, _ = W.lognormal(W.ns_oracle())
    n = 150
    s, rate, info = m.metropolis_hastings(lp, init, num_samples=n, proposal_scale=0.05,
                                          random_seed=5, return_info=True, return_trace=True)
    ref = S.metropolis_hastings(olp, init, num_samples=n, proposal_scale=0.05, random_seed=5)
    acc = info.trace["accepted"][0].astype(bool)
    assert list(acc) == ref.trace["accepted"] and 0 < acc.mean() < 1
    np.testing.assert_allclose(s["x"], ref.samples, rtol=1e-5, atol=1e-6)


# shape -> (slices, step size, leapfrog steps, chains, warmup, samples, batch)
REPARAM = {"small_tape": ("small", 1, 0.02, 50, 1024, 1000, 20000, 2000),
           "small": ("small", 0, 0.02, 50, 1024, 1000, 20000, 2000),
           "large": ("large", 0, 2e-3, 20, 256, 1000, 60000, 3000),
           "large_general": ("large", 0, 2e-3, 20, 256, 1000, 60000, 3000)}


@pytest.mark.parametrize("case", list(REPARAM))
def test_hier_reparam_posterior_within_one_percent(gpu, case):
    """The hierarchical model in (mu, log tau, log sigma, theta): its exact
    moments are the fixture's (log tau, log sigma) grid moments and the
    (mu, theta) ones (tests/test_exact_posterior.py pins the change of
    variables).  small_tape: the tape kernel k_hmc; small / large: the
    automatic plan, the lane-resident kernels with one / 16 slices (k_hmc_lf;
    large_general: k_hmc_lr)."""
    from mlx_mcmc_amd import _trace

    shape, slices, eps, L, C, Wm, S_, batch = REPARAM[case]
    with open(os.path.join(GOLD, "posterior_exact.json")) as f:
        ex = json.load(f)["shapes"][shape]
    mean = np.array(ex["mean"])
    var = np.array(ex["var"])
    mean[1:3] = ex["log_tau_sigma_mean"]
    var[1:3] = ex["log_tau_sigma_var"]
    from mlx_mcmc_amd import _lib

    lp, init = W.hierarchical_reparam(W.ns_product(), *W.SHAPES[shape])
    prog = _trace.compile_model(lp, init, slices=slices)
    assert prog.slice_kernel == ("unsliced" if slices == 1 else "lanes")
    if case == "large_general":
        _lib.load().mc_debug_lanes_fast(0)  # k_hmc_lr instead of k_hmc_lf
    try:
        g = stream_moments(prog, "hmc", C, prog.layout.flatten(init), step_size=eps,
                           num_warmup=Wm, num_samples=S_, batch=batch, num_leapfrog_steps=L)
    finally:
        _lib.load().mc_debug_lanes_fast(1)
    print(f"hier reparam {case}: kernel {prog.slice_kernel} ({prog.num_slices} slices), accept "
          f"{g['accept_rate'].mean():.3f} (min {g['accept_rate'].min():.3f})")
    assert g["accept_rate"].min() > 0.5
    check_within_one_percent(g, {"mean": mean, "var": var}, label=f"hierarchical {case} (log scales)",
                             z=Z)


def test_lognormal_posterior_within_one_percent(gpu):
    from mlx_mcmc_amd import _trace

    lp, init = W.lognormal(W.ns_product())
    prog = _trace.compile_model(lp, init)
    g = stream_moments(prog, "hmc", 1024, prog.layout.flatten(init), step_size=0.05,
                       num_warmup=500, num_samples=40000, batch=4000, num_leapfrog_steps=40)
    print(f"lognormal: accept {g['accept_rate'].mean():.3f} (min {g['accept_rate'].min():.3f})")
    assert g["accept_rate"].min() > 0.5
    check_within_one_percent(g, W.lognormal_moments(), label="lognormal D=20", z=Z)
