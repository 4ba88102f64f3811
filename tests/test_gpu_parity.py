"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle.

Bars (stated per test): bit-exact for integer work (Philox words), exact or
<= 1 ulp for the draw transforms, fp32 tolerances for the tape (different
summation order than the oracle's autograd), identical accept / tree
decisions until the first near-tie for the sampler traces.
"""
import ctypes

import numpy as np
import pytest

import workloads as W
from oracle import philox as R
from oracle import samplers as S

pytestmark = pytest.mark.gpu


def _lib():
    from mlx_mcmc_amd import _lib

    return _lib


def _rng(gpu, seed, chain, it, tag, sub, index0, n, mode):
    import torch

    L = _lib()
    dt = torch.int32 if mode == 0 else torch.float32
    out = torch.empty(4 * n, dtype=dt, device=gpu)
    L.check(L.load().mc_rng_fill(seed, chain, it, tag, sub, index0, n, mode, L.ptr(out),
                                 L.stream_handle()))
    return out.cpu().numpy()


def test_philox_words_bit_exact(gpu):
    seed = 0x123456789ABCDEF
    got = _rng(gpu, seed, 5, 77, R.TAG_MOMENTUM, 3, 10, 4096, 0).view(np.uint32).reshape(-1, 4)
    ref = R.draw(seed, 5, 77, R.TAG_MOMENTUM, 3, 10 + np.arange(4096))
    np.testing.assert_array_equal(got, ref)


def test_uniform_and_normal_transforms(gpu):
    seed = 42
    u = _rng(gpu, seed, 1, 2, R.TAG_ACCEPT, 0, 0, 4096, 1).reshape(-1, 4)
    ref_w = R.draw(seed, 1, 2, R.TAG_ACCEPT, 0, np.arange(4096))
    np.testing.assert_array_equal(u, R.u01_f32(ref_w))          # exact
    z = _rng(gpu, seed, 1, 2, R.TAG_ACCEPT, 0, 0, 4096, 2).reshape(-1, 4)
    zr = R.normals4(ref_w)
    # the f32 Box-Muller from IEEE operations only: bit-exact (philox.h)
    np.testing.assert_array_equal(z, zr)
    # and the device's accept-uniform log (mc_logf_u01) through the sampler:
    # covered by the HMC trace tests (log U enters every decision)


def _tape_case(name):
    if name == "simple":
        return W.simple_normal(W.ns_product()), W.simple_normal(W.ns_oracle())
    if name == "iso":
        return W.iso_normal(W.ns_product()), W.iso_normal(W.ns_oracle())
    if name == "illcond":
        return W.illcond_normal(W.ns_product()), W.illcond_normal(W.ns_oracle())
    G, N = W.SHAPES[name]
    return W.hierarchical(W.ns_product(), G, N), W.hierarchical(W.ns_oracle(), G, N)


@pytest.mark.parametrize("name", ["simple", "iso", "illcond", "small", "medium", "large"])
def test_tape_matches_autograd(gpu, name):
    """log p and its gradient at random points: GPU tape vs torch autograd (fp32).

    Tolerance: |dlp| <= 2e-6 * sum_i |lp_i| (+1e-4), grad components within
    rtol 1e-4 + 1e-5 * max|grad| — both fp32 sums of the same terms in
    different orders."""
    from mlx_mcmc_amd import _engine, _trace

    (plp, pinit), (olp, oinit) = _tape_case(name)
    prog = _trace.compile_model(plp, pinit)
    M = S.EagerModel(olp, oinit)
    rng = np.random.default_rng(0)
    q0 = M.flatten(oinit)
    pts = np.stack([q0 + rng.normal(0, 0.3, q0.size).astype(np.float32) for _ in range(4)])
    if name in ("simple",):
        pts[:, 1] = np.abs(pts[:, 1]) + 0.5
    if name in ("small", "medium", "large"):
        pts[:, 1:3] = np.abs(pts[:, 1:3]) + 0.5
    lp, g = _engine.logp_grad(prog, pts)
    lp, g = lp.cpu().numpy(), g.cpu().numpy()
    for i, q in enumerate(pts):
        rl, rg = M.logp_grad(q)
        scale = float(np.abs(rl)) + 1.0
        assert abs(lp[i] - rl) <= 2e-6 * scale * max(1.0, np.sqrt(q.size / 100)) + 1e-4, \
            (lp[i], rl)
        np.testing.assert_allclose(g[i], rg, rtol=1e-4, atol=1e-5 * np.abs(rg).max() + 1e-5)


def test_dist_log_prob_kats(gpu):
    """tests/test_distributions.py:18-32,67-79 of the reference, on the GPU path."""
    import mlx_mcmc_amd as m

    assert np.isclose(float(m.Normal(0, 1).log_prob(0.0)), -0.5 * np.log(2 * np.pi),
                      rtol=1e-5)
    assert np.isclose(float(m.Normal(0, 1).log_prob(1.0)), float(m.Normal(0, 1).log_prob(-1.0)),
                      rtol=1e-5)
    assert float(m.HalfNormal(1.0).log_prob(-1.0)) == -np.inf
    assert np.isclose(float(m.HalfNormal(1.0).log_prob(0.0)),
                      np.log(2.0) - 0.5 * np.log(2 * np.pi), rtol=1e-5)
    assert float(m.HalfNormal(1.0).log_prob(0.5)) < 0


def _first_divergence(a, b):
    for i, (x, y) in enumerate(zip(a, b)):
        if bool(x) != bool(y):
            return i
    return None


def test_hmc_trace_parity_simple(gpu):
    """Config 1: same draws -> same accept decisions and bit-identical eps
    sequence, until a near-tie (|log u - ratio| within fp32 noise)."""
    import mlx_mcmc_amd as m

    plp, pinit = W.simple_normal(W.ns_product())
    olp, oinit = W.simple_normal(W.ns_oracle())
    n_w, n_s = 100, 100
    _, _, info = m.hmc(plp, pinit, num_samples=n_s, num_warmup=n_w, key=m.random.key(3),
                       progress=False, return_info=True, return_trace=True)
    ref = S.hmc(olp, oinit, num_samples=n_s, num_warmup=n_w, seed=3)
    ga = info.trace["accepted"][0].astype(bool)
    d = _first_divergence(ga, ref.trace["accepted"])
    upto = len(ga) if d is None else d
    assert upto >= 50, f"decisions diverged at iteration {d}"
    np.testing.assert_array_equal(info.trace["step_size"][0][:upto],
                                  np.array(ref.trace["step_size"][:upto]))
    np.testing.assert_allclose(info.trace["accept_stat"][0][:upto],
                               np.array(ref.trace["ratio"][:upto]), rtol=1e-3, atol=2e-3)
    # a divergence must be a proven near-tie (tests/_near_tie.py): |log U -
    # ratio| within 8 ulp of |H|, ratios and H within that bound before it
    from _near_tie import compare_trace, log_u

    n = n_w + n_s
    gpu_c = {"accepted": ga, "ratio": info.trace["accept_stat"][0],
             "step_size": info.trace["step_size"][0], "energy": info.trace["energy"][0]}
    ref_c = {k: np.asarray(ref.trace[k]) for k in ("accepted", "ratio", "step_size", "energy")}
    ref_c["log_u"] = log_u(3, 0, n)
    assert compare_trace(gpu_c, ref_c, "simple normal", verbose=True) == upto


@pytest.mark.parametrize("kernel", ["auto", "tape"])
def test_nuts_trace_parity_illcond(gpu, kernel):
    """Config 5 (kappa = 1000, slice active): identical tree depths and leaf
    counts until the first near-tie — on the lane-resident NUTS kernel
    (k_nuts_lr, the automatic choice for this model) and on k_nuts."""
    import mlx_mcmc_amd as m

    plp, pinit = W.illcond_normal(W.ns_product())
    olp, oinit = W.illcond_normal(W.ns_oracle())
    n_w, n_s = 30, 10
    _, _, info = m.nuts(plp, pinit, num_samples=n_s, num_warmup=n_w, key=m.random.key(11),
                        progress=False, return_info=True, return_trace=True, nuts_kernel=kernel)
    assert info.extra["kernel"] == ("lanes" if kernel == "auto" else "tape")
    ref = S.nuts(olp, oinit, num_samples=n_s, num_warmup=n_w, seed=11)
    depth = info.trace["tree_depth"][0]
    leaves = info.trace["n_leapfrog"][0]
    same = 0
    for i in range(n_w + n_s):
        if depth[i] != ref.trace["depth"][i] or leaves[i] != ref.trace["leaves"][i]:
            break
        same += 1
    assert same >= 10, f"trees diverged at iteration {same}"
    # alpha feeds dual averaging, so fp32 differences in H (summation order)
    # are amplified iteration by iteration; the first iterations agree closely
    np.testing.assert_allclose(info.trace["accept_stat"][0][:8],
                               np.array(ref.trace["alpha"][:8]), rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(info.trace["step_size"][0][:8],
                               np.array(ref.trace["step_size"][:8]), rtol=3e-4)  # x sqrt(m+1)/gamma gain


def test_nuts_lanes_matches_tape_hierarchical(gpu):
    """k_nuts_lr against k_nuts on a model with broadcast (mu, tau, sigma) and
    private (theta) parameters: the same draws give the same trees until the
    first fp32 near-tie (the kernels differ in summation order only), and
    the same posterior."""
    import mlx_mcmc_amd as m

    lp, init = W.hierarchical(W.ns_product(), *W.SHAPES["small"])

    def run(kernel, **kw):
        return m.nuts(lp, init, num_samples=300, num_warmup=200, key=m.random.key(5),
                      num_chains=16, progress=False, return_info=True, return_trace=True,
                      nuts_kernel=kernel, **kw)

    runs = {k: run(k) for k in ("auto", "tape")}
    assert runs["auto"][2].extra["kernel"] == "lanes"
    assert runs["tape"][2].extra["kernel"] == "tape"
    da, db = runs["auto"][2].trace["tree_depth"], runs["tape"][2].trace["tree_depth"]
    la, lb = runs["auto"][2].trace["n_leapfrog"], runs["tape"][2].trace["n_leapfrog"]
    same = []
    for c in range(16):
        k = 0
        while k < da.shape[1] and da[c, k] == db[c, k] and la[c, k] == lb[c, k]:
            k += 1
        same.append(k)
    assert sorted(same)[4] >= 10, f"trees diverged early: {same}"
    # the same posterior: with the reference's f32 slice (Q7 / Q8) this
    # model (H0 ~ 1400) switches the slice off and counts NaN leaves as
    # alpha = 1, so dual averaging drives most chains to a frozen huge step
    # size or along the funnel — which chains, depends on the last bits (the
    # lane kernel's replicated layout, lanes.h LrCtx::rep, sums in another
    # order than the tape); the f64 slice (slice_mode="exact") keeps the
    # chains mixing, and both kernels' pooled moments must agree
    post = {k: run(k, slice_mode="exact") for k in ("auto", "tape")}
    for name in ("mu", "tau", "sigma"):
        a, b = post["auto"][0][name], post["tape"][0][name]    # [C, S]
        sa = np.sqrt(a.mean(1).var() / a.shape[0] + b.mean(1).var() / b.shape[0])
        assert abs(a.mean() - b.mean()) < 5 * sa + 1e-3, (name, a.mean(), b.mean(), sa)
    # the default mode (the reference's f32 slice) as well, on the chains that
    # keep mixing in both runs: a step size that neither froze huge nor
    # collapsed, and draws that move (the replicated layout's
    # default-mode posterior was otherwise unchecked)
    ea = runs["auto"][2].trace["step_size"][:, -1]
    eb = runs["tape"][2].trace["step_size"][:, -1]
    sa_, sb_ = runs["auto"][0], runs["tape"][0]
    # (which chains freeze depends on the last bits, so each run's mixing
    # chains are pooled on their own: two samples of the same posterior)
    ma = [c for c in range(16) if 1e-4 < ea[c] < 1.0 and np.ptp(sa_["mu"][c]) > 0]
    mb = [c for c in range(16) if 1e-4 < eb[c] < 1.0 and np.ptp(sb_["mu"][c]) > 0]
    print(f"default mode: {len(ma)} / {len(mb)} of 16 chains mixing (lanes / tape)")
    assert len(ma) >= 4 and len(mb) >= 4, (ea, eb)
    for name in ("mu", "tau", "sigma"):
        a, b = sa_[name][ma], sb_[name][mb]
        sa = np.sqrt(a.mean(1).var() / a.shape[0] + b.mean(1).var() / b.shape[0])
        assert abs(a.mean() - b.mean()) < 5 * sa + 1e-3, ("default", name, a.mean(), b.mean(), sa)


@pytest.mark.parametrize("model", ["illcond", "eight_schools"])
def test_dscale_lanes_hmc_matches_tape(gpu, model):
    """Normal terms with a per-element data scale on the lane-resident kernels
    (lanes.h LS_DSCALE: tiles of 1/s^2 and log s) against k_hmc (the tape,
    num_slices=1): same draws, the same accept decisions until the first fp32
    near-tie, positions within rtol 1e-3 before it."""
    import mlx_mcmc_amd as m

    lp, init = (W.illcond_normal(W.ns_product()) if model == "illcond"
                else W.eight_schools(W.ns_product()))
    step = 0.02 if model == "illcond" else 0.2
    out = {}
    for slices in (0, 1):
        s, _, info = m.hmc(lp, init, num_samples=60, num_warmup=60, step_size=step,
                           num_leapfrog_steps=10, key=m.random.key(2), num_chains=8,
                           progress=False, return_info=True, return_trace=True,
                           num_slices=slices)
        out[slices] = (s, info)
    assert out[0][1].extra["kernel"] == "lanes" and out[1][1].extra["kernel"] == "unsliced"
    a, b = out[0][1].trace["accepted"], out[1][1].trace["accepted"]
    assert 0 < a.mean() < 1
    firsts = []
    for c in range(8):
        d = np.nonzero(a[c] != b[c])[0]
        firsts.append(int(d[0]) if d.size else a.shape[1])
    assert sorted(firsts)[2] >= 30, firsts
    # positions: a fresh run's first draws (one warmup iteration, fixed eps),
    # before any divergence
    # (fp32 differences grow along the trajectories iteration by iteration:
    # after 60 iterations of the eight-schools funnel they reach ~1e-2)
    name = "x" if model == "illcond" else "theta"
    pos = {}
    for slices in (0, 1):
        s, _, info = m.hmc(lp, init, num_samples=8, num_warmup=1, step_size=step,
                           num_leapfrog_steps=10, key=m.random.key(9), num_chains=8,
                           progress=False, return_info=True, return_trace=True,
                           num_slices=slices, adapt_step_size=False)
        pos[slices] = (s[name], info.trace["accepted"])
    for c in range(8):
        d = np.nonzero(pos[0][1][c] != pos[1][1][c])[0]  # (trace: 1 warmup + 8)
        k = max(0, int(d[0]) - 1) if d.size else 8
        np.testing.assert_allclose(pos[0][0][c, :k], pos[1][0][c, :k], rtol=1e-3, atol=1e-3)


def test_nuts_lanes_eight_schools(gpu):
    """k_nuts_lr on the data-scale model against k_nuts: same trees until the
    first near-tie for most chains."""
    import mlx_mcmc_amd as m

    lp, init = W.eight_schools(W.ns_product())
    tr = {}
    for kernel in ("auto", "tape"):
        _, _, info = m.nuts(lp, init, num_samples=50, num_warmup=50, key=m.random.key(4),
                            num_chains=8, progress=False, return_info=True, return_trace=True,
                            nuts_kernel=kernel)
        tr[kernel] = info
    assert tr["auto"].extra["kernel"] == "lanes"
    same = []
    for c in range(8):
        k = 0
        while (k < 100 and tr["auto"].trace["tree_depth"][c, k] == tr["tape"].trace["tree_depth"][c, k]
               and tr["auto"].trace["n_leapfrog"][c, k] == tr["tape"].trace["n_leapfrog"][c, k]):
            k += 1
        same.append(k)
    assert sorted(same)[2] >= 10, same


def _measurement(ns, D=100):
    """y_i ~ N(theta_i, s_i), one observation per parameter (no prior): a
    data-scale term whose private operand is the loc and whose value is data."""
    rng = np.random.default_rng(8)
    s = (0.5 + rng.random(D)).astype(np.float32)
    y = rng.normal(0.0, 2.0, D).astype(np.float32)

    def log_prob(p):
        return ns.sum(ns.Normal(p["theta"], s).log_prob(y))

    return log_prob, {"theta": y.copy()}


@pytest.mark.parametrize("model", ["iso", "illcond", "measurement"])
def test_nuts_register_only_trees_match_oracle(gpu, model):
    """k_nuts_lr's register-only variant (one Normal term, one element per
    parameter, constant or data scale; api.hip lanes_register_only): identical
    tree depths and leaf counts to the oracle for the first iterations, on a
    direct term with constant loc / scale (iso), a data-scale term with the
    value private (illcond, config 5) and with the loc private (measurement)."""
    import mlx_mcmc_amd as m
    from mlx_mcmc_amd import _trace

    mk = {"iso": W.iso_normal, "illcond": W.illcond_normal, "measurement": _measurement}[model]
    plp, pinit = mk(W.ns_product())
    olp, oinit = mk(W.ns_oracle())
    assert _trace.compile_model(plp, pinit).nuts_register_only(10)
    n_w, n_s = 20, 10
    _, _, info = m.nuts(plp, pinit, num_samples=n_s, num_warmup=n_w, key=m.random.key(13),
                        progress=False, return_info=True, return_trace=True)
    assert info.extra["kernel"] == "lanes"
    ref = S.nuts(olp, oinit, num_samples=n_s, num_warmup=n_w, seed=13)
    same = 0
    for i in range(n_w + n_s):
        if (info.trace["tree_depth"][0][i] != ref.trace["depth"][i]
                or info.trace["n_leapfrog"][0][i] != ref.trace["leaves"][i]):
            break
        same += 1
    assert same >= 10, f"trees diverged at iteration {same}"
    assert max(ref.trace["depth"][:same]) >= 2   # real trees, not single leaves
    np.testing.assert_allclose(info.trace["accept_stat"][0][:6],
                               np.array(ref.trace["alpha"][:6]), rtol=1e-4, atol=1e-6)


def test_lds_attribute_large_small_large(gpu):
    """one kernel instantiation launched with more, then less, then
    more dynamic LDS (k_nuts<WPC, LDS>: the tree arena grows with
    max_tree_depth) — the per-kernel LDS attribute is raised, never lowered,
    so the third launch is not refused."""
    import mlx_mcmc_amd as m

    lp, init = W.hierarchical(W.ns_product(), *W.SHAPES["small"])
    for depth in (10, 2, 10, 1, 10):
        s, rate = m.nuts(lp, init, num_samples=2, num_warmup=2, step_size=0.01,
                         max_tree_depth=depth, key=m.random.key(0), num_chains=8,
                         progress=False, nuts_kernel="tape")
        assert np.all(np.isfinite(s["mu"]))
