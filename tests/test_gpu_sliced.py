"""Sliced HMC: a chain's log density split over S workgroups, by the term
interpreter (csrc/sliced.h, k_hmc_sl) and the lane-resident kernel
(csrc/lanes.h, k_hmc_lr).

Both run the same sampler as k_hmc (reference hmc.py:7-206); only fp32
summation order differs (per-slice partial sums, combined in slice order).
Every test runs both kernels.  Parity bars:
  * accept decisions and step sizes identical to the unsliced kernel on every
    chain for the whole (short) run, positions within rtol 1e-3 — on models
    that cover every operand combination the planner handles (shared-only
    terms, per-element value / loc / scale parameters, data operands,
    HalfNormal, small terms placed whole in one slice);
  * bit-identical results across runs, across chain splits (chain_offset) and
    across chain-block sizes (8 vs 16 chains per workgroup);
  * the golden HMC trace of tests/golden/hmc_simple.json (oracle) reproduced;
  * at the Large shape (bench.py workload, eps where chains move) decisions
    match the unsliced kernel and are a mix of accepts and rejects.
"""
import json
import os

import numpy as np
import pytest

import workloads as W

pytestmark = pytest.mark.gpu


def _m():
    import mlx_mcmc_amd as m

    return m


# ---------------------------------------------------------------- models --
def model_iid(ns):
    """Only broadcast parameters: every term is shared-only (Pmax = 0)."""
    rng = np.random.default_rng(3)
    y = rng.normal(1.5, 2.0, 3000).astype(np.float32)

    def lp(p):
        return (ns.Normal(0.0, 10.0).log_prob(p["mu"])
                + ns.HalfNormal(5.0).log_prob(p["sigma"])
                + ns.sum(ns.Normal(p["mu"], p["sigma"]).log_prob(ns.array(y))))

    return lp, {"mu": 0.0, "sigma": 1.0}


def model_scale_vec(ns):
    """Per-element scale parameter (elementwise mode) + HalfNormal value pp."""
    rng = np.random.default_rng(4)
    n = 300
    s_true = rng.uniform(0.5, 2.0, n)
    y = (rng.normal(0.0, 1.0, n) * s_true + 0.3).astype(np.float32)

    def lp(p):
        return (ns.Normal(0.0, 5.0).log_prob(p["mu"])
                + ns.sum(ns.HalfNormal(2.0).log_prob(p["s"]))
                + ns.sum(ns.Normal(p["mu"], p["s"]).log_prob(ns.array(y))))

    return lp, {"mu": 0.0, "s": np.ones(n, np.float32)}


def model_value_pp(ns):
    """Per-element value parameter against data loc, and a HalfNormal on data."""
    rng = np.random.default_rng(5)
    n = 500
    m0 = rng.normal(0.0, 1.0, n).astype(np.float32)
    z = np.abs(rng.normal(0.0, 1.5, 200)).astype(np.float32)

    def lp(p):
        return (ns.sum(ns.Normal(ns.array(m0), p["tau"]).log_prob(p["theta"]))
                + ns.HalfNormal(1.0).log_prob(p["tau"])
                + ns.sum(ns.HalfNormal(p["tau"]).log_prob(ns.array(z))))

    return lp, {"theta": np.zeros(n, np.float32), "tau": 1.0}


def model_hier_small(ns):
    G, N = W.SHAPES["small"]
    return W.hierarchical(ns, G, N)


def model_scalar_mix(ns):
    """Hierarchical model whose scalar terms are not all single-parameter
    Normal / HalfNormal priors: z ~ Normal(mu, sigma) couples two shared
    parameters, tau ~ Gamma(3, 1) (the lane-resident kernel's generic scalar path;
    a constant shape with a nonzero gammaln normaliser)."""
    rng = np.random.default_rng(6)
    G, N = 12, 1200
    group = (np.arange(N) * G) // N
    y = (rng.normal(1.0, 1.0, G)[group] + rng.normal(0.0, 0.7, N)).astype(np.float32)

    def lp(p):
        mu, tau, sigma, z, th = p["mu"], p["tau"], p["sigma"], p["z"], p["theta"]
        out = ns.Normal(0.0, 5.0).log_prob(mu) + ns.Gamma(3.0, 1.0).log_prob(tau)
        out = out + ns.HalfNormal(2.0).log_prob(sigma) + ns.Normal(mu, sigma).log_prob(z)
        out = out + ns.sum(ns.Normal(mu, tau).log_prob(th))
        return out + ns.sum(ns.Normal(th[group], sigma).log_prob(ns.array(y)))

    return lp, {"mu": 0.5, "tau": 1.0, "sigma": 0.8, "z": 0.3,
                "theta": np.full(G, 0.9, np.float32)}


def model_ab_beta(ns):
    """Only scalar Beta terms with constant shapes (example 03): the
    normaliser log B(a, b) of every term enters log p."""
    return W.ab_testing(ns)


MODELS = {"iid": model_iid, "scale_vec": model_scale_vec, "value_pp": model_value_pp,
          "hier_small": model_hier_small, "scalar_mix": model_scalar_mix,
          "ab_beta": model_ab_beta}


KERNELS = ["interpreter", "lanes"]


def _run(lp, init, slices, C=8, warm=10, samp=10, L=8, eps=0.02, seed=3, chain_offset=0,
         kernel="auto"):
    m = _m()
    s, rate, info = m.hmc(lp, init, num_samples=samp, num_warmup=warm, step_size=eps,
                          num_leapfrog_steps=L, key=m.random.key(seed), num_chains=C,
                          chain_offset=chain_offset, progress=False, return_info=True,
                          return_trace=True, num_slices=slices, slice_kernel=kernel)
    return s, info


# ----------------------------------------------------------------- tests --
def test_auto_slicing_large_and_small(gpu):
    from mlx_mcmc_amd import _trace

    G, N = W.SHAPES["large"]
    big = _trace.compile_model(*W.hierarchical(W.ns_product(), G, N))
    assert big.num_slices == 16 and big.slice_kernel == "lanes"
    big.set_slice_kernel("interpreter")
    assert big.slice_kernel == "interpreter"
    small = _trace.compile_model(*W.simple_normal(W.ns_product()))
    assert small.num_slices == 1


def test_unsliceable_program_is_rejected(gpu):
    from mlx_mcmc_amd import _lib, _trace

    def lp(p):
        ns = W.ns_product()
        return ns.sum(ns.Normal(0.0, p["s"]).log_prob(p["x"]))   # two per-element params

    prog = _trace.compile_model(lp, {"x": np.zeros(10, np.float32),
                                     "s": np.ones(10, np.float32)})
    with pytest.raises(_lib.EngineError):
        prog.set_slices(2)
    assert prog.num_slices == 1


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("name", sorted(MODELS))
@pytest.mark.parametrize("S", [2, 3])
def test_sliced_matches_unsliced(gpu, name, S, kernel):
    lp, init = MODELS[name](W.ns_product())
    a, ia = _run(lp, init, 1)
    b, ib = _run(lp, init, S, kernel=kernel)
    np.testing.assert_array_equal(ia.trace["accepted"], ib.trace["accepted"])
    np.testing.assert_array_equal(ia.trace["step_size"], ib.trace["step_size"])
    for k in a:
        np.testing.assert_allclose(b[k], a[k], rtol=1e-3, atol=1e-4)
    np.testing.assert_allclose(ib.trace["energy"], ia.trace["energy"], rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("name", ["hier_small", "iid", "scalar_mix", "ab_beta", "iso100"])
def test_lanes_one_slice_matches_unsliced(gpu, name):
    """An unsliced program on the lane-resident kernel (one slice, no
    exchange; slice_kernel="lanes") against k_hmc: same decisions and step
    sizes, positions within rtol 1e-3.  (scale_vec and value_pp have more
    than 256 private parameters: test_lanes_one_slice_selection.)"""
    if name == "iso100":
        lp, init = W.iso_normal(W.ns_product(), 100)
    else:
        lp, init = MODELS[name](W.ns_product())
    a, ia = _run(lp, init, 1, C=12)
    b, ib = _run(lp, init, 1, C=12, kernel="lanes")
    np.testing.assert_array_equal(ia.trace["accepted"], ib.trace["accepted"])
    np.testing.assert_array_equal(ia.trace["step_size"], ib.trace["step_size"])
    for k in a:
        np.testing.assert_allclose(b[k], a[k], rtol=1e-3, atol=1e-4)
    np.testing.assert_allclose(ib.trace["energy"], ia.trace["energy"], rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("C", [1, 3, 17, 100])
def test_lanes_one_slice_chain_counts(gpu, C):
    """The automatic one-slice kernel on part-filled and single-chain blocks
    (dead waves of a workgroup must not store) against k_hmc; L = 0 runs fall
    back to k_hmc on the same program."""
    m = _m()
    lp, init = model_hier_small(W.ns_product())
    a, ia = _run(lp, init, 1, C=C)
    b, ib = _run(lp, init, 0, C=C)
    np.testing.assert_array_equal(ia.trace["accepted"], ib.trace["accepted"])
    for k in a:
        np.testing.assert_allclose(b[k], a[k], rtol=1e-3, atol=1e-4)
    s0, _ = m.hmc(lp, init, num_samples=3, num_warmup=3, num_leapfrog_steps=0,
                  key=m.random.key(1), num_chains=C, progress=False)
    for k in s0:
        assert np.all(np.isfinite(s0[k]))


def test_lanes_one_slice_selection(gpu):
    from mlx_mcmc_amd import _trace

    lp, init = W.iso_normal(W.ns_product(), 100)
    prog = _trace.compile_model(lp, init)          # automatic: one-slice lanes
    assert prog.num_slices == 1 and prog.slice_kernel == "lanes"
    prog.set_slice_kernel("interpreter")           # unsliced: k_hmc
    assert prog.slice_kernel == "unsliced"
    prog.set_slice_kernel("lanes")
    assert prog.num_slices == 1 and prog.slice_kernel == "lanes"
    prog.set_slices(1)                             # an explicit 1: k_hmc
    assert prog.slice_kernel == "unsliced"
    from mlx_mcmc_amd import _lib

    big = _trace.compile_model(*model_value_pp(W.ns_product()))   # 500 private parameters
    assert big.slice_kernel == "unsliced"
    with pytest.raises(_lib.EngineError, match="256 private"):
        big.set_slice_kernel("lanes")
    assert big.slice_kernel == "unsliced"


@pytest.mark.parametrize("kernel", KERNELS)
def test_sliced_determinism_chain_split_and_block_size(gpu, kernel):
    lp, init = model_hier_small(W.ns_product())
    full, _ = _run(lp, init, 4, C=24, kernel=kernel)          # 16-chain blocks
    again, _ = _run(lp, init, 4, C=24, kernel=kernel)
    for k in full:
        np.testing.assert_array_equal(full[k], again[k])
    part, _ = _run(lp, init, 4, C=4, chain_offset=10, kernel=kernel)  # a part-filled block
    for k in full:
        np.testing.assert_array_equal(full[k][10:14], part[k])


@pytest.mark.parametrize("kernel", KERNELS)
def test_sliced_golden_hmc_trace(gpu, kernel):
    m = _m()
    with open(os.path.join(os.path.dirname(__file__), "golden", "hmc_simple.json")) as f:
        h = json.load(f)
    lp, init = W.simple_normal(W.ns_product())
    _, _, info = m.hmc(lp, init, num_samples=h["num_samples"], num_warmup=h["num_warmup"],
                       step_size=h["step_size"], num_leapfrog_steps=h["num_leapfrog_steps"],
                       key=m.random.key(h["seed"]), progress=False, return_info=True,
                       return_trace=True, num_slices=2, slice_kernel=kernel)
    acc = info.trace["accepted"][0].astype(bool).tolist()
    same = next((i for i, (x, y) in enumerate(zip(acc, h["accepted"])) if x != y), len(acc))
    assert same >= 50
    np.testing.assert_array_equal(info.trace["step_size"][0][:same], h["eps"][:same])


@pytest.mark.parametrize("kernel", KERNELS)
def test_sliced_large_matches_unsliced(gpu, kernel):
    """bench.py's workload (16 slices) against k_hmc, at a step size where the
    chains move (eps0 = 3e-3, the reference's rule acting at i = 11..14; at
    eps = 0.01 every trajectory diverges and every proposal is rejected, which
    would compare nothing): decisions, step sizes and energies agree, and the
    decisions are a mix.  The two kernels sum the log density in different
    orders, so a decision may flip at a proven near-tie (tests/_near_tie.py);
    draws are compared up to it.  The oracle comparison at this shape is
    tests/test_gpu_large_parity.py."""
    from _near_tie import compare_trace, log_u

    G, N = W.SHAPES["large"]
    lp, init = W.hierarchical(W.ns_product(), G, N)
    a, ia = _run(lp, init, 1, C=16, warm=15, samp=15, L=20, eps=3e-3)
    b, ib = _run(lp, init, 0, C=16, warm=15, samp=15, L=20, eps=3e-3, kernel=kernel)
    acc = ia.trace["accepted"].astype(bool)
    assert 0 < acc.mean() < 1, "the regime must mix accepts and rejects"
    full = 0
    for c in range(16):
        ref = {"accepted": ia.trace["accepted"][c], "ratio": ia.trace["accept_stat"][c],
               "energy": ia.trace["energy"][c], "step_size": ia.trace["step_size"][c],
               "log_u": log_u(3, c, 30)}
        got = {"accepted": ib.trace["accepted"][c], "ratio": ib.trace["accept_stat"][c],
               "energy": ib.trace["energy"][c], "step_size": ib.trace["step_size"][c]}
        same = compare_trace(got, ref, f"{kernel} chain {c}")
        full += same == 30
        ns = max(0, same - 15)
        for k in a:
            np.testing.assert_allclose(b[k][c, :ns], a[k][c, :ns], rtol=1e-4, atol=1e-5)
    assert full >= 10, "most chains agree over the whole run (the rest to a proven near-tie)"


@pytest.mark.parametrize("kernel", KERNELS)
def test_sliced_posterior(gpu, kernel):
    """Reference-style statistical check through the sliced path
    (tests/test_hmc.py:13-40 posterior of the simple normal model)."""
    m = _m()
    lp, init = W.simple_normal(W.ns_product())
    s, rate = m.hmc(lp, init, num_samples=1000, num_warmup=500, step_size=0.1,
                    num_leapfrog_steps=10, key=m.random.key(0), num_chains=16, progress=False,
                    num_slices=2, slice_kernel=kernel)
    assert abs(float(np.mean(s["mu"])) - 5.0) < 0.6
    assert 1.4 < float(np.mean(s["sigma"])) < 2.6
    assert 0.3 < float(np.mean(rate)) <= 1.0


def test_lanes_launch_split_and_workspace_reuse(gpu):
    """The lane-resident kernel's exchange tags continue across launches on
    one workspace (no clearing between launches): a run split into one launch
    per iteration equals a single launch, also when another kernel (the term
    interpreter, whose tags restart at 1) has used the same workspace in
    between."""
    import torch

    from mlx_mcmc_amd import _engine, _trace

    lp, init = model_hier_small(W.ns_product())
    prog = _trace.compile_model(lp, init, slices=4, slice_kernel="lanes")
    assert prog.slice_kernel == "lanes"
    q0 = prog.layout.flatten(init)
    cfg = dict(chain_offset=0, num_warmup=6, num_samples=6, sample_begin=0, sample_capacity=6,
               seed=11, step_size=0.02, target_accept=0.8, num_leapfrog_steps=6,
               adapt_step_size=True)

    def run(split, other_between=False):
        cs = _engine.ChainSet(prog, 24, q0, 0.02)
        out = torch.zeros((24, 6, prog.D), dtype=torch.float32, device=cs.device)
        if split:
            for it in range(12):
                cs.run_hmc(samples=out, iter_begin=it, iter_count=1, **cfg)
                if other_between and it == 5:
                    other = _engine.ChainSet(prog, 24, q0, 0.02)
                    other._ws = cs._ws          # the same workspace
                    prog.set_slice_kernel("interpreter")
                    try:
                        other.run_hmc(iter_begin=0, iter_count=1, **cfg)
                    finally:
                        prog.set_slice_kernel("lanes")
                        other._ws = None
        else:
            cs.run_hmc(samples=out, iter_begin=0, iter_count=12, **cfg)
        torch.cuda.synchronize()
        cs.check_status()
        return out.cpu().numpy()

    one = run(False)
    np.testing.assert_array_equal(run(True), one)
    np.testing.assert_array_equal(run(True, other_between=True), one)


@pytest.mark.parametrize("kernel", KERNELS)
def test_exchange_timeout_reported_and_state_kept(gpu, kernel):
    """The exchange kernels' timeout path (include/mcmc355.h,
    mc_workspace_status / mc_debug_exchange_fault): with the grid's last
    workgroup never publishing, the other slices of its chain block time out.
    mc_workspace_status then reports MC_ERR_TIMEOUT; the chains of the
    stranded block keep their state (positions and counters as before the
    launch), every other chain equals an undisturbed run; the next launch on
    the same workspace runs clean."""
    import torch

    from mlx_mcmc_amd import _engine, _lib, _trace

    lp, init = model_hier_small(W.ns_product())
    prog = _trace.compile_model(lp, init, slices=4, slice_kernel=kernel)
    q0 = prog.layout.flatten(init)
    cfg = dict(chain_offset=0, num_warmup=4, num_samples=0, sample_begin=0, sample_capacity=0,
               seed=5, step_size=0.02, target_accept=0.8, num_leapfrog_steps=6,
               adapt_step_size=True)
    lib = _lib.load()

    ref = _engine.ChainSet(prog, 40, q0, 0.02)
    ref.run_hmc(iter_begin=0, iter_count=4, **cfg)
    torch.cuda.synchronize()
    ref.check_status()

    cs = _engine.ChainSet(prog, 40, q0, 0.02)
    cs.run_hmc(iter_begin=0, iter_count=2, **cfg)
    torch.cuda.synchronize()
    cs.check_status()
    before_q = cs.positions().cpu().numpy().copy()
    before_n = cs.scalars()["n_total"].copy()
    lib.mc_debug_exchange_fault(1)
    try:
        cs.run_hmc(iter_begin=2, iter_count=2, **cfg)
        torch.cuda.synchronize()
        with pytest.raises(_lib.EngineError, match="timed out"):
            cs.check_status()
    finally:
        lib.mc_debug_exchange_fault(0)
    after_q = cs.positions().cpu().numpy()
    after_n = cs.scalars()["n_total"]
    ref_q = ref.positions().cpu().numpy()
    kept = np.all(after_q == before_q, axis=1) & (after_n == before_n)
    done = np.all(after_q == ref_q, axis=1) & (after_n == before_n + 2)
    assert np.all(kept | done), "every chain is either untouched or finished"
    assert kept.any() and done.any()
    # the next launch on the same workspace starts clean
    cs.run_hmc(iter_begin=2, iter_count=1, **cfg)
    torch.cuda.synchronize()
    cs.check_status()
