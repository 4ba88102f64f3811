"""NUTS against the oracle over a long prefix (VERDICT r2 "Next round" 2;
reference nuts.py:137-319).

Fixtures (scripts/gen_golden_nuts.py, oracle/samplers.py nuts): config 5's
kappa = 1000 Gaussian (chains 0, 1, 33, 63 of the 64-chain launch) and the
small hierarchical model (chains 0, 2, 5; chain 5 shows the Q7/Q8 freeze),
W = 40 warmup iterations with dual averaging acting, S = 20 sampling
iterations.  Every k_nuts_lr variant (register-only, specialised, generic;
mc_debug_nuts_variant) and k_nuts (nuts_kernel="tape") runs the fixture's
launch, and two comparisons are made per fixture chain:

  * replay (strict): the oracle re-runs the chain at test time with the
    GPU's own step-size sequence (oracle nuts(step_sizes=...)), so the only
    difference left is fp32 summation order.  Tree depth and leaf count must
    agree at every iteration until a decision flips, and a flip is allowed
    only where the oracle proves a near-tie: a slice / divergence gap
    |log u + H'| or a relative U-turn dot within TIE of zero, with
    TIE = 8 ulp(|H0| + D) + 4 |H0_gpu - H0_oracle| (|H0| + D bounds the
    magnitude of H's fp32 parts |log p| + K; the H0 difference is the
    positions' accumulated rounding; tests/_near_tie.py's bound for HMC) for
    the slice, 1e-5 + the same relative H0 difference for the U-turn dot.
    The comparison runs while the two states agree to SEP_ULPS ulp of |H0| + D:
    beyond that the trajectories have amplified the rounding differences
    (the hierarchical model's funnel separates them exponentially: chain 0
    from ~1e-6 to ~3 % of H0 within 20 iterations) and a flip says nothing
    about either implementation.  Up to the flip or separation: alpha within
    the relative error of exp(TIE), stored draws within rtol 1e-4; at least
    MIN_REPLAY iterations compared (or every iteration before separation).
    The GPU's dual averaging is recomputed from its own alpha trace
    (nuts.py:299-310 restated here) and must reproduce its step sizes.
  * fixture (the oracle's own adaptation): the trees agree with the
    committed trace for at least MIN_SAME iterations (dual averaging
    amplifies the alpha rounding differences into eps differences
    iteration by iteration — a step of log eps is sqrt(m + 1) / 0.05 times
    the mean alpha difference — so a flip at a gap of that order comes
    within tens of iterations; the replay above is the strict check).

Real trees: the compared iterations include depths >= 3.
"""
import json
import os

import numpy as np
import pytest

import workloads as W

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
MIN_SAME = 8
SEP_ULPS = 64
MIN_REPLAY = 20


def _fixture(name):
    fx = np.load(os.path.join(GOLD, f"nuts_{name}_trace.npz"), allow_pickle=False)
    out = {k: fx[k] for k in fx.files}
    out["config"] = json.loads(str(out["config"]))
    return out


def _model(name, ns):
    if name == "illcond":
        return W.illcond_normal(ns)
    if name in ("medium", "large", "large_da"):
        return W.hierarchical(ns, *W.SHAPES["large" if name.startswith("large") else name])
    return W.hierarchical(ns, *W.SHAPES["small"])


def _gpu_run(name, variant, C):
    import mlx_mcmc_amd as m
    from mlx_mcmc_amd import _lib

    fx = _fixture(name)
    cfg = fx["config"]
    lp, init = _model(name, W.ns_product())
    lib = _lib.load()
    lib.mc_debug_nuts_variant({"auto": -1, "generic": 0, "spec": 1, "tape": -1}[variant])
    try:
        s, rate, info = m.nuts(lp, init, num_samples=cfg["num_samples"],
                               num_warmup=cfg["num_warmup"], step_size=cfg["step_size"],
                               max_tree_depth=cfg["max_tree_depth"],
                               target_accept=cfg["target_accept"], key=m.random.key(cfg["seed"]),
                               num_chains=C, progress=False, return_info=True,
                               return_trace=True, keep_on_device=True,
                               nuts_kernel="tape" if variant == "tape" else "auto")
    finally:
        lib.mc_debug_nuts_variant(-1)
    assert info.extra["kernel"] == ("tape" if variant == "tape" else "lanes")
    return fx, info


def _ulp(x):
    return float(np.spacing(np.float32(abs(x))))


def _hscale(h0, D):
    """Magnitude of H's fp32 parts: |log p| + K <= |H0| + 2K, K ~ D / 2."""
    return abs(float(h0)) + D


def _first_flip(gd, gl, rd, rl, n):
    for i in range(n):
        if gd[i] != rd[i] or gl[i] != rl[i]:
            return i
    return n


def _replay(name, fx, info, j, chain):
    """The strict comparison of one chain (see the module docstring)."""
    from oracle import samplers as S

    cfg = fx["config"]
    n = cfg["num_warmup"] + cfg["num_samples"]
    tr = info.trace
    g_eps = tr["step_size"][chain].astype(np.float64)
    # the GPU's dual averaging, recomputed from its own alpha trace
    da, eps_bar = S.dual_averaging_steps(tr["accept_stat"][chain], cfg["step_size"],
                                         cfg["num_warmup"], cfg["target_accept"])
    np.testing.assert_allclose(g_eps[:cfg["num_warmup"]], da, rtol=1e-4,
                               err_msg=f"{name} chain {chain}: dual averaging")
    np.testing.assert_allclose(g_eps[cfg["num_warmup"]:], eps_bar, rtol=1e-4,
                               err_msg=f"{name} chain {chain}: eps-bar")
    olp, oinit = _model(name, W.ns_oracle())
    ref = S.nuts(olp, oinit, seed=cfg["seed"], chain=chain, step_sizes=g_eps, **{
        k: cfg[k] for k in ("num_warmup", "num_samples", "step_size", "max_tree_depth",
                            "target_accept")})
    rt = {k: np.asarray(v) for k, v in ref.trace.items()}
    gd, gl = tr["tree_depth"][chain], tr["n_leapfrog"][chain]
    h_drift = np.abs(tr["energy"][chain][:n].astype(np.float64) - rt["energy"][:n])
    # the states separate: H0 differs by more than SEP_ULPS ulp (the
    # trajectories amplify rounding differences; in the hierarchical model's
    # funnel they grow exponentially) — the comparison ends there
    D = info.device_samples.shape[-1]
    sep = next((i for i in range(n) if h_drift[i] > SEP_ULPS * _ulp(_hscale(rt["energy"][i], D))),
               n)
    same = _first_flip(gd, gl, rt["depth"], rt["leaves"], sep)
    print(f"{name} chain {chain}: states within {SEP_ULPS} ulp of H0 for {sep} of {n} "
          f"iterations; trees identical for {same}")
    assert same == sep or same >= MIN_REPLAY, f"{name} chain {chain}: compared only {same}"
    if same < sep:
        i = same
        tie = 8 * _ulp(_hscale(rt["energy"][i], D)) + 4 * h_drift[i]
        tie_dot = 1e-5 + 4 * h_drift[i] / max(abs(rt["energy"][i]), 1.0)
        why = (f"{name} chain {chain}: trees differ at iteration {i} (gpu depth {gd[i]} leaves "
               f"{gl[i]}, oracle {rt['depth'][i]} / {rt['leaves'][i]}); oracle margins: slice "
               f"{rt['slice_gap'][i]:.3g}, divergence {rt['div_gap'][i]:.3g}, U-turn "
               f"{rt['uturn_margin'][i]:.3g}; TIE {tie:.3g} / {tie_dot:.3g}")
        print(why)
        assert (rt["slice_gap"][i] <= tie or rt["div_gap"][i] <= tie
                or rt["uturn_margin"][i] <= tie_dot), "not a near-tie: " + why
    # alpha = mean of min(1, exp(H0 - H')): its relative error is that of the
    # exponent, the tie bound of the iteration
    ties = np.array([8 * _ulp(_hscale(rt["energy"][i], D)) + 4 * h_drift[i]
                     for i in range(same)])
    ga = tr["accept_stat"][chain][:same].astype(np.float64)
    ra = np.asarray(rt["alpha"][:same], np.float64)
    bad = np.nonzero(np.abs(ga - ra) > ra * np.expm1(ties) + 1e-6)[0]
    assert bad.size == 0, (f"{name} chain {chain}: alpha at {bad[:5]}: gpu {ga[bad[:5]]} "
                           f"oracle {ra[bad[:5]]} tie {ties[bad[:5]]}")
    ns = max(0, same - cfg["num_warmup"])
    np.testing.assert_allclose(info.device_samples[chain, :ns].cpu().numpy(), ref.samples[:ns],
                               rtol=1e-4, atol=1e-5, err_msg=f"{name} chain {chain}: draws")
    return same, rt["depth"][:same], sep


VARIANTS = {"illcond": ["auto", "spec", "generic", "tape"], "hier": ["auto", "generic", "tape"]}


@pytest.mark.parametrize("name,variant", [(n, v) for n, vs in VARIANTS.items() for v in vs])
def test_nuts_trace_against_oracle(gpu, name, variant):
    C = 64 if name == "illcond" else 8
    fx, info = _gpu_run(name, variant, C)
    cfg = fx["config"]
    n = cfg["num_warmup"] + cfg["num_samples"]
    tr = info.trace
    depths_seen = []
    for j, chain in enumerate(fx["chains"]):
        # the strict replay (two chains per run keep the CPU time small)
        if j < 2 or chain == 5:
            same, depths, _ = _replay(name, fx, info, j, int(chain))
            print(f"{name}/{variant} chain {chain}: replay identical for {same} of {n} "
                  f"iterations, max depth {depths.max() if len(depths) else 0}")
            depths_seen.extend(depths.tolist())
        # the committed trace (the oracle's own adaptation)
        same_fx = _first_flip(tr["tree_depth"][chain], tr["n_leapfrog"][chain], fx["depth"][j],
                              fx["leaves"][j], n)
        i = min(same_fx, n - 1)
        print(f"{name}/{variant} chain {chain}: trees identical to the committed oracle trace "
              f"for {same_fx} of {n} iterations (eps rel. diff there "
              f"{abs(tr['step_size'][chain][i] / fx['step_size'][j][i] - 1):.2e}, oracle slice "
              f"gap {fx['slice_gap'][j][i]:.3g}, U-turn margin {fx['uturn_margin'][j][i]:.3g})")
        assert same_fx >= MIN_SAME, f"chain {chain}: trees diverge from the fixture at {same_fx}"
    assert max(depths_seen) >= 3, "real trees"


@pytest.mark.parametrize("slices,kernel", [(0, "sliced"), (8, "sliced"), (1, "tape")])
def test_nuts_large_shape_against_oracle(gpu, slices, kernel):
    """NUTS on the README "Large" model (D = 1000, N = 100 K; VERDICT r3
    "Next round" 6, r4 "Next round" 1): the sliced kernel k_nuts_sl on the
    automatic plan (16 slices) and on 8 slices, and k_nuts on the tape,
    against the oracle's trace at a fixed step size
    (tests/golden/nuts_large_trace.npz, chains 0-2, depths 7-8): trees
    identical until a near-tie proven by the oracle's own margins (slice /
    divergence gap or relative U-turn dot within the tie bound of the
    iteration), H0 within the tie bound before it, alpha within its relative
    error, stored draws within rtol 1e-4."""
    import mlx_mcmc_amd as m

    fx = _fixture("large")
    cfg = fx["config"]
    lp, init = W.hierarchical(W.ns_product(), *W.SHAPES["large"])
    s, rate, info = m.nuts(lp, init, num_samples=cfg["num_samples"], num_warmup=cfg["num_warmup"],
                           step_size=cfg["step_size"], max_tree_depth=cfg["max_tree_depth"],
                           adapt_step_size=False, target_accept=cfg["target_accept"],
                           key=m.random.key(cfg["seed"]), num_chains=4, progress=False,
                           return_info=True, return_trace=True, keep_on_device=True,
                           num_slices=slices)
    print("large NUTS kernel:", info.extra["kernel"])
    assert info.extra["kernel"] == kernel
    n = cfg["num_warmup"] + cfg["num_samples"]
    tr = info.trace
    D = info.device_samples.shape[-1]
    total = 0
    for j, chain in enumerate(fx["chains"]):
        chain = int(chain)
        gd, gl = tr["tree_depth"][chain], tr["n_leapfrog"][chain]
        np.testing.assert_array_equal(tr["step_size"][chain][:n].astype(np.float32),
                                      np.float32(cfg["step_size"]))
        same = _first_flip(gd, gl, fx["depth"][j], fx["leaves"][j], n)
        h_drift = np.abs(tr["energy"][chain][:n].astype(np.float64) - fx["energy"][j][:n])
        ties = np.array([8 * _ulp(_hscale(fx["energy"][j][i], D)) + 4 * h_drift[i]
                         for i in range(n)])
        print(f"large chain {chain}: trees identical for {same} of {n} iterations, depths "
              f"{fx['depth'][j][:same].tolist()}, H0 drift max {h_drift[:same].max():.3g}")
        if same < n:
            i = same
            tie_dot = 1e-5 + 4 * h_drift[i] / max(abs(fx["energy"][j][i]), 1.0)
            assert (fx["slice_gap"][j][i] <= ties[i] or fx["div_gap"][j][i] <= ties[i]
                    or fx["uturn_margin"][j][i] <= tie_dot), (
                f"chain {chain}: trees differ at {i} without a near-tie (gpu {gd[i]}/{gl[i]}, "
                f"oracle {fx['depth'][j][i]}/{fx['leaves'][j][i]})")
        # H0 of the compared iterations: the positions' fp32 summation order only
        assert np.all(h_drift[:same] <= 1e-5 * (np.abs(fx["energy"][j][:same]) + D)), h_drift
        ga = tr["accept_stat"][chain][:same].astype(np.float64)
        ra = fx["alpha"][j][:same]
        assert np.all(np.abs(ga - ra) <= ra * np.expm1(ties[:same]) + 1e-5), (ga, ra)
        ns = max(0, same - cfg["num_warmup"])
        np.testing.assert_allclose(info.device_samples[chain, :ns].cpu().numpy(),
                                   fx["samples"][j][:ns], rtol=1e-4, atol=1e-5)
        total += same
        assert same >= 6, f"chain {chain}: compared only {same}"
        assert fx["depth"][j][:same].max() >= 7
    print("large NUTS: identical trees over", total, "chain-iterations")


@pytest.mark.parametrize("slices", [0, 8])
def test_nuts_large_dual_averaging_against_oracle(gpu, slices):
    """The Large model with the reference's dual averaging acting (VERDICT r4
    "Next round" 1; tests/golden/nuts_large_da_trace.npz: eps0 = 2e-4, W = 20,
    S = 5, chains 0 and 1) on the sliced kernel: the strict replay (the
    oracle re-runs each chain with the GPU's own step sizes, trees identical
    until a proven near-tie, the GPU's dual averaging recomputed from its own
    acceptance statistics reproduces its step sizes) and the committed trace
    (the oracle's own adaptation) identical for MIN_SAME iterations."""
    import mlx_mcmc_amd as m

    fx = _fixture("large_da")
    cfg = fx["config"]
    lp, init = W.hierarchical(W.ns_product(), *W.SHAPES["large"])
    s, rate, info = m.nuts(lp, init, num_samples=cfg["num_samples"], num_warmup=cfg["num_warmup"],
                           step_size=cfg["step_size"], max_tree_depth=cfg["max_tree_depth"],
                           target_accept=cfg["target_accept"], key=m.random.key(cfg["seed"]),
                           num_chains=4, progress=False, return_info=True, return_trace=True,
                           keep_on_device=True, num_slices=slices)
    assert info.extra["kernel"] == "sliced"
    n = cfg["num_warmup"] + cfg["num_samples"]
    tr = info.trace
    depths = []
    for j, chain in enumerate(fx["chains"]):
        chain = int(chain)
        same, d, sep = _replay("large_da", fx, info, j, chain)
        depths.extend(d.tolist())
        same_fx = _first_flip(tr["tree_depth"][chain], tr["n_leapfrog"][chain], fx["depth"][j],
                              fx["leaves"][j], n)
        print(f"large_da chain {chain}: replay identical for {same} of {n} (states within the "
              f"separation bound for {sep}); committed trace for {same_fx}")
        # the committed trace separates from any other run of the same
        # restatement within a few iterations of eps ~ 4e-3 — the oracle's own
        # at 4 torch threads instead of 1 agrees with it for 3 iterations
        # (chain 0: depths 10, 6, 7, then 4 vs 3; committed as the CPU test
        # test_oracle_pins.py::test_large_dual_averaging_fixture_vs_thread_count):
        # the first 3, which hold the
        # depth-10 tree and the first dual-averaging jump, are pinned; the
        # strict replay above is the comparison beyond them
        assert same_fx >= min(3, sep), f"chain {chain}: trees diverge from the fixture at {same_fx}"
    assert max(depths) >= 5, "real trees"
