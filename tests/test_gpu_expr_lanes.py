"""Expression terms on the sliced lane-resident kernel (csrc/lanes.h LS_EXPR,
element code generated per program by jit.hip gen_lane_term; VERDICT r5
"Next round" 4).  The reference differentiates any MLX expression with
mx.grad (kernels/hmc.py:53-67); GLM likelihoods written out by hand — a
Bernoulli likelihood through mx.sigmoid / mx.log / mx.log1p, two predictors
with a log-scale noise — at N = 100 K observations are sliced over 16
workgroups like the hierarchical bench model, instead of streaming every
observation through one chain-per-workgroup tape per chain.

Bars (as tests/test_gpu_expr.py and tests/test_gpu_large_parity.py):
  * the program is planned onto the lanes and the JIT-compiled lane kernel
    runs (mc_program_expr_jit = 1, no kernel note);
  * HMC decisions / log ratios / H_init / step sizes of chains 0 - 3 equal
    the oracle's (oracle/samplers.py hmc, torch autograd on the same model)
    until a proven near-tie (tests/_near_tie.py, 8 ulp of |H_init|), and the
    stored draws within rtol 1e-3 of the oracle's before it;
  * with the JIT off the same program runs on the tape, bit-identical to the
    unsliced program (num_slices=1) with the JIT off.
"""
import numpy as np
import pytest

import workloads as W
from _near_tie import compare_trace, log_u
from oracle import samplers as S

pytestmark = pytest.mark.gpu

N = 100_000


def _start(model):
    if model == "logistic":
        return W.logistic_regression, {"a": np.float32(-0.3), "b": np.float32(1.1)}
    if model == "huber":
        return W.huber_regression, {"a": np.float32(0.4), "b": np.float32(1.3)}
    x1, x2, y = W.two_predictor_data(N)
    X = np.stack([np.ones(N), x1, x2], 1).astype(np.float64)
    beta, *_ = np.linalg.lstsq(X, y.astype(np.float64), rcond=None)
    res = y - X @ beta
    return W.two_predictor_regression, {
        "a": np.float32(beta[0]), "b1": np.float32(beta[1]), "b2": np.float32(beta[2]),
        "log_sigma": np.float32(np.log(np.std(res)))}


@pytest.mark.parametrize("model,eps,seed", [("logistic", 2e-3, 11), ("two_predictor", 1e-3, 12),
                                            ("huber", 1e-3, 13)])
def test_expr_lanes_hmc_matches_oracle(gpu, model, eps, seed):
    import mlx_mcmc_amd as m
    from mlx_mcmc_amd import _lib, _trace

    f, start = _start(model)
    lp, _ = f(W.ns_product(), N)
    olp, _ = f(W.ns_oracle(), N)
    prog = _trace.compile_model(lp, start)
    assert prog.slice_kernel == "lanes" and prog.num_slices == 16, prog.kernel_note
    kw = dict(num_samples=15, num_warmup=15, step_size=eps, num_leapfrog_steps=10)
    s, rate, info = m.hmc(lp, start, key=m.random.key(seed), num_chains=8, progress=False,
                          return_info=True, return_trace=True, keep_on_device=True, **kw)
    assert info.extra["kernel"] == "lanes" and "kernel_note" not in info.extra
    assert _lib.load().mc_program_expr_jit(prog.handle) == 1
    draws = info.device_samples.cpu().numpy()
    n = 30
    tr = info.trace
    total = 0
    for c in (0, 1, 2, 3):
        ref = S.hmc(olp, start, seed=seed, chain=c, **kw)
        gpu_c = {"accepted": tr["accepted"][c][:n], "ratio": tr["accept_stat"][c][:n],
                 "step_size": tr["step_size"][c][:n], "energy": tr["energy"][c][:n]}
        ref_c = {k: np.asarray(ref.trace[k])[:n] for k in ("accepted", "ratio", "step_size",
                                                           "energy")}
        ref_c["log_u"] = log_u(seed, c, n)
        same = compare_trace(gpu_c, ref_c, f"{model} chain {c}", verbose=True)
        assert same >= 5, f"{model} chain {c}: compared only {same}"
        total += same
        ns = max(0, same - kw["num_warmup"])
        np.testing.assert_allclose(draws[c, :ns], np.asarray(ref.samples)[:ns], rtol=1e-3,
                                   atol=1e-4, err_msg=f"{model} chain {c}")
    # (a proven near-tie may end a chain's comparison early; over four chains
    # most iterations are compared)
    assert total >= 80, f"{model}: compared {total} of 120 chain-iterations"


def test_expr_lanes_without_jit_run_on_the_tape(gpu):
    """mc_debug_expr_jit(0): the lane plan cannot run (its LS_EXPR sweep
    exists only compiled per program), so the launch takes the tape — the
    same bits as the unsliced program on the tape."""
    import mlx_mcmc_amd as m
    from mlx_mcmc_amd import _lib

    lib = _lib.load()
    f, start = _start("logistic")
    lp, _ = f(W.ns_product(), 20_000)
    kw = dict(num_samples=6, num_warmup=4, step_size=5e-3, num_leapfrog_steps=5,
              key=m.random.key(3), num_chains=4, progress=False, return_info=True)
    lib.mc_debug_expr_jit(0)
    try:
        a, _, ia = m.hmc(lp, start, **kw)
        b, _, ib = m.hmc(lp, start, num_slices=1, **kw)
    finally:
        lib.mc_debug_expr_jit(-1)
    assert ia.extra["kernel"] == "unsliced" and ib.extra["kernel"] == "unsliced"
    for k in start:
        np.testing.assert_array_equal(a[k], b[k])
    c, _, ic = m.hmc(lp, start, **kw)
    assert ic.extra["kernel"] == "lanes"
    for k in start:  # (the lane kernel: another summation order, same chain)
        np.testing.assert_allclose(c[k], a[k], rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("model,eps,seed", [("logistic", 2e-3, 21), ("two_predictor", 1e-3, 22)])
def test_expr_lanes_nuts_matches_oracle(gpu, model, eps, seed):
    """NUTS on the sliced kernel (k_nuts_sl's run-time form compiled with the
    program's expression terms: one chain per wave, element pairs packed):
    trees (depth, leaves) identical to the oracle's NUTS (oracle/samplers.py
    nuts, restating nuts.py:137-330) for the first iterations at a fixed step
    size — the oracle sums the 100 K-element log density in another order, so
    the comparison ends at the first tree that differs, which must not come
    before iteration 6 on either chain — and the draws before it within rtol
    1e-3.  With dual averaging acting the run completes on the same kernel."""
    import mlx_mcmc_amd as m
    from mlx_mcmc_amd import _lib, _trace

    f, start = _start(model)
    lp, _ = f(W.ns_product(), N)
    olp, _ = f(W.ns_oracle(), N)
    prog = _trace.compile_model(lp, start)
    assert prog.nuts_kernel(10) == "sliced", prog.kernel_note
    kw = dict(num_samples=8, num_warmup=4, step_size=eps, max_tree_depth=10,
              adapt_step_size=False)
    s, rate, info = m.nuts(lp, start, key=m.random.key(seed), num_chains=8, progress=False,
                           return_info=True, return_trace=True, keep_on_device=True, **kw)
    assert info.extra["kernel"] == "sliced"
    assert _lib.load().mc_program_expr_jit(prog.handle) == 1
    draws = info.device_samples.cpu().numpy()
    n = kw["num_samples"] + kw["num_warmup"]
    tr = info.trace
    for c in (0, 5):
        ref = S.nuts(olp, start, seed=seed, chain=c, **kw)
        same = 0
        for i in range(n):
            if (tr["tree_depth"][c][i] != ref.trace["depth"][i]
                    or tr["n_leapfrog"][c][i] != ref.trace["leaves"][i]):
                break
            same += 1
        print(f"{model} NUTS chain {c}: trees identical for {same} of {n}, depths "
              f"{list(ref.trace['depth'][:same])}")
        assert same >= 6, f"{model} chain {c}: trees differ at iteration {same}"
        ns = max(0, same - kw["num_warmup"])
        np.testing.assert_allclose(draws[c, :ns], np.asarray(ref.samples)[:ns], rtol=1e-3,
                                   atol=1e-4, err_msg=f"{model} NUTS chain {c}")
    # dual averaging acting: the same kernel, moving chains
    s2, rate2, info2 = m.nuts(lp, start, key=m.random.key(seed), num_chains=16, progress=False,
                              return_info=True, num_samples=20, num_warmup=20, step_size=eps)
    assert info2.extra["kernel"] == "sliced"
    assert np.all(info2.mean_tree_depth >= 1)


@pytest.mark.parametrize("model", ["linear_regression", "linear_regression_exp"])
def test_affine_regression_nuts_runs_sliced(gpu, model):
    """NUTS on a linear regression at N = 100 K: its fused affine-loc term
    keeps k_nuts_lr / k_nuts_sl off and would run the tape (k_nuts); nuts()
    runs the same model with that term as an expression term
    (_trace.nuts_program) on the sliced kernel instead.  Trees identical to
    the oracle's for >= 6 iterations on two chains at a fixed step size, the
    draws before the first difference within rtol 1e-3 (as above).
    linear_regression_exp: sigma ~ Exponential(1), a scalar term the sliced
    kernels cannot take as an own prior, rebuilt as an expression term too."""
    import mlx_mcmc_amd as m
    from mlx_mcmc_amd import _lib, _trace

    x, y = W.regression_data(N)
    b, a = np.polyfit(x.astype(np.float64), y.astype(np.float64), 1)
    sd = float(np.std(y - (a + b * x)))
    start = {"a": np.float32(a), "b": np.float32(b), "sigma": np.float32(sd)}
    lp, _ = getattr(W, model)(W.ns_product(), N)
    olp, _ = getattr(W, model)(W.ns_oracle(), N)
    prog = _trace.compile_model(lp, start)
    assert prog.model.n_affines == 1 and prog.nuts_kernel(10) == "tape"
    alt = _trace.nuts_program(prog, 10)
    assert alt is not prog and alt.nuts_kernel(10) == "sliced"
    # with the JIT off the expression form would run interpreted: kept fused
    lib = _lib.load()
    lib.mc_debug_expr_jit(0)
    try:
        assert _trace.nuts_program(prog, 10) is prog
    finally:
        lib.mc_debug_expr_jit(-1)
    kw = dict(num_samples=8, num_warmup=4, step_size=2e-3, max_tree_depth=10,
              adapt_step_size=False)
    s, rate, info = m.nuts(lp, start, key=m.random.key(41), num_chains=8, progress=False,
                           return_info=True, return_trace=True, keep_on_device=True, **kw)
    assert info.extra["kernel"] == "sliced"
    draws = info.device_samples.cpu().numpy()
    n = kw["num_samples"] + kw["num_warmup"]
    tr = info.trace
    for c in (0, 3):
        ref = S.nuts(olp, start, seed=41, chain=c, **kw)
        same = 0
        for i in range(n):
            if (tr["tree_depth"][c][i] != ref.trace["depth"][i]
                    or tr["n_leapfrog"][c][i] != ref.trace["leaves"][i]):
                break
            same += 1
        print(f"{model} NUTS chain {c}: trees identical for {same} of {n}, depths "
              f"{list(ref.trace['depth'][:same])}")
        assert same >= 6, f"chain {c}: trees differ at iteration {same}"
        ns = max(0, same - kw["num_warmup"])
        np.testing.assert_allclose(draws[c, :ns], np.asarray(ref.samples)[:ns], rtol=1e-3,
                                   atol=1e-4, err_msg=f"affine regression NUTS chain {c}")


@pytest.mark.parametrize("model,scale,seed", [("logistic", 4e-3, 31), ("huber", 3e-3, 32)])
def test_expr_lanes_mh_matches_oracle(gpu, model, scale, seed):
    """Random-walk MH (metropolis.py:6-101, the MCMC.run default) on the
    sliced kernel k_mh_sl's run-time form compiled with the expression terms
    (value only): the same proposals as the oracle, decisions equal until a
    proven near-tie (8 ulp of |log p|), log p and draws before it."""
    import mlx_mcmc_amd as m
    from mlx_mcmc_amd import _lib, _trace
    from _near_tie import tie_bound

    f, start = _start(model)
    lp, _ = f(W.ns_product(), N)
    olp, _ = f(W.ns_oracle(), N)
    prog = _trace.compile_model(lp, start)
    assert _lib.load().mc_program_mh_sliced(prog.handle) == 1, prog.kernel_note
    n = 60
    s, rate, info = m.metropolis_hastings(lp, start, num_samples=n, proposal_scale=scale,
                                          random_seed=seed, return_info=True,
                                          return_trace=True, keep_on_device=True)
    ref = S.metropolis_hastings(olp, start, num_samples=n, proposal_scale=scale,
                                random_seed=seed)
    acc = info.trace["accepted"][0].astype(bool)
    racc = np.array(ref.trace["accepted"])
    assert 0 < racc.sum() < n, "mixed decisions"
    flips = np.nonzero(acc != racc)[0]
    same = int(flips[0]) if flips.size else n
    print(f"{model} MH: decisions identical for {same} of {n}")
    if same < n:
        lu = log_u(m.random.key(seed).seed, 0, n)
        tie = tie_bound(ref.trace["logp"][same])
        gap = abs(float(lu[same]) - ref.trace["ratio"][same])
        assert gap <= tie, f"flip at {same} is not a near-tie: gap {gap} > {tie}"
    assert same >= 20
    np.testing.assert_allclose(info.trace["energy"][0][:same], ref.trace["logp"][:same],
                               rtol=2e-6)
    draws = info.device_samples[0].cpu().numpy()
    np.testing.assert_allclose(draws[:same], np.asarray(ref.samples)[:same], rtol=1e-5,
                               atol=1e-6)


@pytest.mark.parametrize("model", ["linear_regression", "linear_regression_exp"])
def test_affine_regression_mh_runs_sliced(gpu, model):
    """Random-walk MH on the N = 100 K linear regression: the fused affine
    term keeps k_mh_sl off; metropolis_hastings() runs the model with it as an
    expression term (_trace.mh_program) on the sliced kernel.  Decisions equal
    the oracle's until a proven near-tie, log p and draws before it (the bars
    of test_expr_lanes_mh_matches_oracle)."""
    import mlx_mcmc_amd as m
    from mlx_mcmc_amd import _lib, _trace
    from _near_tie import tie_bound

    x, y = W.regression_data(N)
    b, a = np.polyfit(x.astype(np.float64), y.astype(np.float64), 1)
    sd = float(np.std(y - (a + b * x)))
    start = {"a": np.float32(a), "b": np.float32(b), "sigma": np.float32(sd)}
    lp, _ = getattr(W, model)(W.ns_product(), N)
    olp, _ = getattr(W, model)(W.ns_oracle(), N)
    lib = _lib.load()
    prog = _trace.compile_model(lp, start)
    assert lib.mc_program_mh_sliced(prog.handle) == 0
    mp = _trace.mh_program(prog)  # (kept alive while its handle is queried)
    assert lib.mc_program_mh_sliced(mp.handle) == 1
    n, scale, seed = 60, 2e-3, 42
    s, rate, info = m.metropolis_hastings(lp, start, num_samples=n, proposal_scale=scale,
                                          random_seed=seed, return_info=True,
                                          return_trace=True, keep_on_device=True)
    ref = S.metropolis_hastings(olp, start, num_samples=n, proposal_scale=scale,
                                random_seed=seed)
    acc = info.trace["accepted"][0].astype(bool)
    racc = np.array(ref.trace["accepted"])
    assert 0 < racc.sum() < n, "mixed decisions"
    flips = np.nonzero(acc != racc)[0]
    same = int(flips[0]) if flips.size else n
    print(f"{model} MH: decisions identical for {same} of {n}")
    if same < n:
        lu = log_u(m.random.key(seed).seed, 0, n)
        tie = tie_bound(ref.trace["logp"][same])
        gap = abs(float(lu[same]) - ref.trace["ratio"][same])
        assert gap <= tie, f"flip at {same} is not a near-tie: gap {gap} > {tie}"
    assert same >= 20
    np.testing.assert_allclose(info.trace["energy"][0][:same], ref.trace["logp"][:same],
                               rtol=2e-6)
    draws = info.device_samples[0].cpu().numpy()
    np.testing.assert_allclose(draws[:same], np.asarray(ref.samples)[:same], rtol=1e-5,
                               atol=1e-6)
