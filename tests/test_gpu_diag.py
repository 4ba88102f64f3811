"""Device diagnostics (csrc/diag.h) against the oracle.

Parity bars:
  * ESS per series: the reference rule (examples/06_nuts_comparison.py:22-41)
    in f64, rtol 1e-9 against oracle.diag / oracle.samplers.compute_ess —
    including the lag cap (rho ~ 1), short series (n < 4: no lags), constant
    series (var = 0 -> n) and every lag-block boundary;
  * split R-hat: rtol 1e-9 against oracle.diag.split_rhat (BDA3 11.4; parity
    unpinned against the reference, which has none); the sharded two-stage
    reduction (what ranks all-reduce) equals the one-shard result;
  * summary: median / percentiles bit-identical to mcmc.py:191-227's numpy
    calls (exact device order statistics), mean / std within 1e-5 relative
    (numpy accumulates float32 pools in float32, the device in f64);
  * order statistics: NaN pools give NaN, ties, +-0, +-inf, pools of 1e7.
"""
import numpy as np
import pytest

import workloads as W

pytestmark = pytest.mark.gpu


def _ar1(rng, n, rho, mu=0.0):
    e = rng.normal(size=n)
    x = np.empty(n)
    x[0] = e[0]
    for t in range(1, n):
        x[t] = rho * x[t - 1] + e[t]
    return (x + mu).astype(np.float32)


def _dev(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda()


@pytest.mark.parametrize("n", [1, 2, 3, 4, 7, 8, 9, 15, 16, 17, 100, 1001, 5000])
def test_ess_per_series_matches_reference_rule(gpu, n):
    from mlx_mcmc_amd import diagnostics as Dg
    from oracle import samplers as S

    rng = np.random.default_rng(n)
    rhos = [0.0, 0.5, 0.9, 0.99, 0.9995, -0.4]
    C, D = 3, len(rhos) + 1
    x = np.zeros((C, n, D), np.float32)
    for c in range(C):
        for j, rho in enumerate(rhos):
            x[c, :, j] = _ar1(rng, n, rho, mu=10.0 * j)
        x[c, :, -1] = 2.5                         # constant: ESS = n
    got = Dg.ess(_dev(x))
    ref = np.array([[S.compute_ess(x[c, :, d]) for d in range(D)] for c in range(C)])
    np.testing.assert_allclose(got, ref, rtol=1e-9)
    assert np.all(got[:, -1] == n)


def test_compute_ess_one_series(gpu):
    import mlx_mcmc_amd as m
    from oracle import samplers as S

    x = _ar1(np.random.default_rng(3), 3000, 0.8)
    assert abs(m.compute_ess(x) - S.compute_ess(x)) <= 1e-9 * S.compute_ess(x)


def test_split_rhat_and_sharded_reduction(gpu):
    import torch

    from mlx_mcmc_amd import _lib
    from mlx_mcmc_amd import diagnostics as Dg
    from oracle.diag import split_rhat

    rng = np.random.default_rng(5)
    C, S, D = 12, 501, 9
    x = np.stack([np.stack([_ar1(rng, S, 0.6, mu=0.05 * c * (d % 3)) for d in range(D)], -1)
                  for c in range(C)])                                       # [C, S, D]
    d = Dg.chain_diagnostics(_dev(x), group=False)
    ref = np.array([split_rhat(x[:, :, j]) for j in range(D)])
    np.testing.assert_allclose(d["rhat"], ref, rtol=1e-9)
    np.testing.assert_allclose(d["ess_sum"], d["ess"].sum(axis=0), rtol=1e-12)

    # the multi-GPU composition: shards reduce locally, sums are added
    lib = _lib.load()
    st = [Dg.series_stats(_dev(x[a:b])) for a, b in ((0, 5), (5, 12))]
    shp = [(5, S, D), (7, S, D)]
    red = [torch.empty((2, D), dtype=torch.float64, device="cuda") for _ in st]
    for s_, r, (c, _, _) in zip(st, red, shp):
        _lib.check(lib.mc_stats_reduce(c, S, D, _lib.ptr(s_), None, 0, _lib.ptr(r),
                                       _lib.stream_handle()))
    center = (red[0] + red[1])[0].contiguous()
    spread = [torch.empty((2, D), dtype=torch.float64, device="cuda") for _ in st]
    for s_, r, (c, _, _) in zip(st, spread, shp):
        _lib.check(lib.mc_stats_reduce(c, S, D, _lib.ptr(s_), _lib.ptr(center), 2 * C,
                                       _lib.ptr(r), _lib.stream_handle()))
    tot = (spread[0] + spread[1]).contiguous()
    rh = torch.empty(D, dtype=torch.float64, device="cuda")
    _lib.check(lib.mc_rhat(D, 2 * C, S, _lib.ptr(tot), _lib.ptr(rh), _lib.stream_handle()))
    np.testing.assert_allclose(rh.cpu().numpy(), ref, rtol=1e-9)


def test_rhat_requires_four_draws(gpu):
    from mlx_mcmc_amd import diagnostics as Dg

    d = Dg.chain_diagnostics(_dev(np.ones((2, 3, 1))), group=False)
    assert np.isnan(d["rhat"]).all() and np.all(d["ess_sum"] == 6)


def _check_summary(got, ref):
    assert got.keys() == ref.keys()
    for name in ref:
        assert got[name].keys() == ref[name].keys()
        for k, v in ref[name].items():
            if k in ("mean", "std"):
                assert abs(got[name][k] - v) <= 1e-5 * (abs(v) + 1e-3), (name, k)
            else:
                assert got[name][k] == v, (name, k, got[name][k], v)


@pytest.mark.parametrize("method", ["hmc", "nuts"])
def test_mcmc_summary_matches_reference_numpy(gpu, method):
    import mlx_mcmc_amd as m
    from oracle import diag as Od

    G, N = W.SHAPES["small"]
    lp, init = W.hierarchical(W.ns_product(), G, N)
    mc = m.MCMC(lp)
    # (NUTS with slice_mode="exact": on this model the reference's f32 slice
    # rule freezes chains whose dual averaging runs eps up to
    # ~2e4 — the engine reproduces that, tests/test_oracle_pins.py — and a
    # series frozen in every chain has no R-hat)
    kw = (dict(num_leapfrog_steps=8, step_size=0.05) if method == "hmc"
          else dict(step_size=0.05, slice_mode="exact"))
    s = mc.run(init, num_samples=300, num_warmup=200, method=method, random_seed=2,
               verbose=False, num_chains=4, progress=False, **kw)
    for ci in (0.95, 0.8):
        _check_summary(mc.summary(ci), Od.summary(s, ci))
    # the dict path (host arrays uploaded) agrees as well
    from mlx_mcmc_amd import diagnostics as Dg

    _check_summary(Dg.summarize(s), Od.summary(s))
    dg = mc.diagnostics()
    for name in s:
        assert dg[name]["ess"].shape == (4,) + s[name].shape[2:]
        assert np.all(np.isfinite(dg[name]["r_hat"]))


def test_order_statistics_edges(gpu):
    from mlx_mcmc_amd import diagnostics as Dg

    x = np.array([3.0, -0.0, 0.0, np.inf, -np.inf, 1.0, 1.0, -2.5], np.float32)
    got = Dg.order_statistics(_dev(x[None, :, None]), 0, 1, range(len(x)))
    np.testing.assert_array_equal(got, np.sort(x))
    y = x.copy()
    y[3] = np.nan
    got = Dg.order_statistics(_dev(y[None, :, None]), 0, 1, [0, 4, 7])
    assert np.isnan(got).all()
    # a large pool spread over many workgroups, a sub-range of elements
    rng = np.random.default_rng(0)
    z = rng.standard_t(3, size=(4, 250_000, 12)).astype(np.float32)
    sub = np.sort(z[:, :, 3:10].reshape(-1))
    ranks = [0, 1, len(sub) // 2, len(sub) - 2, len(sub) - 1, 12345, 6_999_000, 31]
    got = Dg.order_statistics(_dev(z), 3, 7, ranks)
    np.testing.assert_array_equal(got, sub[ranks])
