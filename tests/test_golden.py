"""Golden fixtures (tests/golden/, made by scripts/gen_golden.py from the oracle).

CPU: the oracle re-derives every fixture, and the fixtures' float32 log
densities agree with their float64 closed forms.
GPU: the HIP path (through the C-ABI) reproduces them — integer work exactly,
floating point within the stated tolerances.
"""
import json
import os

import numpy as np
import pytest

import workloads as W

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLD, name + ".json")) as f:
        return json.load(f)


# ------------------------------- CPU ------------------------------------------
def test_rng_fixture_rederived():
    import scripts.gen_golden as gg

    assert gg.rng_kats() == load("rng_kats")


def test_tape_fixture_rederived_and_closed_form():
    import scripts.gen_golden as gg

    new = gg.tape_kats()
    old = load("tape_kats")
    for name, pts in old.items():
        for a, b in zip(pts, new[name]):
            np.testing.assert_allclose(a["logp_f32"], b["logp_f32"], rtol=1e-6)
            np.testing.assert_allclose(a["grad"], b["grad"], rtol=1e-5, atol=1e-6)
            # f32 restatement vs float64 closed form (tolerance: fp32 summation)
            scale = abs(a["logp_f64"]) + 1
            assert abs(a["logp_f32"] - a["logp_f64"]) <= 2e-7 * scale * np.sqrt(len(a["q"])) + 1e-4


def test_trace_fixtures_rederived():
    import scripts.gen_golden as gg

    h = gg.hmc_simple()
    assert h["accepted"] == load("hmc_simple")["accepted"]
    assert h["eps"] == load("hmc_simple")["eps"]
    n = gg.nuts_illcond()
    assert n["depth"] == load("nuts_illcond")["depth"]
    assert n["leaves"] == load("nuts_illcond")["leaves"]


# ------------------------------- GPU ------------------------------------------
@pytest.mark.gpu
def test_gpu_rng_matches_fixture(gpu):
    import torch

    from mlx_mcmc_amd import _lib

    k = load("rng_kats")
    lib = _lib.load()
    out = torch.empty(4 * k["n"], dtype=torch.int32, device=gpu)
    _lib.check(lib.mc_rng_fill(k["seed"], k["chain"], k["iteration"], k["tag"], k["sub"],
                               k["index0"], k["n"], 0, _lib.ptr(out), _lib.stream_handle()))
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32).reshape(-1, 4),
                                  np.array(k["words"], np.uint32))
    f = torch.empty(4 * k["n"], dtype=torch.float32, device=gpu)
    _lib.check(lib.mc_rng_fill(k["seed"], k["chain"], k["iteration"], k["tag"], k["sub"],
                               k["index0"], k["n"], 1, _lib.ptr(f), _lib.stream_handle()))
    np.testing.assert_array_equal(f.cpu().numpy().reshape(-1, 4),
                                  np.array(k["uniforms"], np.float32))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["simple", "iso", "illcond", "small", "medium"])
def test_gpu_tape_matches_fixture(gpu, name):
    """GPU log p within 2e-6 relative of the float64 closed form (x sqrt(D/100)),
    gradient within rtol 1e-4 of the oracle's autograd gradient."""
    from mlx_mcmc_amd import _engine, _trace

    if name == "simple":
        lp, init = W.simple_normal(W.ns_product())
    elif name == "iso":
        lp, init = W.iso_normal(W.ns_product())
    elif name == "illcond":
        lp, init = W.illcond_normal(W.ns_product())
    else:
        G, N = W.SHAPES[name]
        lp, init = W.hierarchical(W.ns_product(), G, N)
    prog = _trace.compile_model(lp, init)
    pts = load("tape_kats")[name]
    q = np.array([p["q"] for p in pts], np.float32)
    glp, gg = _engine.logp_grad(prog, q)
    glp, gg = glp.cpu().numpy(), gg.cpu().numpy()
    for i, p in enumerate(pts):
        scale = abs(p["logp_f64"]) + 1
        assert abs(glp[i] - p["logp_f64"]) <= 2e-6 * scale * max(1, np.sqrt(len(p["q"]) / 100)) \
            + 1e-4
        rg = np.array(p["grad"])
        np.testing.assert_allclose(gg[i], rg, rtol=1e-4, atol=1e-5 * np.abs(rg).max() + 1e-5)


@pytest.mark.gpu
def test_gpu_hmc_matches_trace_fixture(gpu):
    import mlx_mcmc_amd as m

    h = load("hmc_simple")
    lp, init = W.simple_normal(W.ns_product())
    _, _, info = m.hmc(lp, init, num_samples=h["num_samples"], num_warmup=h["num_warmup"],
                       step_size=h["step_size"], num_leapfrog_steps=h["num_leapfrog_steps"],
                       key=m.random.key(h["seed"]), progress=False, return_info=True,
                       return_trace=True)
    acc = info.trace["accepted"][0].astype(bool).tolist()
    same = next((i for i, (a, b) in enumerate(zip(acc, h["accepted"])) if a != b), len(acc))
    assert same >= 50
    np.testing.assert_array_equal(info.trace["step_size"][0][:same], h["eps"][:same])


@pytest.mark.gpu
def test_gpu_nuts_matches_trace_fixture(gpu):
    import mlx_mcmc_amd as m

    n = load("nuts_illcond")
    lp, init = W.illcond_normal(W.ns_product())
    _, _, info = m.nuts(lp, init, num_samples=n["num_samples"], num_warmup=n["num_warmup"],
                        step_size=n["step_size"], key=m.random.key(n["seed"]), progress=False,
                        return_info=True, return_trace=True)
    d = info.trace["tree_depth"][0].tolist()
    lv = info.trace["n_leapfrog"][0].tolist()
    same = next((i for i in range(len(d)) if d[i] != n["depth"][i] or lv[i] != n["leaves"][i]),
                len(d))
    assert same >= 10


def test_large_trace_fixture_is_mixed():
    """tests/golden/hmc_large_trace.npz (scripts/gen_golden_large.py): the
    oracle's trace at the bench shape mixes accepts and rejects and its
    chains move (the GPU test in test_gpu_large_parity.py relies on it)."""
    fx = np.load(os.path.join(GOLD, "hmc_large_trace.npz"), allow_pickle=False)
    acc = fx["accepted"].astype(bool)
    assert 0.2 < acc.mean() < 0.95
    assert acc[:, :12].any() and not acc[:, :12].all()
    assert np.all(np.ptp(fx["samples"][:, :, 3:], axis=1).max(axis=1) > 0)
    # log U is the shared Philox stream's accept draw (oracle/philox.py)
    from oracle import philox as R

    c = int(fx["chains"][2])
    assert fx["log_u"][2][5] == R.logf_u01(R.uniform(0, c, 5, R.TAG_ACCEPT))


def test_oracle_nuts_fixture_replay_and_dual_averaging():
    """The committed NUTS traces (scripts/gen_golden_nuts.py) are what the
    oracle computes: replaying chain 0 with the recorded step sizes gives the
    same trees, and dual averaging restated from the recorded alphas gives
    the recorded step sizes (the helper the GPU test recomputes the kernel's
    adaptation with)."""
    import json

    from oracle import samplers as S

    fx = np.load(os.path.join(GOLD, "nuts_illcond_trace.npz"), allow_pickle=False)
    cfg = json.loads(str(fx["config"]))
    da, eps_bar = S.dual_averaging_steps(fx["alpha"][0], cfg["step_size"], cfg["num_warmup"],
                                         cfg["target_accept"])
    np.testing.assert_array_equal(da, fx["step_size"][0][:cfg["num_warmup"]])
    assert np.all(fx["step_size"][0][cfg["num_warmup"]:] == eps_bar)
    lp, init = W.illcond_normal(W.ns_oracle())
    r = S.nuts(lp, init, seed=cfg["seed"], chain=int(fx["chains"][0]),
               step_sizes=fx["step_size"][0],
               **{k: cfg[k] for k in ("num_warmup", "num_samples", "step_size", "max_tree_depth",
                                      "target_accept")})
    np.testing.assert_array_equal(r.trace["depth"], fx["depth"][0])
    np.testing.assert_array_equal(r.trace["leaves"], fx["leaves"][0])
    np.testing.assert_array_equal(r.samples, fx["samples"][0])
    assert fx["depth"].max() >= 5


def test_box_muller_and_unit_log_host_bit_exact():
    """The samplers' Box-Muller and uniform log (philox.h mc_box_muller /
    mc_logf_unit: IEEE float32 operations only) on the host build of the same
    code (mc_box_muller_host / mc_logf_unit_host) are bit-identical to the
    oracle's NumPy float32 restatement (oracle/philox.py box_muller /
    logf_unit), edge words included, and within a few ulp of the exact
    transform of the same uniforms."""
    import ctypes

    from mlx_mcmc_amd import _lib
    from oracle import philox as R

    lib = _lib.load()
    rng = np.random.default_rng(5)
    n = 400_000
    w = rng.integers(0, 2 ** 32, size=(n, 2), dtype=np.uint64).astype(np.uint32)
    w[:256, 0] = np.arange(256)                     # u1 at the smallest values
    w[256:512, 0] = 2 ** 32 - 1 - np.arange(256)    # u1 -> 1 (r -> 0)
    w[512:4608, 1] = (np.arange(4096) * (2 ** 32 // 4096)).astype(np.uint32)  # quadrant edges
    out = np.zeros((n, 2), np.float32)
    assert lib.mc_box_muller_host(w.ctypes.data_as(ctypes.c_void_p), n,
                                  out.ctypes.data_as(ctypes.c_void_p)) == 0
    z0, z1 = R.box_muller(w[:, 0], w[:, 1])
    np.testing.assert_array_equal(out[:, 0], z0)
    np.testing.assert_array_equal(out[:, 1], z1)
    # accuracy against the exact transform of the same f32 uniforms
    u1 = R.u01_boxf(w[:, 0]).astype(np.float64)
    u2 = R.u01_boxf(w[:, 1]).astype(np.float64)
    r = np.sqrt(-2.0 * np.log(u1))
    for got, ex in ((z0, r * np.cos(2 * np.pi * u2)), (z1, r * np.sin(2 * np.pi * u2))):
        big = np.abs(ex) > 1e-3
        ulp = np.abs(got[big] - ex[big]) / np.spacing(np.abs(ex[big]).astype(np.float32))
        assert ulp.max() <= 4.0, ulp.max()
    u = R.u01_f32(w[:, 0])
    lg = np.zeros(n, np.float32)
    assert lib.mc_logf_unit_host(u.ctypes.data_as(ctypes.c_void_p), n,
                                 lg.ctypes.data_as(ctypes.c_void_p)) == 0
    np.testing.assert_array_equal(lg, R.logf_unit(u))
    ex = np.log(u.astype(np.float64))
    assert (np.abs(lg - ex) / np.spacing(np.abs(ex).astype(np.float32))).max() <= 1.0
