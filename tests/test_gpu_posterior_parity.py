"""Posterior parity against the reference restatement (SURVEY 8(d) "Parity").

Per parameter, |mean_gpu - mean_ref| <= max(1 % of |mean_ref|, k MCSE) and
the same for the variance (k = 3, Bonferroni-widened to 4.42 for the
1000-parameter model: z_bound), with the MCSE of both runs combined (batch means,
20 batches per chain: oracle/diag.py mcse_batch — the reference's
autocorrelation ESS rule breaks down on antithetic HMC draws).  The reference side is the CPU oracle's
HMC (hmc.py:7-206) on the small hierarchical shape at a fixed step size and
its Metropolis-Hastings (metropolis.py:6-101) on example 01's model (8 and 4
chains), held as moments in tests/golden/posterior_small.json
(scripts/gen_posterior.py says why the step size is fixed).  The GPU runs the
same sampler settings on 64 chains through the product API (HMC on the
lane-resident kernel, MH on k_mh).
"""
import json
import os

import numpy as np
import pytest

import workloads as W

pytestmark = pytest.mark.gpu

FIXTURE = os.path.join(os.path.dirname(__file__), "golden", "posterior_small.json")


def _ref(kind):
    with open(FIXTURE) as f:
        fx = json.load(f)
    return fx[kind], {k: np.asarray(v) for k, v in fx[kind + "_moments"].items()}


def _flat(samples, init):
    """Product samples {name: [C, S, *shape]} -> [C, S, D] in layout order."""
    C, S = np.asarray(samples[next(iter(init))]).shape[:2]
    return np.concatenate([np.asarray(samples[k], np.float64).reshape(C, S, -1) for k in init],
                          axis=2)


def _moments(x):
    from oracle.diag import mcse_batch

    pooled = x.reshape(-1, x.shape[-1])
    mcse_m, mcse_v = mcse_batch(x)
    return {"mean": pooled.mean(0), "var": pooled.var(0), "mcse_mean": mcse_m,
            "mcse_var": mcse_v}


def z_bound(n_params):
    """SURVEY 8(d)'s 3 MCSE, widened for multiplicity: with 2 n_params
    comparisons (means and variances) the bound is the normal quantile that
    keeps the family-wise false-failure rate at 1 % (Bonferroni): 3.0 for the
    small models, 4.42 at D = 1000 — where 3 MCSE would fail ~5 of 2000
    comparisons of identical distributions by chance."""
    from scipy.stats import norm

    return max(3.0, float(norm.ppf(1.0 - 0.01 / (2.0 * 2 * n_params))))


def _check(g, r):
    k = z_bound(len(r["mean"]))
    tol_m = np.maximum(0.01 * np.abs(r["mean"]),
                       k * np.hypot(g["mcse_mean"], r["mcse_mean"]))
    tol_v = np.maximum(0.01 * r["var"], k * np.hypot(g["mcse_var"], r["mcse_var"]))
    dm = np.abs(g["mean"] - r["mean"])
    dv = np.abs(g["var"] - r["var"])
    bm = np.nonzero(dm > tol_m)[0]
    bv = np.nonzero(dv > tol_v)[0]
    assert bm.size == 0, (f"means of {bm.size} parameters (first {bm[:8]}): gpu "
                          f"{g['mean'][bm[:8]]} ref {r['mean'][bm[:8]]} tol {tol_m[bm[:8]]}")
    assert bv.size == 0, (f"variances of {bv.size} parameters (first {bv[:8]}): gpu "
                          f"{g['var'][bv[:8]]} ref {r['var'][bv[:8]]} tol {tol_v[bv[:8]]} "
                          f"mcse gpu {g['mcse_var'][bv[:8]]} ref {r['mcse_var'][bv[:8]]}")


def test_hmc_posterior_matches_oracle_small_hierarchical(gpu):
    import mlx_mcmc_amd as m

    cfg, ref = _ref("hmc")
    lp, init = W.hierarchical(W.ns_product(), *W.SHAPES["small"])
    s, rate = m.hmc(lp, init, num_samples=cfg["num_samples"], num_warmup=cfg["num_warmup"],
                    step_size=cfg["step_size"], num_leapfrog_steps=cfg["num_leapfrog_steps"],
                    adapt_step_size=cfg["adapt_step_size"], key=m.random.key(0), num_chains=64,
                    progress=False)
    _check(_moments(_flat(s, init)), ref)


def test_mh_posterior_matches_oracle_example01(gpu):
    import mlx_mcmc_amd as m

    cfg, ref = _ref("mh")
    lp, init = W.simple_normal(W.ns_product())
    s, rate = m.metropolis_hastings(lp, init, num_samples=cfg["num_samples"],
                                    proposal_scale=cfg["proposal_scale"], random_seed=0,
                                    num_chains=64)
    _check(_moments(_flat(s, init)), ref)


# ---- the bench's own shape (BASELINE configs[2]: D = 1000, N = 100 K) -------
FIXTURE_LARGE = os.path.join(os.path.dirname(__file__), "golden", "posterior_large.json")


def _moments_device(x):
    """_moments of a [C, S, D] device tensor, computed on the device in f64
    (the same batch-means rule as oracle/diag.py mcse_batch, 20 batches per
    chain): the 256-chain run holds 2 GB of draws."""
    import torch

    x = x.to(torch.float64)
    C, S, D = x.shape
    nb = 20
    b = S // nb
    mean = x.mean(dim=(0, 1))
    var = ((x - mean) ** 2).mean(dim=(0, 1))
    xb = x[:, :b * nb].reshape(C, nb, b, D)
    m1 = xb.mean(2).reshape(-1, D)
    m2 = ((xb - mean) ** 2).mean(2).reshape(-1, D)
    n = C * nb
    out = {"mean": mean, "var": var, "mcse_mean": m1.std(0) / np.sqrt(n),
           "mcse_var": m2.std(0) / np.sqrt(n)}
    return {k: v.cpu().numpy() for k, v in out.items()}


def _ref_large():
    with open(FIXTURE_LARGE) as f:
        fx = json.load(f)
    return fx["hmc"], {k: np.asarray(v) for k, v in fx["hmc_moments"].items()}


def test_hmc_posterior_matches_oracle_large(gpu):
    """north_star's "posterior moments within 1 % of reference" at the
    1000-parameter / 100 K-observation model, through the bench kernel
    (k_hmc_lr, 16 slices): the oracle's 16 chains at fixed eps = 2e-3
    (tests/golden/posterior_large.json, scripts/gen_golden_large.py) against 64
    independent GPU chains (ids 1000..1063) with the same settings; SURVEY
    8(d)'s rule per parameter for means and variances."""
    import mlx_mcmc_amd as m

    cfg, ref = _ref_large()
    lp, init = W.hierarchical(W.ns_product(), *W.SHAPES["large"])
    s, rate, info = m.hmc(lp, init, num_samples=cfg["num_samples"],
                          num_warmup=cfg["num_warmup"], step_size=cfg["step_size"],
                          num_leapfrog_steps=cfg["num_leapfrog_steps"],
                          adapt_step_size=cfg["adapt_step_size"], key=m.random.key(0),
                          num_chains=64, chain_offset=1000, progress=False, return_info=True,
                          keep_on_device=True)
    assert np.all(info.accept_rate > 0.5)
    _check(_moments_device(info.device_samples), ref)


def test_hmc_posterior_adapted_large(gpu):
    """The reference's warmup rule on the bench's launch: 256
    chains from eps0 = 3e-3, W = 300, S = 2000.  The rule leaves some chains
    at a step size past stability where they never accept again (the oracle's
    16 chains: 2 such, tests/golden/posterior_large_adapt.json); those are
    excluded, the others' pooled moments must match the fixed-eps oracle
    posterior by the same rule: the adapted sampler targets the same
    distribution."""
    import mlx_mcmc_amd as m

    _, ref = _ref_large()
    with open(os.path.join(os.path.dirname(__file__), "golden", "posterior_large_adapt.json")) as f:
        ad = json.load(f)["hmc"]
    lp, init = W.hierarchical(W.ns_product(), *W.SHAPES["large"])
    s, rate, info = m.hmc(lp, init, num_samples=ad["num_samples"], num_warmup=ad["num_warmup"],
                          step_size=ad["step_size"], num_leapfrog_steps=ad["num_leapfrog_steps"],
                          adapt_step_size=True, key=m.random.key(0), num_chains=256,
                          progress=False, return_info=True, keep_on_device=True)
    moving = info.accept_rate > 0
    frozen_oracle = sum(a == 0 for a in ad["accept_rate"]) / len(ad["accept_rate"])
    frozen_gpu = 1 - moving.mean()
    print(f"frozen chains: GPU {frozen_gpu:.3f} of 256, oracle {frozen_oracle:.3f} of 16")
    assert frozen_gpu < 0.5 and moving.sum() >= 64
    import torch

    idx = torch.from_numpy(np.nonzero(moving)[0]).to(info.device_samples.device)
    _check(_moments_device(info.device_samples.index_select(0, idx)), ref)
