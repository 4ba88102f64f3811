"""Posterior moments of long device runs without holding every draw: the
sampler is launched in batches of `batch` sampling iterations into one
[C, batch, D] device buffer (include/mcmc355.h sample_begin /
sample_capacity), and per (chain, batch) the f64 means of x - shift and of
(x - shift)^2 are kept (shift = the first batch's pooled mean, so nothing
cancels).  Moments and their batch-means MCSE follow (the rule of
oracle/diag.py mcse_batch, with batches of `batch` draws).  A run split
into launches gives the same draws as one launch (_engine.ChainSet).
"""
from __future__ import annotations

import numpy as np


def stream_moments(program, algorithm, num_chains, q0, *, step_size, num_warmup, num_samples,
                   batch, seed=0, chain_offset=0, num_leapfrog_steps=10, max_tree_depth=10,
                   adapt_step_size=False, target_accept=0.8):
    import torch

    from mlx_mcmc_amd import _engine

    if num_samples % batch:
        raise ValueError("num_samples must be a multiple of batch")
    C, D = int(num_chains), program.D
    chains = _engine.ChainSet(program, C, q0, step_size)
    dev = chains.device
    cfg = dict(chain_offset=chain_offset, num_warmup=num_warmup, num_samples=num_samples,
               seed=seed, step_size=step_size, target_accept=target_accept,
               adapt_step_size=adapt_step_size)
    if algorithm == "hmc":
        cfg["num_leapfrog_steps"] = num_leapfrog_steps
        launch = chains.run_hmc
    elif algorithm == "nuts":
        cfg["max_tree_depth"] = max_tree_depth
        launch = chains.run_nuts
    else:
        raise ValueError(algorithm)
    launch(samples=None, iter_begin=0, iter_count=num_warmup, sample_begin=0,
           sample_capacity=0, **cfg)
    nb = num_samples // batch
    buf = torch.empty((C, batch, D), dtype=torch.float32, device=dev)
    m1 = torch.empty((C, nb, D), dtype=torch.float64, device=dev)
    m2 = torch.empty((C, nb, D), dtype=torch.float64, device=dev)
    shift = None
    for b in range(nb):
        launch(samples=buf, iter_begin=num_warmup + b * batch, iter_count=batch,
               sample_begin=b * batch, sample_capacity=batch, **cfg)
        x = buf.to(torch.float64)
        if shift is None:
            shift = x.mean(dim=(0, 1))
        x -= shift
        m1[:, b] = x.mean(dim=1)
        m2[:, b] = (x * x).mean(dim=1)
        del x
    torch.cuda.synchronize()
    chains.check_status()
    d = m1.mean(dim=(0, 1))                      # pooled mean - shift
    mean = shift + d
    # per batch: second moment about the pooled mean
    v_b = (m2 - 2.0 * m1 * d + d * d).reshape(-1, D)
    var = v_b.mean(0)
    n = C * nb
    out = {"mean": mean, "var": var,
           "mcse_mean": m1.reshape(-1, D).std(0) / np.sqrt(n),
           "mcse_var": v_b.std(0) / np.sqrt(n)}
    out = {k: v.cpu().numpy() for k, v in out.items()}
    s = chains.scalars()
    out["accept_rate"] = s["n_accept"] / np.maximum(s["n_total"], 1)
    out["step_size"] = s["step_size"].copy()
    out["draws"] = C * num_samples
    if algorithm == "nuts":
        out["mean_tree_depth"] = s["depth_sum"] / num_samples
    return out


def check_within_one_percent(g, exact, *, label, z, tol=0.01, tol_var=None):
    """Per parameter: |mean_gpu - mean| <= max(tol * max(|mean|, sd), z MCSE)
    and |var_gpu - var| <= max(tol_var * var, z MCSE_var), with the effective
    bound printed; the run must be long enough that the MCSE never dominates
    (z MCSE <= the 1 % bound for every parameter), so the check IS "within 1 %".
    `exact` holds the exact moments (no Monte-Carlo error of their own)."""
    tol_var = tol if tol_var is None else tol_var
    mean, var = np.asarray(exact["mean"], np.float64), np.asarray(exact["var"], np.float64)
    sd = np.sqrt(var)
    scale_m = np.maximum(np.abs(mean), sd)
    eff_m = np.maximum(tol * scale_m, z * g["mcse_mean"]) / scale_m
    eff_v = np.maximum(tol_var * var, z * g["mcse_var"]) / var
    rel_m = np.abs(g["mean"] - mean) / scale_m
    rel_v = np.abs(g["var"] - var) / var
    print(f"{label}: {g['draws']} draws per parameter; effective bound max "
          f"{100 * eff_m.max():.3f} % (means, of max(|mean|, sd)), "
          f"{100 * eff_v.max():.3f} % (variances); observed max {100 * rel_m.max():.3f} % / "
          f"{100 * rel_v.max():.3f} %, median {100 * np.median(rel_m):.3f} % / "
          f"{100 * np.median(rel_v):.3f} %; z MCSE max {100 * (z * g['mcse_mean'] / scale_m).max():.3f} % / "
          f"{100 * (z * g['mcse_var'] / var).max():.3f} %")
    assert eff_m.max() <= tol + 1e-12, "run too short: MCSE dominates the mean bound"
    assert eff_v.max() <= tol_var + 1e-12, "run too short: MCSE dominates the variance bound"
    bm = np.nonzero(rel_m > eff_m)[0]
    bv = np.nonzero(rel_v > eff_v)[0]
    assert bm.size == 0, (f"{label}: means of {bm.size} parameters (first {bm[:8]}) "
                          f"off by {rel_m[bm[:8]]} of max(|mean|, sd)")
    assert bv.size == 0, (f"{label}: variances of {bv.size} parameters (first {bv[:8]}) "
                          f"off by {rel_v[bv[:8]]} relative; gpu {g['var'][bv[:8]]} "
                          f"exact {var[bv[:8]]}")
    return eff_m.max(), eff_v.max(), rel_m.max(), rel_v.max()
