"""Throughput of the other BASELINE.json configs (not the headline bench line):
config 2 (100-dim isotropic Normal, HMC L=10, 64 chains) and config 5 (NUTS
depth 10 + dual averaging on the 100-dim kappa=1000 Gaussian, 64 chains per
GPU = 512 over 8).  Prints one JSON object; leapfrog steps count every leaf
built."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    import __graft_entry__ as ge

    m = ge._ensure_pkg()
    import workloads as W

    out = {}
    # config 2, automatic (one-slice lane-resident kernel) and on k_hmc (num_slices=1)
    lp, init = W.iso_normal(W.ns_product(), 100)
    for label, slices, kernel in (("", 0, "auto"), ("_k_hmc", 1, "auto")):
        t = time.perf_counter()
        s, rate, info = m.hmc(lp, init, num_samples=1000, num_warmup=1000, step_size=0.1,
                              num_leapfrog_steps=10, key=m.random.key(0), num_chains=64,
                              progress=False, return_info=True, num_slices=slices,
                              slice_kernel=kernel)
        wall = time.perf_counter() - t
        steps = 64 * 2000 * 10
        x = s["x"]
        rate_s = 64 * 1000 * 10 / info.sampling_seconds
        out["config2_iso100_hmc" + label] = {
            "chains": 64,
            # F = 16 D flops per chain-leapfrog-step (the direct Normal term
            # 10 D, kicks and drift 6 D) against the FP32 vector peak; 64
            # chains are 32 waves on 1024 SIMDs: latency-bound
            "fp32_roofline_frac": rate_s * 16 * 100 / 157.3e12,
            "leapfrog_steps_per_s": steps / (info.warmup_seconds + info.sampling_seconds),
            "sampling_steps_per_s": 64 * 1000 * 10 / info.sampling_seconds,
            "wall_s": wall, "accept_rate": float(np.mean(rate)),
            "mean_abs_mean": float(np.abs(x.mean(axis=(0, 1))).mean()),
            "mean_var": float(x.var(axis=(0, 1)).mean())}
    # config 5
    lp, init = W.illcond_normal(W.ns_product(), 100)
    t = time.perf_counter()
    s, rate, info = m.nuts(lp, init, num_samples=1000, num_warmup=1000, step_size=0.1,
                           max_tree_depth=10, key=m.random.key(0), num_chains=64,
                           progress=False, return_info=True)
    wall = time.perf_counter() - t
    leaves = float(np.sum(info.n_grad))
    sc = W.illcond_scales(100)
    x = s["x"]
    out["config5_illcond_nuts"] = {
        "chains": 64, "leaf_steps_per_s": leaves / (info.warmup_seconds + info.sampling_seconds),
        "wall_s": wall, "accept_rate": float(np.mean(rate)),
        "mean_tree_depth": float(np.mean(info.mean_tree_depth)),
        "rel_var_err_median": float(np.median(np.abs(x.var(axis=(0, 1)) / sc ** 2 - 1)))}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
