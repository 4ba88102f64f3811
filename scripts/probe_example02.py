"""Diagnostic: example 02's HMC run (examples/02_hmc_comparison.py:86-100,
seed 42) on many chains on the GPU; per-chain statistics of the example's own
helpers -> gpurun_out/example02_gpu.json."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import __graft_entry__ as ge  # noqa: E402

m = ge._ensure_pkg()
import workloads as W  # noqa: E402


def ess02_batch(x):
    """examples/02_hmc_comparison.py:111-128 over the columns of x [n, m]."""
    x = np.asarray(x, np.float64)
    n, k = x.shape
    mean = x.mean(0)
    c0 = ((x - mean) ** 2).mean(0)
    xc = x - mean
    acf_sum = np.zeros(k)
    active = np.ones(k, bool)
    for lag in range(1, min(n // 2, 100)):
        c = np.mean(xc[:-lag] * xc[lag:], axis=0) / c0
        acf_sum = np.where(active, acf_sum + c, acf_sum)
        if lag > 1:
            active = active & ~(c < 0.05)
        if not active.any():
            break
    return n / (1 + 2 * acf_sum)


C = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
lp, init = W.simple_normal(W.ns_product())
s, rate, info = m.hmc(lp, init, num_samples=5000, num_warmup=1000, step_size=0.1,
                      num_leapfrog_steps=10, adapt_step_size=True, target_accept=0.8,
                      key=m.random.key(42), num_chains=C, progress=False, return_info=True)
mu, sg = np.asarray(s["mu"]), np.asarray(s["sigma"])     # [C, S]
out = {"accept_rate": np.asarray(info.accept_rate).tolist(),
       "step_size": np.asarray(info.step_size).tolist(),
       "ess_mu": ess02_batch(mu.T).tolist(), "ess_sigma": ess02_batch(sg.T).tolist(),
       "err_mu": np.abs(mu.astype(np.float64).mean(1) - 5).tolist(),
       "err_sigma": np.abs(sg.astype(np.float64).mean(1) - 2).tolist()}
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "example02_gpu.json"), "w"))
for k, v in out.items():
    v = np.asarray(v)
    print(k, "quantiles 0/10/50/90/100:", np.quantile(v, [0, .1, .5, .9, 1]).round(5))
