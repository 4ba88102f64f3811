"""Debug: GPU vs oracle posterior moments on the small hierarchical model."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import __graft_entry__ as ge  # noqa: E402

m = ge._ensure_pkg()
import workloads as W  # noqa: E402
import test_gpu_posterior_parity as T  # noqa: E402

np.set_printoptions(precision=4, linewidth=200, suppress=True)
lp, init = W.hierarchical(W.ns_product(), *W.SHAPES["small"])
cfg, ref = T._ref("hmc")
s, rate, info = m.hmc(lp, init, num_samples=cfg["num_samples"], num_warmup=cfg["num_warmup"],
                      step_size=cfg["step_size"], num_leapfrog_steps=cfg["num_leapfrog_steps"],
                      key=m.random.key(0), num_chains=64, progress=False, return_info=True)
x = T._flat(s, init)
g = T._moments(x)
print("rate", np.round(rate, 3)[:16], "eps", np.round(info.step_size, 4)[:16])
for k in ("mean", "var", "mcse_mean"):
    print(k, "gpu", g[k]); print(k, "ref", ref[k])
print("per-chain means of mu", np.round(x[:, :, 0].mean(1), 3))
print("per-chain means of tau", np.round(x[:, :, 1].mean(1), 3))
