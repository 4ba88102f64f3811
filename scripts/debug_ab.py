"""Debug: A/B-testing model (only scalar Beta terms) on k_hmc vs one-slice lanes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import __graft_entry__ as ge  # noqa: E402

m = ge._ensure_pkg()
import workloads as W  # noqa: E402

np.set_printoptions(precision=6, linewidth=160)
lp, init = W.ab_testing(W.ns_product())
for slices, kernel in ((1, "auto"), (1, "lanes")):
    s, rate, info = m.hmc(lp, init, num_samples=4, num_warmup=2, step_size=0.01,
                          num_leapfrog_steps=10, key=m.random.key(0), num_chains=2,
                          progress=False, return_info=True, return_trace=True,
                          num_slices=slices, slice_kernel=kernel)
    print(kernel, "pA", s["p_A"][:, :6], "pB", s["p_B"][:, :6])
    for k in ("accepted", "accept_stat", "energy", "step_size"):
        print("  ", k, np.asarray(info.trace[k])[:, :6])
