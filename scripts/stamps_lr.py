"""Diagnostic: cycles per leapfrog step by section in the lane-resident
sliced kernel (csrc/lanes.h; stamps build, workgroup 0, per wave).
    make -C mlx-mcmc_amd/csrc stamps && python scripts/stamps_lr.py [C] [kernel]"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

ge._ensure_pkg()
from mlx_mcmc_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(ROOT, "scripts", os.environ.get("STAMPS_LIB", "libmcmc355_stamps.so"))
lib = _lib.load()
lib.mc_debug_stamps_lanes.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import workloads as W  # noqa: E402
from mlx_mcmc_amd import _engine, _trace  # noqa: E402

C = int(sys.argv[1]) if len(sys.argv) > 1 else 256
VAR = sys.argv[2] if len(sys.argv) > 2 else "full"
G, N = W.SHAPES["large"]
fn, init = W.hierarchical(W.ns_product(), G, N)
SL = 0
if VAR == "iso100":  # config 2 on the one-slice lane-resident kernel
    fn, init = W.iso_normal(W.ns_product(), 100)
    SL = 1
elif VAR != "full":  # one term family only (diagnostic)
    ns = W.ns_product()
    y, group = W.hierarchical_data(G, N)

    def lik(p):
        return ns.sum(ns.Normal(p["theta"][group], p["sigma"]).log_prob(ns.array(y)))

    def lik_prior(p):
        return lik(p) + ns.sum(ns.Normal(p["mu"], p["tau"]).log_prob(p["theta"]))

    fn = {"lik": lik, "lik_prior": lik_prior}[VAR]
    init = ({"sigma": np.float32(1), "theta": init["theta"]} if VAR == "lik" else
            {"mu": np.float32(1), "tau": np.float32(2), "sigma": np.float32(1),
             "theta": init["theta"]})
prog = _trace.compile_model(fn, init, slices=SL, slice_kernel="lanes")
print(f"variant={VAR} slices={prog.num_slices} kernel={prog.slice_kernel} chains={C}")
cs = _engine.ChainSet(prog, C, prog.layout.flatten(init), 1e-4)
L = 10 if VAR == "iso100" else 20
cfg = dict(chain_offset=0, num_warmup=0, num_samples=10, sample_begin=0, sample_capacity=0,
           seed=1, step_size=1e-4, target_accept=0.8, num_leapfrog_steps=L,
           adapt_step_size=False)
cs.run_hmc(iter_begin=0, iter_count=1, **cfg)
torch.cuda.synchronize()
cs.check_status()
lib.mc_debug_stamps_lanes(None, None, 1)
t = time.perf_counter()
cs.run_hmc(iter_begin=1, iter_count=2, **cfg)
torch.cuda.synchronize()
dt = time.perf_counter() - t
cs.check_status()
acc = (ctypes.c_ulonglong * (16 * 32))()
cnt = (ctypes.c_ulonglong * (16 * 32))()
lib.mc_debug_stamps_lanes(acc, cnt, 0)
a = np.array(acc[:], dtype=np.float64).reshape(16, 32)
c = np.array(cnt[:], dtype=np.float64).reshape(16, 32)
steps = max(c[0, 1], 1)
print(f"2 iterations in {dt * 1e3:.3f} ms ({dt / (2 * L) * 1e6:.2f} us/step incl. launch)")
SECS = [(5, "iteration start (per step)"), (0, "kick+drift"), (1, "evaluation"),
        (7, "scalar terms"), (2, "reductions+publish"), (3, "poll (wait)"), (4, "slice sums+scalar terms"),
        (6, "accept+store (per step)")]
print("  section (cycles/step)         " + " ".join(f"  wave{w}" for w in range(8)))
for sec, name in SECS:
    vals = " ".join(f"{a[w, sec] / steps:7.0f}" for w in range(8))
    print(f"  {name:28s} {vals}")
wg = (ctypes.c_ulonglong * (1024 * 16))()
lib.mc_debug_stamps_lanes_wg.argtypes = [ctypes.c_void_p]
lib.mc_debug_stamps_lanes_wg(wg)
wga = np.array(wg[:], dtype=np.float64).reshape(1024, 16) / steps
# chain block 0's slices (XCD-aware placement: workgroup 8 r holds slice r)
print("  block 0, wave 0, per slice:  eval / publish / poll")
for sl in range(prog.num_slices):
    w = 8 * sl
    print(f"    slice {sl:2d}: {wga[w, 1]:7.0f} {wga[w, 2]:7.0f} {wga[w, 3]:7.0f}")
