"""Diagnostic: cycles per leapfrog step by section of the fast-form kernel
k_hmc_lf (csrc/lanes_fast.h; stamps build, s_memtime ticks, workgroup 0 per
wave and wave 0 of every slice of chain block 0).
    make -C mlx-mcmc_amd/csrc stamps && python scripts/stamps_lf.py [shape] [C]"""
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

SHAPE = sys.argv[1] if len(sys.argv) > 1 else "large"
C = int(sys.argv[2]) if len(sys.argv) > 2 else 256
ITERS = int(os.environ.get("STAMPS_ITERS", "20"))
G, N = W.SHAPES[SHAPE]
fn, init = W.hierarchical(W.ns_product(), G, N)
prog = _trace.compile_model(fn, init)
print(f"shape={SHAPE} slices={prog.num_slices} kernel={prog.slice_kernel} fast={prog.lanes_fast} "
      f"chains={C}")
cs = _engine.ChainSet(prog, C, prog.layout.flatten(init), 2e-3)
L = 20
cfg = dict(chain_offset=0, num_warmup=0, num_samples=10, sample_begin=0, sample_capacity=0,
           seed=1, step_size=2e-3, target_accept=0.8, num_leapfrog_steps=L,
           adapt_step_size=False)
# warm the clock (untimed), then one stamped launch
for i in range(40):
    cs.run_hmc(iter_begin=i * 10, iter_count=10, **cfg)
torch.cuda.synchronize()
cs.check_status()
lib.mc_debug_stamps_lanes(None, None, 1)
t = time.perf_counter()
cs.run_hmc(iter_begin=400, iter_count=ITERS, **cfg)
torch.cuda.synchronize()
dt = time.perf_counter() - t
cs.check_status()
acc = (ctypes.c_ulonglong * (16 * 32))()
cnt = (ctypes.c_ulonglong * (16 * 32))()
lib.mc_debug_stamps_lanes(acc, cnt, 0)
a = np.array(acc[:], dtype=np.float64).reshape(16, 32)
c = np.array(cnt[:], dtype=np.float64).reshape(16, 32)
steps = max(c[0, 1], 1)
nw = 8 if prog.num_slices > 8 else (4 if prog.num_slices > 1 else 1)
print(f"{ITERS} iterations in {dt * 1e3:.3f} ms ({dt / (ITERS * L) * 1e6:.3f} us/step incl. launch)")
SECS = [(5, "momentum (per step)"), (0, "first sweep / loop"), (1, "finish + direct"),
        (2, "reduce-scatter + publish"), (8, "drift + sweep"), (7, "first poll round trip"),
        (3, "poll spins"), (4, "slice sums + shared drift"), (6, "accept + store (per step)")]
print("  section (ticks/step)          " + " ".join(f"  wave{w}" for w in range(nw)))
tot = np.zeros(nw)
for sec, name in SECS:
    v = a[:nw, sec] / steps
    tot += v
    print(f"  {name:28s} " + " ".join(f"{x:7.0f}" for x in v))
print(f"  {'total':28s} " + " ".join(f"{x:7.0f}" for x in tot))
print(f"  ticks per us (total / measured step incl. launch): "
      f"{tot.mean() / (dt / (ITERS * L) * 1e6):.0f}")
wg = (ctypes.c_ulonglong * (1024 * 16))()
lib.mc_debug_stamps_lanes_wg.argtypes = [ctypes.c_void_p]
lib.mc_debug_stamps_lanes_wg(wg)
wga = np.array(wg[:], dtype=np.float64).reshape(1024, 16) / steps
S = prog.num_slices
if S > 1:
    # chain block 0's slices (XCD-aware placement: workgroup 8 r holds slice r
    # when the grid is a multiple of 8 blocks), wave 0 of each
    nwg = (C // (2 * nw)) * S
    xcd = nwg % 8 == 0 and (nwg // 8) % S == 0
    print("  block 0, wave 0, per slice: finish / publish / sweep / poll / spins / sums")
    for sl in range(S):
        w = 8 * sl if xcd else sl
        print(f"    slice {sl:2d}: " + " ".join(f"{wga[w, k]:7.0f}" for k in (1, 2, 8, 7, 3, 4)))
    allw = wga[:nwg]
    print("  all workgroups, wave 0: mean / max of sweep, spins: "
          f"{allw[:, 8].mean():.0f} / {allw[:, 8].max():.0f}, {allw[:, 3].mean():.0f} / "
          f"{allw[:, 3].max():.0f}")
