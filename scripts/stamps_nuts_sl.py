"""Diagnostic: cycles per leaf by section in k_nuts_sl (stamps build,
workgroup 0: the chains of chain block 0 in slice 0, one per wave).  The
README "Large" hierarchical model, 256 chains, the bench's NUTS line (20
dual-averaging iterations from eps0 = 2e-3, then 10 measured ones).
    make -C mlx-mcmc_amd/csrc stamps && python scripts/stamps_nuts_sl.py [slices]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

ge._ensure_pkg()
from mlx_mcmc_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(ROOT, "scripts", os.environ.get("STAMPS_LIB", "libmcmc355_stamps.so"))
lib = _lib.load()
lib.mc_debug_stamps_nuts_sl.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import workloads as W  # noqa: E402
from mlx_mcmc_amd import _engine, _trace  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 8
C = int(os.environ.get("CHAINS", "256"))
fn, init = W.hierarchical(W.ns_product(), *W.SHAPES["large"])
prog = _trace.compile_model(fn, init, slices=S)
assert prog.nuts_kernel(10) == "sliced"
cs = _engine.ChainSet(prog, C, prog.layout.flatten(init), 2e-3)
cfg = dict(chain_offset=0, num_warmup=20, num_samples=10, sample_begin=0, sample_capacity=0,
           seed=0, step_size=2e-3, target_accept=0.8, max_tree_depth=10, adapt_step_size=True,
           slice_mode=0)
cs.run_nuts(iter_begin=0, iter_count=20, **cfg)
torch.cuda.synchronize()
lib.mc_debug_stamps_nuts_sl(None, None, 1)
n0 = cs.scalars()["n_grad"].copy()
cs.run_nuts(iter_begin=20, iter_count=10, **cfg)
torch.cuda.synchronize()
cs.check_status()
leaves = (cs.scalars()["n_grad"] - n0)[:8]
acc = (ctypes.c_ulonglong * (16 * 32))()
cnt = (ctypes.c_ulonglong * (16 * 32))()
lib.mc_debug_stamps_nuts_sl(acc, cnt, 0)
a = np.array(acc[:], dtype=np.float64).reshape(16, 32)
c = np.array(cnt[:], dtype=np.float64).reshape(16, 32)
print(f"slices {S}; leaves (chains 0-7):", leaves)
SECS = [(14, "iteration start"), (0, "leapfrog + derive (+ sweep)"), (1, "finish + record"),
        (2, "publish + park (private)"), (8, "sweep-ahead"), (3, "poll wait"),
        (10, "totals + decisions + park"), (12, "merges + U-turns"), (13, "top level"),
        (15, "iteration end")]
print("  section (cycles per leaf)        " + " ".join(f" chain{w}" for w in range(8)))
for sec, name in SECS:
    vals = " ".join(f"{a[w, sec] / max(leaves[w], 1):7.0f}" for w in range(8))
    print(f"  {name:32s} {vals}")
tot = [a[w, :16].sum() / max(leaves[w], 1) for w in range(8)]
print("  total                            " + " ".join(f"{t:7.0f}" for t in tot))
