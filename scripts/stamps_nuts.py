"""Diagnostic: cycles per NUTS leaf by section in k_nuts (stamps build,
workgroup 0, one chain per wave).  Config 5: kappa = 1000 100-dim Gaussian,
64 chains, depth 10.
    make -C mlx-mcmc_amd/csrc stamps && python scripts/stamps_nuts.py"""
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
lib.mc_debug_stamps_nuts.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import workloads as W  # noqa: E402
from mlx_mcmc_amd import _engine, _trace  # noqa: E402

C = 64
fn, init = W.illcond_normal(W.ns_product(), 100)
prog = _trace.compile_model(fn, init)
cs = _engine.ChainSet(prog, C, prog.layout.flatten(init), 0.1)
cfg = dict(chain_offset=0, num_warmup=200, num_samples=100, sample_begin=0, sample_capacity=0,
           seed=0, step_size=0.1, target_accept=0.8, max_tree_depth=10, adapt_step_size=True,
           slice_mode=0)
cs.run_nuts(iter_begin=0, iter_count=200, **cfg)   # warm up the step size
torch.cuda.synchronize()
lib.mc_debug_stamps_nuts(None, None, 1)
n0 = cs.scalars()["n_grad"].copy()
cs.run_nuts(iter_begin=200, iter_count=20, **cfg)
torch.cuda.synchronize()
leaves = (cs.scalars()["n_grad"] - n0)[:4]
acc = (ctypes.c_ulonglong * (16 * 32))()
cnt = (ctypes.c_ulonglong * (16 * 32))()
lib.mc_debug_stamps_nuts(acc, cnt, 0)
a = np.array(acc[:], dtype=np.float64).reshape(16, 32)
c = np.array(cnt[:], dtype=np.float64).reshape(16, 32)
print("leaves (chains 0-3):", leaves)
SECS = [(14, "iteration start"), (8, "leapfrog r/q"), (9, "gradient tape"), (10, "kinetic+decisions"),
        (11, "park candidate"), (12, "merges + U-turns"), (13, "top level"), (15, "iteration end")]
print("  section (cycles per leaf)      " + " ".join(f"  chain{w}" for w in range(4)))
for sec, name in SECS:
    vals = " ".join(f"{a[w, sec] / max(leaves[w], 1):8.0f}" for w in range(4))
    print(f"  {name:28s} {vals}")
print("  inside the tape: g zero + sync_before (2) / term 0 (3) / lp flush + sync (18) / finalize (19); in term: preamble (20) / element loop (21) / finish + flush (22)")
for sec in (2, 3, 18, 19, 20, 21, 22):
    vals = " ".join(f"{a[w, sec] / max(leaves[w], 1):8.0f}" for w in range(4))
    print(f"  tape section {sec:<15d} {vals}")
tot = [a[w, 8:16].sum() / max(leaves[w], 1) for w in range(4)]
print("  total                        " + " ".join(f"{t:8.0f}" for t in tot))
