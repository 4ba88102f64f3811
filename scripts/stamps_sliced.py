"""Diagnostic: cycles per leapfrog step by section in the sliced kernel
(stamps build, workgroup 0): 0 position update, 1 slice evaluation,
2 kinetic partial + exchange (publish, wait for all slices, sum).
    make -C mlx-mcmc_amd/csrc stamps && python scripts/stamps_sliced.py [S] [C]"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

ge._ensure_pkg()
from mlx_mcmc_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(ROOT, "scripts", "libmcmc355_stamps.so")
lib = _lib.load()
lib.mc_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import workloads as W  # noqa: E402
from mlx_mcmc_amd import _engine, _trace  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 0
C = int(sys.argv[2]) if len(sys.argv) > 2 else 256
VAR = sys.argv[3] if len(sys.argv) > 3 else "full"
G, N = W.SHAPES["large"]
if len(sys.argv) > 4:
    N = int(sys.argv[4])
fn, init = W.hierarchical(W.ns_product(), G, N)
if VAR != "full":
    ns = W.ns_product()
    y, group = W.hierarchical_data(G, N)

    def lik(p):
        return ns.sum(ns.Normal(p["theta"][group], p["sigma"]).log_prob(ns.array(y)))

    def prior(p):
        return ns.sum(ns.Normal(p["mu"], p["tau"]).log_prob(p["theta"]))

    fn = {"lik": lik, "prior": prior}[VAR]
    init = ({"sigma": np.float32(1), "theta": init["theta"]} if VAR == "lik" else
            {"mu": np.float32(1), "tau": np.float32(2), "theta": init["theta"]})
prog = _trace.compile_model(fn, init, slices=S)
print(f"variant={VAR} N={N} slices={prog.num_slices} chains={C}")
cs = _engine.ChainSet(prog, C, prog.layout.flatten(init), 1e-4)
L = 20
cfg = dict(chain_offset=0, num_warmup=0, num_samples=10, sample_begin=0, sample_capacity=0,
           seed=1, step_size=1e-4, target_accept=0.8, num_leapfrog_steps=L,
           adapt_step_size=False)
cs.run_hmc(iter_begin=0, iter_count=1, **cfg)
torch.cuda.synchronize()
cs.check_status()
lib.mc_debug_stamps(None, None, 1)
t = time.perf_counter()
cs.run_hmc(iter_begin=1, iter_count=2, **cfg)
torch.cuda.synchronize()
dt = time.perf_counter() - t
cs.check_status()
acc = (ctypes.c_ulonglong * (16 * 32))()
cnt = (ctypes.c_ulonglong * (16 * 32))()
lib.mc_debug_stamps(acc, cnt, 0)
a = np.array(acc[:], dtype=np.float64).reshape(16, 32)
c = np.array(cnt[:], dtype=np.float64).reshape(16, 32)
steps = max(c[0, 1], 1)
print(f"2 iterations in {dt * 1e3:.3f} ms ({dt / (2 * L) * 1e6:.2f} us/step incl. launch)")
SECS = [(0, "position update"), (1, "evaluation"), (2, "kinetic+exchange")]
SECS += [(4 + t, f" term {t}") for t in range(5)] + [
    (11, " final sync"), (12, "  term setup"), (13, "  run tables+theta"), (14, "  moments"),
    (15, "  finish+rest of runs"), (16, "  deposits"), (17, " x publish"), (18, " x scalar stage"),
    (19, " x poll"), (20, " x barrier"), (21, " x totals+scalar"), (22, "  load_slterm"),
    (23, "  round start")]
wg = (ctypes.c_ulonglong * (1024 * 4))()
lib.mc_debug_stamps_wg.argtypes = [ctypes.c_void_p]
lib.mc_debug_stamps_wg(wg)
wga = np.array(wg[:], dtype=np.float64).reshape(1024, 4)[: 16 * ((C + 15) // 16)] / steps
for sec, name in ((0, "pos(+hoist)"), (1, "eval"), (2, "collect")):
    v = wga[:, sec]
    print(f"  per-WG {name:12s} min {v.min():7.0f} median {np.median(v):7.0f} max {v.max():7.0f}"
          f"  argmax WG {int(v.argmax())}")
for sec, name in SECS:
    vals = " ".join(f"{a[w, sec] / steps:7.0f}" for w in range(8))
    print(f"  {name:18s} {vals}")
