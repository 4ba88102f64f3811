"""Diagnostic: per-section cycle shares inside one leapfrog step (stamps build).

Loads scripts/libmcmc355_stamps.so (make -C mlx-mcmc_amd/csrc stamps) in place
of the product library; reads wave 0 of workgroup 0's s_memtime accumulators.
Sections: 0 position update, 1 whole evaluation, 2k/2k+1 term k start/end,
18 lp slot + barrier, 19 finalize."""
import ctypes
import os
import sys

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

sys.path.insert(0, os.path.join(ROOT, "scripts"))
from probe_eval import variants  # noqa: E402  (runs its own timing first)
from mlx_mcmc_amd import _engine, _trace  # noqa: E402

NAMES = {0: "position update+sync", 1: "evaluation total", 18: "lp slot+barrier",
         19: "finalize+barrier"}
for name, fn, init in variants():
    prog = _trace.compile_model(fn, init)
    cs = _engine.ChainSet(prog, 256, prog.layout.flatten(init), 1e-4)
    cfg = dict(chain_offset=0, num_warmup=0, num_samples=10, sample_begin=0, sample_capacity=0,
               seed=1, step_size=1e-4, target_accept=0.8, num_leapfrog_steps=20,
               adapt_step_size=False)
    cs.run_hmc(iter_begin=0, iter_count=1, **cfg)
    torch.cuda.synchronize()
    lib.mc_debug_stamps(None, None, 1)
    cs.run_hmc(iter_begin=1, iter_count=2, **cfg)
    torch.cuda.synchronize()
    acc = (ctypes.c_ulonglong * (16 * 32))()
    cnt = (ctypes.c_ulonglong * (16 * 32))()
    lib.mc_debug_stamps(acc, cnt, 0)
    a = np.array(acc[:], dtype=np.float64).reshape(16, 32)
    c = np.array(cnt[:], dtype=np.float64).reshape(16, 32)
    W = prog.waves_per_chain
    steps = max(c[0, 1], 1)
    print(f"== {name} (wpc={W}, {int(steps)} leapfrog steps recorded; cycles/step per wave)")
    for sec in range(32):
        if c[0, sec]:
            label = NAMES.get(sec, f"term {(sec - 2) // 2} {'pre' if sec % 2 == 0 else 'body'}")
            vals = " ".join(f"{a[w, sec] / steps:7.0f}" for w in range(W))
            print(f"   {label:22s} {vals}")
