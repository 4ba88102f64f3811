"""How many exchange groups (chain blocks) found their slices on one XCD
(sliced.h xcd_agree; mc_debug_workspace_xcd) on the bench shapes."""
import ctypes
import os
import sys
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__)))]
import numpy as np
import torch
import workloads as W
from mlx_mcmc_amd import _engine, _lib, _trace

lib = _lib.load()
for shape in ("large", "medium", "small"):
    G, N = W.SHAPES[shape]
    lp, init = W.hierarchical(W.ns_product(), G, N)
    prog = _trace.compile_model(lp, init)
    cs = _engine.ChainSet(prog, 256, prog.layout.flatten(init), 1e-3, device=torch.device("cuda"))
    cfg = dict(chain_offset=0, num_warmup=10 ** 6, num_samples=0, sample_begin=0,
               sample_capacity=0, seed=0, step_size=1e-3, target_accept=0.8,
               num_leapfrog_steps=20, adapt_step_size=False)
    for k in range(5):
        cs.run_hmc(iter_begin=k, iter_count=1, **cfg)
    torch.cuda.synchronize()
    cs.check_status()
    a, b = ctypes.c_int32(), ctypes.c_int32()
    _lib.check(lib.mc_debug_workspace_xcd(ctypes.c_void_p(cs._ws.data_ptr()), ctypes.byref(a),
                                          ctypes.byref(b)))
    print(f"{shape}: {prog.num_slices} slices, kernel {prog.slice_kernel}: blocks local "
          f"{a.value}, not local {b.value} (5 launches)", flush=True)
