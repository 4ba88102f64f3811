"""Find where a NUTS Large chain leaves the posterior (the bench's balance
probe saw one chain at sigma ~ 3e6): warmup one iteration per launch, the
chain's (mu, tau, sigma), step size, tree depth and energy per iteration."""
import os
import sys
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__)))]
import numpy as np
import torch
import workloads as W
from mlx_mcmc_amd import _engine, _trace

C, WM = 256, int(os.environ.get("WARMUP", "500"))
CH = int(os.environ.get("CHAIN", "24"))
G, N = W.SHAPES["large"]
lp, init = W.hierarchical(W.ns_product(), G, N)
prog = _trace.compile_model(lp, init, slices=16)
eps0 = 6.1458e-4
cs = _engine.ChainSet(prog, C, prog.layout.flatten(init), eps0, device=torch.device("cuda"))
cfg = dict(chain_offset=0, num_warmup=WM, num_samples=0, sample_begin=0, sample_capacity=0,
           seed=0, step_size=eps0, target_accept=0.8, max_tree_depth=10, adapt_step_size=True,
           slice_mode=0)
names = prog.layout.names
off = {n: prog.layout.offsets[names.index(n)] for n in ("mu", "tau", "sigma")}
tr = _engine.make_trace(C, 0, WM, cs.device)
for it in range(WM):
    cs.run_nuts(trace=tr, iter_begin=it, iter_count=1, **cfg)
    torch.cuda.synchronize()
    q = cs.positions()[CH].cpu().numpy()
    sig = q[off["sigma"]]
    t = tr.numpy()
    line = (f"it {it}: mu {q[off['mu']]:.4g} tau {q[off['tau']]:.4g} sigma {sig:.4g} "
            f"eps {t['step_size'][CH][it]:.3g} depth {t['tree_depth'][CH][it]} "
            f"leaves {t['n_leapfrog'][CH][it]} H0 {t['energy'][CH][it]:.6g} "
            f"acc {t['accept_stat'][CH][it]:.3g}")
    if it < 40 or it % 25 == 0 or not (0.1 < sig < 100):
        print(line, flush=True)
    if not (0.1 < sig < 100):
        np.save("gpurun_out/stuck_state.npy", cs.positions()[CH].cpu().numpy())
        break
