"""Per-chain work of the bench's NUTS Large line (hier 'large', 256 chains,
20 warmup + 20 timed iterations, one launch each): leaves per chain over the
timed window (min / median / mean / max), the step sizes, and the launch time
— the launch lasts as long as its longest chain, so mean / max is the share of
the chip's chain slots that stay busy."""
import os
import sys
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__)))]
import numpy as np
import torch
import workloads as W
from mlx_mcmc_amd import _engine, _trace

C = int(os.environ.get("CHAINS", "256"))
WM, K = int(os.environ.get("WARMUP", "20")), int(os.environ.get("STEPS", "20"))
G, N = W.SHAPES["large"]
lp, init = W.hierarchical(W.ns_product(), G, N)
prog = _trace.compile_model(lp, init, slices=int(os.environ.get("SLICES", "16")))
eps0 = float(os.environ.get("EPS0", "6.1458e-4"))
cs = _engine.ChainSet(prog, C, prog.layout.flatten(init), eps0, device=torch.device("cuda"))
smp = torch.empty((C, K, prog.D), dtype=torch.float32, device="cuda")
cfg = dict(chain_offset=0, num_warmup=WM, num_samples=K, sample_begin=0, sample_capacity=K,
           seed=0, step_size=eps0, target_accept=0.8, max_tree_depth=10, adapt_step_size=True,
           slice_mode=0)
cs.run_nuts(samples=smp, iter_begin=0, iter_count=WM, **cfg)
torch.cuda.synchronize()
g0 = cs.scalars()["n_grad"].astype(np.int64)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
cs.run_nuts(samples=smp, iter_begin=WM, iter_count=K, **cfg)
e1.record()
torch.cuda.synchronize()
sc = cs.scalars()
lv = sc["n_grad"].astype(np.int64) - g0
ms = e0.elapsed_time(e1)
print(f"{prog.nuts_kernel(10)} S={prog.num_slices}: launch {ms:.2f} ms, {lv.sum() / ms / 1e3:.3f} M leaf-steps/s")
print("leaves per chain: min %d  median %d  mean %.0f  max %d  (mean/max %.3f)" %
      (lv.min(), np.median(lv), lv.mean(), lv.max(), lv.mean() / lv.max()))
print("per-leaf time of the longest chain: %.2f us" % (ms * 1e3 / lv.max()))
eps = sc["step_size"]
print("step sizes: min %.3g median %.3g max %.3g" % (eps.min(), np.median(eps), eps.max()))
q = np.percentile(lv, [10, 25, 50, 75, 90, 99])
print("leaf percentiles 10/25/50/75/90/99:", q.astype(int).tolist())
# the longest chain's state (mu, tau, sigma) against the median chain's
q = cs.positions().cpu().numpy()
names = prog.layout.names
off = {n: prog.layout.offsets[names.index(n)] for n in ("mu", "tau", "sigma")}
for lab, c in (("longest", int(np.argmax(lv))), ("median", int(np.argsort(lv)[len(lv) // 2]))):
    print(f"{lab} chain {c}: leaves {lv[c]}, eps {eps[c]:.3g}, " +
          ", ".join(f"{n}={q[c, o]:.4g}" for n, o in off.items()) +
          f", theta[:3]={q[c, off['sigma'] + 1:off['sigma'] + 4]}")
