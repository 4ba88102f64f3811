"""How an idle gap before a launch changes its duration (clock / power
state): 20-iteration launches of the bench kernel after idle gaps of
0 .. 100 ms (HIP events), each gap preceded by 200 ms of back-to-back work."""
import sys
import time
sys.path[:0] = ["."]
import numpy as np
import torch
import workloads as W
from mlx_mcmc_amd import _engine, _trace

G, N = W.SHAPES["large"]
lp_fn, init = W.hierarchical(W.ns_product(), G, N)
prog = _trace.compile_model(lp_fn, init)
C = 256
chains = _engine.ChainSet(prog, C, prog.layout.flatten(init), 6.1458e-4, device=torch.device("cuda"))
samples = torch.empty((C, 1, prog.D), dtype=torch.float32, device="cuda")
cfg = dict(chain_offset=0, num_warmup=10 ** 7, num_samples=1, sample_begin=0, sample_capacity=1,
           seed=0, step_size=6.1458e-4, target_accept=0.8, num_leapfrog_steps=20,
           adapt_step_size=False)
it = 0
stream = torch.cuda.current_stream()


def run(n):
    global it
    chains.run_hmc(samples=samples, iter_begin=it, iter_count=n, **cfg)
    it += n


def busy(ms):
    t0 = time.time()
    while (time.time() - t0) * 1e3 < ms:
        for _ in range(4):
            run(5)
        torch.cuda.synchronize()


def spin(us):
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e6 < us:
        pass


busy(500)
for gap_us in [0, 20, 100, 300, 1000, 3000, 10000, 100000]:
    out = []
    for rep in range(4):
        busy(200)
        spin(gap_us)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        run(20)
        e1.record(stream)
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1))
    print(f"idle {gap_us:>6} us before a 20-iteration launch: ms {[round(x, 4) for x in out]}")
# back to back (no sync between)
busy(200)
evs = []
for rep in range(6):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    run(20)
    e1.record(stream)
    evs.append((e0, e1))
torch.cuda.synchronize()
print("back to back:", [round(a.elapsed_time(b), 4) for a, b in evs])
