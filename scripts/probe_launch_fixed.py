"""Per-launch fixed cost of the bench kernel: HIP-event time of launches of
1..50 iterations on the large shape (256 chains), interleaved, after a
clock warm on the same buffers.  Prints a least-squares fit ms = a + b * n."""
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
cfg = dict(chain_offset=0, num_warmup=100000, num_samples=1, sample_begin=0, sample_capacity=1,
           seed=0, step_size=6.1458e-4, target_accept=0.8, num_leapfrog_steps=20,
           adapt_step_size=False)
it = 0


def run(n):
    global it
    chains.run_hmc(samples=samples, iter_begin=it, iter_count=n, **cfg)
    it += n


t0 = time.time()
while time.time() - t0 < 0.6:
    run(20)
torch.cuda.synchronize()
sizes = [1, 2, 5, 10, 20, 50]
res = {n: [] for n in sizes}
stream = torch.cuda.current_stream()
for rep in range(6):
    for n in sizes:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        run(n)
        e1.record(stream)
        torch.cuda.synchronize()
        res[n].append(e0.elapsed_time(e1))
xs, ys = [], []
for n in sizes:
    v = sorted(res[n])[1:-1]
    print(n, "iters: median ms", round(float(np.median(res[n])), 4), "all", [round(x, 4) for x in res[n]])
    xs += [n] * len(v)
    ys += v
b, a = np.polyfit(xs, ys, 1)
print(f"fit: {a * 1000:.1f} us fixed + {b * 1000:.2f} us per iteration")

# host-side cost of one launch call and the wall time of a synchronised
# 20-iteration launch (the driver's timed region)
torch.cuda.synchronize()
hs, ws_, evs = [], [], []
for rep in range(8):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    run(20)
    t1 = time.perf_counter()
    e1.record(stream)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    hs.append((t1 - t0) * 1e3)
    ws_.append((t2 - t0) * 1e3)
    evs.append(e0.elapsed_time(e1))
print("host submit ms", [round(x, 4) for x in hs])
print("wall ms", [round(x, 4) for x in ws_])
print("event ms", [round(x, 4) for x in evs])
import cProfile, pstats
pr = cProfile.Profile()
pr.enable()
for rep in range(50):
    run(1)
pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("cumulative").print_stats(12)
