"""Per-step cost of an expression program against N (the JIT'd tape kernel):
logistic and two-predictor regressions, 256 chains, L = 10, HIP events
around one launch — a linear fit separates the fixed per-step cost from the
per-element one."""
import os
import sys
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__)))]
import numpy as np
import torch
import workloads as W
from mlx_mcmc_amd import _engine, _trace


def step_us(lp, init, chains=256, L=10, iters=10):
    prog = _trace.compile_model(lp, init)
    cs = _engine.ChainSet(prog, chains, prog.layout.flatten(init), 1e-3, device=torch.device("cuda"))
    smp = torch.empty((chains, 1, prog.D), dtype=torch.float32, device="cuda")
    cfg = dict(chain_offset=0, num_warmup=10 ** 6, num_samples=1, sample_begin=0,
               sample_capacity=1, seed=0, step_size=1e-3, target_accept=0.8,
               num_leapfrog_steps=L, adapt_step_size=False)
    cs.run_hmc(samples=smp, iter_begin=0, iter_count=2, **cfg)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    cs.run_hmc(samples=smp, iter_begin=2, iter_count=iters, **cfg)
    e1.record()
    torch.cuda.synchronize()
    cs.check_status()
    return e0.elapsed_time(e1) * 1e3 / (iters * L)


chains = int(os.environ.get("CHAINS", "256"))
for name, mk, init in (("logistic", W.logistic_regression, {"a": np.float32(-0.3), "b": np.float32(1.1)}),
                       ("two-predictor", W.two_predictor_regression,
                        {"a": np.float32(0.5), "b1": np.float32(1.2), "b2": np.float32(-0.8),
                         "log_sigma": np.float32(-0.5)})):
    ns, ts = [], []
    for n in (6250, 12500, 25000, 50000, 100000, 200000):
        lp, _ = mk(W.ns_product(), n)
        t = step_us(lp, init, chains=chains)
        ns.append(n)
        ts.append(t)
        print(f"{name} N={n}: {t:.2f} us/step, {chains / t:.3f} M chain-steps/s", flush=True)
    b, a = np.polyfit(ns, ts, 1)
    print(f"{name}: fixed {a:.2f} us/step + {b * 1e3:.3f} us per 1000 elements")
