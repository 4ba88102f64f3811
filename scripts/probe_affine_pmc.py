"""One HMC launch of the N = 100 K affine regression (and of the same
likelihood as an expression term) for rocprofv3 counter passes: what bounds
the chain-per-workgroup tape at large N."""
import os
import sys
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__)))]
import numpy as np
import torch
import mlx_mcmc_amd as m
import mlx_mcmc_amd.core as mx
import workloads as W
from mlx_mcmc_amd import _engine, _trace

N = 100000
x, y = W.regression_data(N)
X, Y = mx.array(x), mx.array(y)
which = sys.argv[1] if len(sys.argv) > 1 else "fused"


def fused(p):
    lp = m.Normal(0, 10).log_prob(p["a"]) + m.Normal(0, 10).log_prob(p["b"])
    lp = lp + m.HalfNormal(5).log_prob(p["sigma"])
    return lp + mx.sum(m.Normal(p["a"] + p["b"] * X, p["sigma"]).log_prob(Y))


def handwritten(p):
    lp = m.Normal(0, 10).log_prob(p["a"]) + m.Normal(0, 10).log_prob(p["b"])
    lp = lp + m.HalfNormal(5).log_prob(p["sigma"])
    z = (Y - (p["a"] + p["b"] * X)) / p["sigma"]
    return lp + mx.sum(-0.5 * mx.square(z) - mx.log(p["sigma"]) - 0.9189385)


init = {"a": np.float32(1.5), "b": np.float32(2.0), "sigma": np.float32(0.5)}
prog = _trace.compile_model(fused if which == "fused" else handwritten, init)
cs = _engine.ChainSet(prog, 256, prog.layout.flatten(init), 1e-3, device=torch.device("cuda"))
samples = torch.empty((256, 1, prog.D), dtype=torch.float32, device="cuda")
cfg = dict(chain_offset=0, num_warmup=10 ** 6, num_samples=1, sample_begin=0, sample_capacity=1,
           seed=0, step_size=1e-3, target_accept=0.8, num_leapfrog_steps=10, adapt_step_size=False)
for i in range(3):
    cs.run_hmc(samples=samples, iter_begin=2 * i, iter_count=2, **cfg)
torch.cuda.synchronize()
print("ok", which)
