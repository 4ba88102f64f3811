"""Time one batched gradient evaluation (mc_logp_grad) per model variant."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

ge._ensure_pkg()
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mlx_mcmc_amd as m  # noqa: E402
import mlx_mcmc_amd.core as mx  # noqa: E402
import workloads as W  # noqa: E402
from mlx_mcmc_amd import _engine, _trace  # noqa: E402

G, N = W.SHAPES["large"]
y, group = W.hierarchical_data(G, N)


def variants():
    lp_full, init = W.hierarchical(W.ns_product(), G, N)
    yield "full", lp_full, init

    def lik_only(p):
        return mx.sum(m.Normal(p["theta"][group], p["sigma"]).log_prob(y))
    yield "likelihood", lik_only, {"sigma": np.float32(1), "theta": init["theta"]}

    def prior_only(p):
        lp = m.Normal(0, 10).log_prob(p["mu"]) + m.HalfNormal(5).log_prob(p["tau"])
        return lp + mx.sum(m.Normal(p["mu"], p["tau"]).log_prob(p["theta"]))
    yield "prior", prior_only, {"mu": np.float32(1), "tau": np.float32(2), "theta": init["theta"]}

    def iid(p):
        return mx.sum(m.Normal(p["mu"], p["sigma"]).log_prob(y))
    yield "iid_100k", iid, {"mu": np.float32(1), "sigma": np.float32(2)}

    def scalar(p):
        return m.Normal(0, 1).log_prob(p["x"])
    yield "scalar", scalar, {"x": np.float32(0.5)}


for name, fn, init in variants():
    prog = _trace.compile_model(fn, init)
    q0 = prog.layout.flatten(init)
    for P in (1, 256):
        q = torch.tensor(np.tile(q0, (P, 1)), device="cuda")
        _engine.logp_grad(prog, q)
        torch.cuda.synchronize()
        reps = 20
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            _engine.logp_grad(prog, q)
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / reps
        print(f"{name:12s} wpc={prog.waves_per_chain:2d} points={P:4d}  {ms * 1e3:9.1f} us/launch  "
              f"{ms * 1e3 / max(P / 256, 1):9.1f} us per 256-point wave", flush=True)

# ---- per-leapfrog-step time of the HMC kernel, per model variant ------------
print("--- k_hmc, 256 chains, L=20, one iteration per launch ---")
for name, fn, init in variants():
    prog = _trace.compile_model(fn, init)
    q0 = prog.layout.flatten(init)
    cs = _engine.ChainSet(prog, 256, q0, 1e-4)
    cfg = dict(chain_offset=0, num_warmup=0, num_samples=10, sample_begin=0, sample_capacity=0,
               seed=1, step_size=1e-4, target_accept=0.8, num_leapfrog_steps=20,
               adapt_step_size=False)
    cs.run_hmc(iter_begin=0, iter_count=1, **cfg)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for it in range(5):
        cs.run_hmc(iter_begin=1 + it, iter_count=1, **cfg)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 5
    print(f"{name:12s} wpc={prog.waves_per_chain}  {ms * 1e3:8.1f} us/iteration  "
          f"{ms * 1e3 / 20:7.2f} us/leapfrog", flush=True)
