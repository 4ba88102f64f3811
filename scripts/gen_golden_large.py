"""Oracle fixtures at the bench's own shape (BASELINE configs[2], SURVEY 8d
"Large": hierarchical Normal, D = 1000, N = 100 K, L = 20) — test
infrastructure, run here on the CPU and committed.

  tests/golden/hmc_large_trace.npz
      The oracle's HMC (oracle/samplers.py, restating hmc.py:7-206) for
      global chains 0, 1, 77 and 255 of seed 0 (different waves, workgroups
      and lane positions of the 256-chain launch) from the workload's init:
      eps0 = 3e-3 (a step size at which the chains move and the decisions
      are a mix — at the bench's old eps0 = 0.01 every trajectory blows up
      and every proposal is rejected), W = 15 warmup iterations with the
      reference's rule on (it acts at i = 11..14, hmc.py:163; a longer
      warmup raises eps past stability on some chains), S = 15 sampling
      iterations.  Per chain and iteration: accept bit, log ratio
      -(H_prop - H_init), f32 log U of the accept draw, step size, H_init;
      the 15 stored draws [S, D].
  tests/golden/posterior_large.json
      Posterior moments at the same shape: 16 chains (0..15, seed 0) at a
      fixed eps = 2e-3 (accept ~0.9), W = 200, S = 2000; per parameter the
      pooled mean / variance and their batch-means MCSE (oracle/diag.py) —
      north_star's "posterior moments within 1 % of reference" at the
      1000-parameter / 100 K-observation model.
  tests/golden/posterior_large_adapt.json
      The same 16 chains with the reference's warmup rule on (eps0 = 3e-3,
      W = 300, S = 2000): per chain the final step size and the sampling
      accept rate (the rule leaves chains 0 and 13 at eps = 5.4e-3, past
      stability, where they never accept again — SURVEY Q4), and the pooled
      moments of all 16 chains (informational: frozen chains are no
      posterior draws).

    python scripts/gen_golden_large.py [trace|posterior|adapt|all]
"""
import json
import os
import sys
from multiprocessing import Pool

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLD = os.path.join(ROOT, "tests", "golden")

TRACE = dict(num_samples=15, num_warmup=15, step_size=3e-3, num_leapfrog_steps=20,
             adapt_step_size=True, target_accept=0.8)
TRACE_CHAINS = (0, 1, 77, 255)
POST = dict(num_samples=2000, num_warmup=200, step_size=2e-3, num_leapfrog_steps=20,
            adapt_step_size=False, target_accept=0.8)
ADAPT = dict(num_samples=2000, num_warmup=300, step_size=3e-3, num_leapfrog_steps=20,
             adapt_step_size=True, target_accept=0.8)
POST_CHAINS = 16


def _run(job):
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    import numpy as np
    import torch

    torch.set_num_threads(1)
    import workloads as W
    from oracle import philox as R
    from oracle import samplers as S

    kind, chain = job
    lp, init = W.hierarchical(W.ns_oracle(), *W.SHAPES["large"])
    cfg = {"trace": TRACE, "posterior": POST, "adapt": ADAPT}[kind]
    r = S.hmc(lp, init, seed=0, chain=chain, record=(kind == "trace"), **cfg)
    out = {"samples": r.samples, "step_size": r.step_size, "accept_rate": r.accept_rate}
    if kind == "trace":
        n = cfg["num_warmup"] + cfg["num_samples"]
        out["log_u"] = np.array([R.logf_u01(R.uniform(0, chain, i, R.TAG_ACCEPT))
                                 for i in range(n)], np.float32)
        for k in ("accepted", "ratio", "step_size", "energy"):
            out["t_" + k] = np.asarray(r.trace[k])
    return kind, chain, out


def trace(pool):
    import numpy as np

    res = pool.map(_run, [("trace", c) for c in TRACE_CHAINS])
    res = [o for _, _, o in sorted(res, key=lambda t: TRACE_CHAINS.index(t[1]))]
    arrays = {"chains": np.array(TRACE_CHAINS, np.int32),
              "samples": np.stack([o["samples"] for o in res]).astype(np.float32),
              "accepted": np.stack([o["t_accepted"] for o in res]).astype(np.uint8),
              "ratio": np.stack([o["t_ratio"] for o in res]).astype(np.float32),
              "log_u": np.stack([o["log_u"] for o in res]),
              "step_size": np.stack([o["t_step_size"] for o in res]).astype(np.float64),
              "energy": np.stack([o["t_energy"] for o in res]).astype(np.float32),
              "config": np.array(json.dumps(dict(TRACE, seed=0, shape="large")))}
    path = os.path.join(GOLD, "hmc_large_trace.npz")
    np.savez_compressed(path, **arrays)
    acc = arrays["accepted"]
    print("wrote", path, "accept fraction per chain", acc.mean(1))


def posterior(pool, kind="posterior"):
    import numpy as np

    from oracle.diag import ess_batch, mcse_batch

    cfg = POST if kind == "posterior" else ADAPT
    res = pool.map(_run, [(kind, c) for c in range(POST_CHAINS)])
    res = sorted(res, key=lambda t: t[1])
    x = np.stack([o["samples"] for _, _, o in res]).astype(np.float64)   # [C, S, D]
    pooled = x.reshape(-1, x.shape[-1])
    mcse_m, mcse_v = mcse_batch(x)
    ess = np.sum([ess_batch(xc) for xc in x], axis=0)
    out = {"hmc": dict(cfg, chains=POST_CHAINS, seed=0,
                       model="hierarchical large (G=997, N=100000), workloads.hierarchical; "
                             "layout order mu, tau, sigma, theta[0..996]",
                       final_step_size=[float(o["step_size"]) for _, _, o in res],
                       accept_rate=[float(o["accept_rate"]) for _, _, o in res]),
           "hmc_moments": {"mean": pooled.mean(0).tolist(), "var": pooled.var(0).tolist(),
                           "ess_reference_rule": ess.tolist(), "mcse_mean": mcse_m.tolist(),
                           "mcse_var": mcse_v.tolist()}}
    path = os.path.join(GOLD, "posterior_large.json" if kind == "posterior"
                        else "posterior_large_adapt.json")
    with open(path, "w") as f:
        json.dump(out, f)
    print("wrote", path, "final eps", out["hmc"]["final_step_size"],
          "accept", out["hmc"]["accept_rate"])


def main():
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    with Pool(min(16, os.cpu_count() or 1)) as pool:
        if what in ("trace", "all"):
            trace(pool)
        if what in ("posterior", "all"):
            posterior(pool)
        if what in ("adapt", "all"):
            posterior(pool, "adapt")


if __name__ == "__main__":
    main()
