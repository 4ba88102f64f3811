"""Posterior-moment fixture of the CPU oracle (test infrastructure).

tests/golden/posterior_small.json: SURVEY 8(d)'s parity rule needs reference
means and variances with their Monte-Carlo standard errors.  The oracle's HMC
(oracle/samplers.py, restating hmc.py:7-206) is run on the small hierarchical
shape (D = 10, N = 1 K, W.SHAPES["small"]) at the large config's eps = 0.01
and L = 20 with the step size held fixed (the reference's warmup rule, SURVEY
Q4, leaves some chains with a step size at which they never move again —
those are not posterior draws; the rule itself is pinned bit-exactly by the
trace tests) for 8 chains of 8000 draws after 500 warmup iterations, and its
Metropolis-Hastings (metropolis.py:6-101) on example 01's model with its
proposal scale 0.3 (examples/01_simple_normal.py:56-61) for 4 chains of
20000 draws; per parameter the fixture holds the pooled mean and variance,
the summed ESS (reference compute_ess rule, informational) and the MCSE of
both by batch means (oracle/diag.py mcse_batch).  Runs the
chains in parallel processes (about 10 minutes on 8 cores):

    python scripts/gen_posterior.py
"""
import json
import os
import sys
from multiprocessing import Pool

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

HMC = dict(num_samples=8000, num_warmup=500, step_size=0.01, num_leapfrog_steps=20,
           adapt_step_size=False)
MH = dict(num_samples=20000, proposal_scale=0.3)
CHAINS = {"hmc": 8, "mh": 4}


def _run(job):
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    import torch

    torch.set_num_threads(1)
    import workloads as W
    from oracle import samplers as S

    kind, chain = job
    if kind == "hmc":
        olp, oinit = W.hierarchical(W.ns_oracle(), *W.SHAPES["small"])
        r = S.hmc(olp, oinit, seed=0, chain=chain, record=False, **HMC)
    else:
        olp, oinit = W.simple_normal(W.ns_oracle())
        r = S.metropolis_hastings(olp, oinit, random_seed=0, chain=chain, record=False, **MH)
    return kind, chain, r.samples


def main():
    import numpy as np

    from oracle.diag import ess_batch, mcse_batch

    jobs = [(k, c) for k in ("hmc", "mh") for c in range(CHAINS[k])]
    with Pool(min(len(jobs), os.cpu_count() or 1)) as pool:
        res = pool.map(_run, jobs)
    out = {"hmc": dict(HMC, chains=CHAINS["hmc"], seed=0,
                       model="hierarchical small (G=7, N=1000), workloads.hierarchical; "
                             "layout order mu, tau, sigma, theta[0..6]"),
           "mh": dict(MH, chains=CHAINS["mh"], random_seed=0,
                      model="example 01 simple normal, workloads.simple_normal; mu, sigma")}
    for kind in ("hmc", "mh"):
        xs = [s for k, c, s in sorted(res, key=lambda t: (t[0], t[1])) if k == kind]
        x = np.stack(xs).astype(np.float64)            # [C, S, D]
        pooled = x.reshape(-1, x.shape[-1])
        mean = pooled.mean(0)
        var = pooled.var(0)
        ess = np.sum([ess_batch(xc) for xc in x], axis=0)
        mcse_m, mcse_v = mcse_batch(x)
        out[kind + "_moments"] = {
            "mean": mean.tolist(), "var": var.tolist(), "ess_reference_rule": ess.tolist(),
            "mcse_mean": mcse_m.tolist(), "mcse_var": mcse_v.tolist()}
    path = os.path.join(ROOT, "tests", "golden", "posterior_small.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
