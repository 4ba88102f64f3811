"""Oracle HMC trace of BASELINE configs[1] (isotropic N(0, I_100), L = 10) —
test infrastructure, run here on the CPU and committed.

  tests/golden/hmc_iso_trace.npz
      The oracle's HMC (oracle/samplers.py, restating hmc.py:7-206) for global
      chains 0, 1, 33, 63 of the config's 64-chain launch, seed 0, from x = 0:
      eps0 = 0.9 (the decisions are a mix: the config's eps0 = 0.1 accepts
      every proposal), W = 30 warmup iterations with the reference's rule on
      (it acts at i = 11..29, hmc.py:163), S = 20.  Per chain and iteration:
      accept bit, log ratio -(H_prop - H_init), f32 log U of the accept draw,
      step size, H_init; the S stored draws [S, D].

    python scripts/gen_golden_iso.py
"""
import json
import os
import sys
from multiprocessing import Pool

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLD = os.path.join(ROOT, "tests", "golden")

TRACE = dict(num_samples=20, num_warmup=30, step_size=0.9, num_leapfrog_steps=10,
             adapt_step_size=True, target_accept=0.8)
CHAINS = (0, 1, 33, 63)


def _run(chain):
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    import numpy as np
    import torch

    torch.set_num_threads(1)
    import workloads as W
    from oracle import philox as R
    from oracle import samplers as S

    lp, init = W.iso_normal(W.ns_oracle())
    r = S.hmc(lp, init, seed=0, chain=chain, record=True, **TRACE)
    n = TRACE["num_warmup"] + TRACE["num_samples"]
    out = {"samples": r.samples,
           "log_u": np.array([R.logf_u01(R.uniform(0, chain, i, R.TAG_ACCEPT)) for i in range(n)],
                             np.float32)}
    for k in ("accepted", "ratio", "step_size", "energy"):
        out[k] = np.asarray(r.trace[k])
    return chain, out


def main():
    import numpy as np

    with Pool(len(CHAINS)) as pool:
        res = dict(pool.map(_run, CHAINS))
    outs = [res[c] for c in CHAINS]
    arrays = {"chains": np.array(CHAINS, np.int32),
              "samples": np.stack([o["samples"] for o in outs]).astype(np.float32),
              "accepted": np.stack([o["accepted"] for o in outs]).astype(np.uint8),
              "ratio": np.stack([o["ratio"] for o in outs]).astype(np.float32),
              "log_u": np.stack([o["log_u"] for o in outs]),
              "step_size": np.stack([o["step_size"] for o in outs]).astype(np.float64),
              "energy": np.stack([o["energy"] for o in outs]).astype(np.float32),
              "config": np.array(json.dumps(dict(TRACE, seed=0, model="iso D=100")))}
    path = os.path.join(GOLD, "hmc_iso_trace.npz")
    np.savez_compressed(path, **arrays)
    print("wrote", path, "accept fraction per chain", arrays["accepted"].mean(1),
          "final eps", arrays["step_size"][:, -1])


if __name__ == "__main__":
    main()
