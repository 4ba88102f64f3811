"""Oracle NUTS traces (oracle/samplers.py nuts, restating nuts.py:16-358) —
test infrastructure, run here on the CPU and committed.

  tests/golden/nuts_illcond_trace.npz
      BASELINE configs[4]'s model (kappa = 1000 diagonal Gaussian, D = 100),
      global chains 0, 1, 33, 63 of the 64-chain launch, seed 0, eps0 = 0.1,
      W = 40 warmup iterations with dual averaging acting, S = 20 sampling
      iterations at eps-bar, max_tree_depth 10.
  tests/golden/nuts_large_trace.npz
      The README "Large" hierarchical model (D = 1000, N = 100 K), chains 0,
      1, 2, seed 0, a fixed step size 2e-3 (adapt_step_size=False), W = 2,
      S = 10, max_tree_depth 10 (depths 7-8).
  tests/golden/nuts_large_da_trace.npz
      The same model and chains 0, 1 with dual averaging acting: eps0 = 2e-4,
      W = 20, S = 5 (the sliced NUTS kernel's adaptation check).
  tests/golden/nuts_hier_trace.npz
      The small hierarchical model (workloads.hierarchical, G = 7, N = 1 K:
      broadcast mu, tau, sigma and private theta), chains 0, 2 and 5 (5: the
      Q7/Q8 freeze — H0 ~ 1400 switches the f32 slice off and NaN leaves count
      as alpha = 1), same
      settings with eps0 = 0.01.

Per chain and iteration: tree depth, leaves, mean acceptance statistic
alpha, step size, H0, the f32 log U of the slice draw, and the decision
margins (smallest slice gap |log u + H'|, divergence gap, relative U-turn
dot; oracle/samplers.py nuts); the S stored draws [S, D].

    python scripts/gen_golden_nuts.py [illcond hier large large_da]
"""
import json
import os
import sys
from multiprocessing import Pool

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLD = os.path.join(ROOT, "tests", "golden")

RUNS = {
    "illcond": dict(chains=(0, 1, 33, 63), cfg=dict(num_warmup=40, num_samples=20, step_size=0.1,
                                                    max_tree_depth=10, target_accept=0.65)),
    "hier": dict(chains=(0, 2, 5), cfg=dict(num_warmup=40, num_samples=20, step_size=0.01,
                                         max_tree_depth=10, target_accept=0.65)),
    # the README "Large" row (D = 1000, N = 100 K) at a fixed step size (no
    # dual averaging: the trees are then compared without an adaptation that
    # amplifies alpha rounding into eps): depths 7-8, 127-255 leaves
    "large": dict(chains=(0, 1, 2), cfg=dict(num_warmup=2, num_samples=10, step_size=2e-3,
                                          max_tree_depth=10, target_accept=0.65,
                                          adapt_step_size=False)),
    # the same model with the reference's dual averaging acting (VERDICT r4
    # "Next round" 1): W = 20 warmup iterations from eps0 = 2e-4, S = 5 (the
    # first update moves eps to 10 eps0 e^(...) ~ 4e-3 and it settles near
    # 1e-3; from eps0 = 2e-3 it jumps to 0.034, where a leapfrog step
    # amplifies fp32 rounding differences ~300-fold and any two
    # implementations separate within two iterations)
    "large_da": dict(chains=(0, 1), cfg=dict(num_warmup=20, num_samples=5, step_size=2e-4,
                                             max_tree_depth=10, target_accept=0.65)),
}
SEED = 0
KEYS = ("depth", "leaves", "alpha", "step_size", "energy", "slice_gap", "div_gap",
        "uturn_margin", "da_step_size")


def model(name, ns):
    import workloads as W

    if name == "illcond":
        return W.illcond_normal(ns)
    if name in ("large", "large_da"):
        return W.hierarchical(ns, *W.SHAPES["large"])
    return W.hierarchical(ns, *W.SHAPES["small"])


def _run(job):
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    import numpy as np
    import torch

    torch.set_num_threads(1)
    import workloads as W
    from oracle import philox as R
    from oracle import samplers as S

    name, chain = job
    lp, init = model(name, W.ns_oracle())
    cfg = RUNS[name]["cfg"]
    r = S.nuts(lp, init, seed=SEED, chain=chain, **cfg)
    n = cfg["num_warmup"] + cfg["num_samples"]
    out = {k: np.asarray(r.trace[k], np.float64) for k in KEYS}
    out["log_u"] = np.array([R.logf_u01(R.uniform(SEED, chain, i, R.TAG_SLICE))
                             for i in range(n)], np.float32)
    out["samples"] = r.samples
    return name, chain, out


def main():
    import numpy as np

    only = sys.argv[1:] or list(RUNS)
    jobs = [(n, c) for n, r in RUNS.items() if n in only for c in r["chains"]]
    with Pool(min(8, len(jobs))) as pool:
        res = pool.map(_run, jobs)
    for name, spec in RUNS.items():
        if name not in only:
            continue
        outs = [o for n, c, o in sorted((t for t in res if t[0] == name),
                                        key=lambda t: spec["chains"].index(t[1]))]
        arrays = {k: np.stack([o[k] for o in outs]) for k in KEYS + ("log_u",)}
        arrays["depth"] = arrays["depth"].astype(np.int32)
        arrays["leaves"] = arrays["leaves"].astype(np.int32)
        arrays["samples"] = np.stack([o["samples"] for o in outs]).astype(np.float32)
        arrays["chains"] = np.array(spec["chains"], np.int32)
        arrays["config"] = np.array(json.dumps(dict(spec["cfg"], seed=SEED, model=name)))
        path = os.path.join(GOLD, f"nuts_{name}_trace.npz")
        np.savez_compressed(path, **arrays)
        print("wrote", path, "depths", arrays["depth"][:, :12].tolist(),
              "min slice gap", arrays["slice_gap"].min(), "min uturn", arrays["uturn_margin"].min())


if __name__ == "__main__":
    main()
