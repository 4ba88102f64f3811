"""Generate tests/golden/*.json from the CPU oracle (run here, committed).

  rng_kats.json        Philox words / uniforms / normals at fixed counters
  tape_kats.json       log p (oracle f32 and float64 closed form) and gradient
                       at fixed points of every BASELINE workload shape
  hmc_simple.json      config-1 HMC trace (accept bits, ratios, eps) seed 3
  nuts_illcond.json    config-5 NUTS trace (depth, leaves, alpha, eps) seed 11

tests/test_golden.py re-derives every fixture from the oracle (CPU) and the
GPU tests compare the HIP path against them.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import workloads as W  # noqa: E402
from oracle import philox as R  # noqa: E402
from oracle import samplers as S  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


def rng_kats():
    seed = 0x0123456789ABCDEF
    idx = np.arange(64)
    w = R.draw(seed, 3, 17, R.TAG_MOMENTUM, 0, idx)
    return {"seed": seed, "chain": 3, "iteration": 17, "tag": R.TAG_MOMENTUM, "sub": 0,
            "index0": 0, "n": 64, "words": w.astype(np.int64).tolist(),
            "uniforms": R.u01_f32(w).astype(float).tolist(),
            "normals": R.normals4(w).astype(float).tolist()}


def f64_logp(name, q):
    """Closed-form float64 log density of the workload at q (independent of torch)."""
    q = np.asarray(q, np.float64)
    c = -0.5 * np.log(2 * np.pi)

    def normal(x, m, s):
        return np.sum(c - np.log(s) - 0.5 * ((x - m) / s) ** 2)

    def half(x, s):
        return (np.log(2) + c - np.log(s) - 0.5 * (x / s) ** 2) if x >= 0 else -np.inf
    if name == "simple":
        y = W.simple_normal_data()
        return normal(q[0], 0, 10) + half(q[1], 5) + normal(y, q[0], q[1])
    if name == "iso":
        return normal(q, 0, 1)
    if name == "illcond":
        return normal(q, 0, W.illcond_scales(q.size).astype(np.float64))
    G, N = W.SHAPES[name]
    y, g = W.hierarchical_data(G, N)
    mu, tau, sg, th = q[0], q[1], q[2], q[3:]
    return (normal(mu, 0, 10) + half(tau, 5) + half(sg, 5) + normal(th, mu, tau)
            + normal(y.astype(np.float64), th[g], sg))


def tape_case(name):
    if name == "simple":
        return W.simple_normal(W.ns_oracle())
    if name == "iso":
        return W.iso_normal(W.ns_oracle())
    if name == "illcond":
        return W.illcond_normal(W.ns_oracle())
    G, N = W.SHAPES[name]
    return W.hierarchical(W.ns_oracle(), G, N)


def tape_kats():
    out = {}
    for name in ("simple", "iso", "illcond", "small", "medium"):
        lp, init = tape_case(name)
        M = S.EagerModel(lp, init)
        q0 = M.flatten(init)
        rng = np.random.default_rng(123)
        pts = []
        for _ in range(3):
            q = (q0 + rng.normal(0, 0.3, q0.size)).astype(np.float32)
            if name == "simple":
                q[1] = abs(q[1]) + 0.5
            if name in ("small", "medium"):
                q[1:3] = np.abs(q[1:3]) + 0.5
            l, g = M.logp_grad(q)
            pts.append({"q": q.astype(float).tolist(), "logp_f32": float(l),
                        "logp_f64": float(f64_logp(name, q)),
                        "grad": g.astype(float).tolist()})
        out[name] = pts
    return out


def hmc_simple():
    lp, init = W.simple_normal(W.ns_oracle())
    r = S.hmc(lp, init, num_samples=100, num_warmup=100, seed=3)
    return {"seed": 3, "num_warmup": 100, "num_samples": 100, "step_size": 0.1,
            "num_leapfrog_steps": 10, "accepted": [bool(x) for x in r.trace["accepted"]],
            "ratio": r.trace["ratio"], "eps": r.trace["step_size"],
            "samples_head": r.samples[:20].astype(float).tolist(),
            "accept_rate": r.accept_rate}


def nuts_illcond():
    lp, init = W.illcond_normal(W.ns_oracle())
    r = S.nuts(lp, init, num_samples=10, num_warmup=30, seed=11)
    return {"seed": 11, "num_warmup": 30, "num_samples": 10, "step_size": 0.1,
            "depth": r.trace["depth"], "leaves": r.trace["leaves"],
            "alpha": r.trace["alpha"], "eps": r.trace["step_size"]}


GENERATORS = {"rng_kats": rng_kats, "tape_kats": tape_kats, "hmc_simple": hmc_simple,
              "nuts_illcond": nuts_illcond}


def main():
    os.makedirs(OUT, exist_ok=True)
    for name, fn in GENERATORS.items():
        with open(os.path.join(OUT, name + ".json"), "w") as f:
            json.dump(fn(), f)
        print("wrote", name)


if __name__ == "__main__":
    main()
