"""Example 02's HMC run on the oracle (test infrastructure, run here, committed).

The only sampler-level numbers the reference publishes are example 02's HMC
results (PROGRESS.md:74-82): acceptance 99.98 %, ESS(mu) 264 / 5000, ESS(sigma)
463 / 5000, |mean(mu) - 5| = 0.210, |mean(sigma) - 2| = 0.163, from
MCMC(log_prob).run({'mu': 0, 'sigma': 1}, num_samples=5000, num_warmup=1000,
method='hmc', step_size=0.1, num_leapfrog_steps=10, adapt_step_size=True,
target_accept=0.8, random_seed=42) on np.random.seed(42) data
(examples/02_hmc_comparison.py:23-28,40-55,86-100; ESS by the example's own
helper :111-128).  Those numbers come from one draw of MLX's RNG, which is
not available here; the oracle restates the sampler (oracle/samplers.py)
with the shared Philox stream, so a run here is a different realisation of
the same random process.  This script runs it for seed 42 (MCMC.run's key),
chains 0..63 (64 realisations, ~5 minutes on 8 cores), and records per chain
the same five statistics:

    tests/golden/example02_hmc.json

tests/test_oracle_pins.py checks the fixture against the published numbers
(tolerances stated there); tests/test_gpu_samplers.py runs the same 64 chains
through MCMC.run / hmc() on the GPU and checks them against the fixture.

    python scripts/gen_example02.py
"""
import json
import os
import sys
from multiprocessing import Pool

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CFG = dict(num_samples=5000, num_warmup=1000, step_size=0.1, num_leapfrog_steps=10,
           adapt_step_size=True, target_accept=0.8)
SEED = 42
CHAINS = 64


def _run(chain):
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    import torch

    torch.set_num_threads(1)
    import workloads as W
    from oracle import samplers as S
    from oracle.diag import compute_ess_02

    lp, init = W.simple_normal(W.ns_oracle())
    r = S.hmc(lp, init, seed=SEED, chain=chain, record=False, **CFG)
    mu, sigma = r.samples[:, 0], r.samples[:, 1]
    return {"chain": chain, "accept_rate": r.accept_rate,
            "warmup_accept_rate": r.warmup_accept_rate, "step_size": r.step_size,
            "ess_mu": compute_ess_02(mu), "ess_sigma": compute_ess_02(sigma),
            "mean_mu": float(mu.astype("float64").mean()),
            "mean_sigma": float(sigma.astype("float64").mean()),
            "err_mu": abs(float(mu.astype("float64").mean()) - 5.0),
            "err_sigma": abs(float(sigma.astype("float64").mean()) - 2.0)}


def main():
    with Pool(min(CHAINS, os.cpu_count() or 1)) as pool:
        res = pool.map(_run, range(CHAINS))
    out = {"config": dict(CFG, seed=SEED, chains=CHAINS, init={"mu": 0.0, "sigma": 1.0},
                          model="examples/02_hmc_comparison.py:40-52 (workloads.simple_normal)"),
           "published": {"accept_rate": 0.9998, "ess_mu": 264, "ess_sigma": 463,
                         "err_mu": 0.210, "err_sigma": 0.163,
                         "source": "PROGRESS.md:74-82"},
           "chains": res}
    path = os.path.join(ROOT, "tests", "golden", "example02_hmc.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    for r in res:
        print({k: round(v, 4) if isinstance(v, float) else v for k, v in r.items()})


if __name__ == "__main__":
    main()
