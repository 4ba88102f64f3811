"""Float64 known answers for the hierarchical posteriors (oracle/exact.py) —
test infrastructure, run here on the CPU and committed.

  tests/golden/posterior_exact.json
      For each README shape (small G=7/N=1K, medium G=97/N=10K, large
      G=997/N=100K — workloads.SHAPES, data workloads.hierarchical_data seed 0):
      exact posterior means and variances in layout order (mu, tau, sigma,
      theta[0..G-1]), the moments of (log tau, log sigma) (the unconstrained
      parameters of workloads.hierarchical_reparam, whose layout order is
      mu, log_tau, log_sigma, theta), the quadrature grid, and the quadrature
      error (both sets of moments) measured by
      halving the grid spacing (relative to max(|mean|, sd) for means and to
      the variance for variances).

    python scripts/gen_posterior_exact.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLD = os.path.join(ROOT, "tests", "golden")

N_GRID = 161


def main():
    import workloads as W
    from oracle import exact as E

    out = {"model": "workloads.hierarchical: mu ~ N(0,10), tau ~ HalfNormal(5), "
                    "sigma ~ HalfNormal(5), theta_g ~ N(mu, tau), y_i ~ N(theta_{g_i}, sigma); "
                    "layout order mu, tau, sigma, theta[0..G-1]",
           "method": "oracle/exact.py: (mu, theta) integrated in closed form given "
                     "(tau, sigma); 2-D equally spaced rule in (log tau, log sigma), "
                     f"{N_GRID}x{N_GRID} points over +-10 Laplace sd",
           "shapes": {}}
    for shape, (G, N) in W.SHAPES.items():
        y, g = W.hierarchical_data(G, N)
        r = E.hierarchical_moments(y, g, G, n_grid=N_GRID)
        em, ev = E.quadrature_error(y, g, G, n_grid=N_GRID)
        out["shapes"][shape] = {"G": G, "N": N, "mean": r["mean"].tolist(),
                                "var": r["var"].tolist(),
                                "log_tau_sigma_mean": r["log_tau_sigma_mean"],
                                "log_tau_sigma_var": r["log_tau_sigma_var"],
                                "mode_log_tau_sigma": r["mode_log_tau_sigma"],
                                "laplace_sd_log_tau_sigma": r["laplace_sd_log_tau_sigma"],
                                "edge_weight": r["edge_weight"],
                                "quadrature_rel_error_mean": em,
                                "quadrature_rel_error_var": ev}
        print(shape, "mu/tau/sigma mean", r["mean"][:3], "quadrature error", em, ev)
    path = os.path.join(GOLD, "posterior_exact.json")
    with open(path, "w") as f:
        json.dump(out, f)
    print("wrote", path)


if __name__ == "__main__":
    main()
