"""north_star's "posterior moments within 1 %", against known answers with no
Monte-Carlo error of their own (VERDICT r2 "Next round" 1):

  * BASELINE configs[2] — the Large hierarchical model (D = 1000, N = 100 K)
    on the bench kernel (k_hmc_lf, 16 slices): exact f64 moments from
    oracle/exact.py (tests/golden/posterior_exact.json; pinned against the
    oracle's HMC in tests/test_exact_posterior.py), and the README's medium
    and small shapes the same way;
  * configs[1] — isotropic N(0, I_100), HMC L = 10: mean 0, variance 1;
  * configs[4] — NUTS depth 10 with dual averaging on the kappa = 1000
    diagonal Gaussian: mean 0, variance s_i^2.

Each run is long enough that z MCSE (z = 4.42: Bonferroni over 2 x 1000
comparisons at 1 % family-wise, as in test_gpu_posterior_parity.py) stays
below 1 % for every parameter, so the per-parameter check is "within 1 %":
means within 1 % of max(|mean|, sd) (a mean near zero has no relative
scale of its own; the posterior sd is the parameter's natural one),
variances within 1 % of the variance.  The effective bounds are printed.

HMC runs at a fixed step size (adapt_step_size=False): the reference's
warmup rule can leave chains at a step size where they never
move again (test_gpu_posterior_parity.py covers that regime separately);
NUTS runs the reference's dual averaging and samples at the adapted eps-bar.
"""
import json
import os

import numpy as np
import pytest

import workloads as W
from _streaming import check_within_one_percent, stream_moments

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
Z = 4.42


def _exact(shape):
    with open(os.path.join(GOLD, "posterior_exact.json")) as f:
        return json.load(f)["shapes"][shape]


# shape -> (step size, leapfrog steps, chains, warmup, samples, batch)
HIER = {
    "large": (2e-3, 20, 256, 1000, 60000, 3000),
    "medium": (5e-3, 20, 256, 1000, 60000, 3000),
    "small": (0.01, 100, 1024, 2000, 80000, 4000),
}


@pytest.mark.parametrize("shape", ["large", "medium", "small"])
def test_hierarchical_posterior_within_one_percent(gpu, shape):
    from mlx_mcmc_amd import _trace

    eps, L, C, Wm, S, batch = HIER[shape]
    lp, init = W.hierarchical(W.ns_product(), *W.SHAPES[shape])
    prog = _trace.compile_model(lp, init)
    if shape == "large":
        assert prog.slice_kernel == "lanes" and prog.lanes_fast, "not the bench kernel"
    g = stream_moments(prog, "hmc", C, prog.layout.flatten(init), step_size=eps,
                       num_warmup=Wm, num_samples=S, batch=batch, num_leapfrog_steps=L)
    print(f"{shape}: kernel {prog.slice_kernel} fast={prog.lanes_fast}, accept "
          f"{g['accept_rate'].mean():.3f} (min {g['accept_rate'].min():.3f})")
    assert g["accept_rate"].min() > 0.5
    check_within_one_percent(g, _exact(shape), label=f"hierarchical {shape}", z=Z)


def test_isotropic_posterior_within_one_percent(gpu):
    """BASELINE configs[1]: sum(Normal(0, 1).log_prob(x)), D = 100, eps 0.1,
    L = 10 (the config's settings, step size held)."""
    from mlx_mcmc_amd import _trace

    lp, init = W.iso_normal(W.ns_product())
    prog = _trace.compile_model(lp, init)
    g = stream_moments(prog, "hmc", 256, prog.layout.flatten(init), step_size=0.1,
                       num_warmup=500, num_samples=20000, batch=1000, num_leapfrog_steps=10)
    print(f"isotropic: kernel {prog.slice_kernel} fast={prog.lanes_fast}, accept "
          f"{g['accept_rate'].mean():.3f}")
    check_within_one_percent(g, {"mean": np.zeros(100), "var": np.ones(100)},
                             label="isotropic D=100", z=Z)


def test_illcond_nuts_posterior_within_one_percent(gpu):
    """BASELINE configs[4]: NUTS max_tree_depth 10, dual averaging (target
    0.65, eps0 0.1, W = 1000) on N(0, diag(s^2)), kappa = 1000."""
    from mlx_mcmc_amd import _trace

    lp, init = W.illcond_normal(W.ns_product())
    prog = _trace.compile_model(lp, init)
    g = stream_moments(prog, "nuts", 1024, prog.layout.flatten(init), step_size=0.1,
                       num_warmup=1000, num_samples=4000, batch=1000, max_tree_depth=10,
                       adapt_step_size=True, target_accept=0.65)
    print(f"illcond NUTS: kernel {prog.nuts_kernel(10)}, eps-bar median "
          f"{np.median(g['step_size']):.4g}, mean depth {g['mean_tree_depth'].mean():.2f}")
    s = W.illcond_scales().astype(np.float64)
    check_within_one_percent(g, {"mean": np.zeros_like(s), "var": s * s},
                             label="illcond NUTS D=100", z=Z)
