"""A layout the lane-resident kernel declines is reported, not silent (VERDICT
r1 weak 8): mc_program_kernel_note names the reason and hmc() warns when a
program the automatic plan would slice runs on a slower kernel."""
import warnings

import numpy as np
import pytest

import workloads as W

pytestmark = pytest.mark.gpu


def _six_scalars(ns):
    """Three data blocks, each y_k ~ N(mu_k, s_k): six broadcast parameters
    (the lane-resident layout holds four), 3000 elements."""
    rng = np.random.default_rng(3)
    ys = [rng.normal(k, 1.0 + k, 1000).astype(np.float32) for k in range(3)]

    def log_prob(p):
        lp = 0.0
        for k in range(3):
            lp = lp + ns.sum(ns.Normal(p[f"mu{k}"], p[f"s{k}"]).log_prob(ys[k]))
        return lp

    init = {}
    for k in range(3):
        init[f"mu{k}"] = np.float32(k)
        init[f"s{k}"] = np.float32(1.0 + k)
    return log_prob, init


def test_declined_layout_warns(gpu):
    import mlx_mcmc_amd as m
    from mlx_mcmc_amd import _trace

    lp, init = _six_scalars(W.ns_product())
    prog = _trace.compile_model(lp, init)
    assert prog.slice_kernel != "lanes"
    assert "broadcast parameters" in prog.kernel_note
    with pytest.warns(RuntimeWarning, match="broadcast parameters"):
        _, _, info = m.hmc(lp, init, num_samples=5, num_warmup=5, step_size=0.01,
                           num_leapfrog_steps=5, key=m.random.key(0), progress=False,
                           return_info=True)
    assert "broadcast parameters" in info.extra["kernel_note"]
    # an explicit kernel choice is the caller's decision: no warning
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        m.hmc(lp, init, num_samples=5, num_warmup=5, step_size=0.01, num_leapfrog_steps=5,
              key=m.random.key(0), progress=False, num_slices=1)


def test_lane_resident_layout_is_quiet(gpu):
    import mlx_mcmc_amd as m
    from mlx_mcmc_amd import _trace

    lp, init = W.hierarchical(W.ns_product(), *W.SHAPES["small"])
    prog = _trace.compile_model(lp, init)
    assert prog.slice_kernel == "lanes" and prog.kernel_note == ""
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        _, _, info = m.hmc(lp, init, num_samples=5, num_warmup=5, step_size=0.01,
                           num_leapfrog_steps=5, key=m.random.key(0), progress=False,
                           return_info=True)
    assert info.extra["kernel"] == "lanes" and "kernel_note" not in info.extra
