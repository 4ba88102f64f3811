"""The expression-term JIT's code generation and compilation, on the CPU
(csrc/jit.hip; hiprtc cross-compiles gfx950 without a device): every
expression model of tests/test_gpu_expr.py compiles into each tape kernel
that runs it (k_hmc, k_nuts, k_mh), and the generated source depends on the
model's structure only (the same model over different data generates the same
source, so one code object serves both).  Running the code is
tests/test_gpu_expr_jit.py."""
import ctypes

import pytest

import workloads as W
from _jit_models import MODELS, host_program

KERNELS = ["mc::k_hmc<8, true, true>", "mc::k_nuts<8, false, true>", "mc::k_mh<1, true, true>"]


def _source(h):
    from mlx_mcmc_amd import _lib

    lib = _lib.load()
    n = lib.mc_debug_expr_jit_source(h, None, 0)
    buf = ctypes.create_string_buffer(n + 1)
    lib.mc_debug_expr_jit_source(h, buf, n + 1)
    return buf.value.decode()


@pytest.mark.parametrize("model", list(MODELS))
def test_jit_compiles(model):
    from mlx_mcmc_amd import _lib

    lib = _lib.load()
    lp, init = MODELS[model](W.ns_product())
    h = host_program(lp, init)
    try:
        src = _source(h)
        assert "mc_jit_expr" in src and "ex_fwd(" in src and "ex_bwd(" in src
        for k in KERNELS if model in ("logistic", "varying_slopes") else KERNELS[:1]:
            rc = lib.mc_debug_expr_jit_compile(h, k.encode())
            assert rc == 0, (lib.mc_last_error() or b"").decode()
    finally:
        lib.mc_program_destroy(h)


def test_jit_source_is_data_independent():
    from mlx_mcmc_amd import _lib

    lib = _lib.load()
    srcs = []
    for n in (500, 3000):
        lp, init = W.logistic_regression(W.ns_product(), n)
        h = host_program(lp, init)
        srcs.append(_source(h))
        lib.mc_program_destroy(h)
    assert srcs[0] == srcs[1]


def _lane_source(h):
    from mlx_mcmc_amd import _lib

    lib = _lib.load()
    n = lib.mc_debug_expr_jit_lane_source(h, None, 0)
    buf = ctypes.create_string_buffer(n + 1)
    lib.mc_debug_expr_jit_lane_source(h, buf, n + 1)
    return buf.value.decode()


@pytest.mark.parametrize("model,nsh", [("logistic", 3), ("two_predictor", 4), ("huber", 3)])
def test_lane_expression_source_compiles(model, nsh):
    """GLM expression programs sliced onto the lane-resident layout (lanes.h
    LS_EXPR): the host planner takes them, and the generated lane code
    (jit.hip gen_lane_term) compiles into k_hmc_lr with the sliced exchange
    (8 slices, 4 waves) and its L2-resident variant, and into the sliced NUTS
    and MH kernels' run-time forms."""
    from mlx_mcmc_amd import _lib

    lib = _lib.load()
    lp, init = MODELS[model](W.ns_product(), 20_000)
    h = host_program(lp, init)
    try:
        assert lib.mc_debug_lane_plan_host(h, 8) == 0, (lib.mc_last_error() or b"").decode()
        src = _lane_source(h)
        assert "mc_jit_lane_expr" in src and "ex2_fwd(" in src and "#include \"mh_sliced.h\"" in src
        kernels = [f"mc::k_hmc_lr<1, {nsh}, 4, false, {xl}>" for xl in ("false", "true")]
        # NUTS and MH: the sliced kernels' run-time forms (one chain per wave)
        kernels += [f"mc::k_nuts_sl<1, {nsh}, 8, 2, -1, false>",
                    f"mc::k_mh_sl<1, {nsh}, 8, 2, -1, true>"]
        for k in kernels:
            rc = lib.mc_debug_expr_jit_compile(h, k.encode())
            assert rc == 0, (k, (lib.mc_last_error() or b"").decode()[:3000])
    finally:
        lib.mc_program_destroy(h)


def test_lane_plan_declines_vector_leaves():
    """An expression with a gathered parameter vector (varying slopes) is not
    a lane-resident expression program: the planner declines it (the tape
    runs it)."""
    from mlx_mcmc_amd import _lib

    lib = _lib.load()
    lp, init = W.varying_slopes(W.ns_product())
    h = host_program(lp, init)
    try:
        assert lib.mc_debug_lane_plan_host(h, 4) != 0
        assert _lane_source(h) == ""
    finally:
        lib.mc_program_destroy(h)
