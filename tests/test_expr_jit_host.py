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
