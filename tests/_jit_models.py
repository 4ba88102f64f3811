"""Expression models for the JIT tests (tests/test_expr_jit_host.py on the
CPU, tests/test_gpu_expr_jit.py on the GPU): the models of
tests/test_gpu_expr.py, and the helper that builds a program's host tables
without a device (mc_debug_program_host_only)."""
import ctypes

import numpy as np

import workloads as W


def tiny_scalar(ns):
    """Only broadcast parameters in small expression terms (the wave-task path)."""
    def log_prob(params):
        a, b = params["a"], params["b"]
        lp = ns.Normal(0, 1).log_prob(a * b) + ns.Normal(a / (1.0 + b * b), 2.0).log_prob(0.3)
        return lp + ns.Normal(0, 3).log_prob(a) + ns.Normal(0, 3).log_prob(b) - 0.1 * ns.square(a - b)

    return log_prob, {"a": np.float32(0.5), "b": np.float32(-0.4)}


MODELS = {"two_predictor": W.two_predictor_regression,
          "logistic": W.logistic_regression,
          "varying_slopes": W.varying_slopes,
          "cauchy": W.cauchy_location,
          "gamma_beta": W.gamma_beta_regression,
          "axis_reductions": W.axis_reductions,
          "huber": W.huber_regression,
          "weighted_indexed": W.weighted_indexed,
          "tempered": W.tempered,
          "tiny_scalar": tiny_scalar}


def host_program(lp, init):
    """mc_program_create_expr on host tables only (never launched)."""
    from mlx_mcmc_amd import _lib, _trace

    lib = _lib.load()
    model = _trace.trace(lp, init)
    h = ctypes.c_void_p()
    data = np.ascontiguousarray(model.data, np.float32)
    index = np.ascontiguousarray(model.index, np.int32)
    lib.mc_debug_program_host_only(1)
    try:
        _lib.check(lib.mc_program_create_expr(
            model.c_terms, len(model.terms), model.c_affines, model.n_affines, model.c_exprs,
            model.n_exprs, model.c_nodes, model.n_nodes, model.layout.size, model.lp_const,
            data.ctypes.data_as(ctypes.c_void_p), data.size,
            index.ctypes.data_as(ctypes.c_void_p), index.size, ctypes.byref(h)))
    finally:
        lib.mc_debug_program_host_only(0)
    return h
