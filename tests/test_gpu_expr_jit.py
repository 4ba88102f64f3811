"""The expression-term JIT on the GPU (csrc/jit.hip, VERDICT r4 "Next round"
3): every expression model of tests/test_gpu_expr.py sampled with the
program's expression terms compiled (hiprtc) and with the interpreter
(mc_debug_expr_jit(0)) — HMC, NUTS and Metropolis-Hastings — gives
bit-identical draws, trace and counters: the generated code performs the
interpreter's operations in the interpreter's order.  The interpreter itself
is held to the CPU oracle by tests/test_gpu_expr.py, which runs on the JIT by
default, so those oracle bars hold for the compiled kernels too."""
import numpy as np
import pytest

import workloads as W
from _jit_models import MODELS

pytestmark = pytest.mark.gpu


def _run(algo, model, jit):
    import mlx_mcmc_amd as m
    from mlx_mcmc_amd import _lib, _trace

    lib = _lib.load()
    lib.mc_debug_expr_jit(1 if jit else 0)
    try:
        lp, init = MODELS[model](W.ns_product())
        if algo == "hmc":
            s, rate, info = m.hmc(lp, init, num_samples=12, num_warmup=12, step_size=0.02,
                                  num_leapfrog_steps=5, key=m.random.key(4), num_chains=16,
                                  progress=False, return_info=True, return_trace=True)
        elif algo == "nuts":
            s, rate, info = m.nuts(lp, init, num_samples=8, num_warmup=8, step_size=0.02,
                                   max_tree_depth=6, key=m.random.key(4), num_chains=16,
                                   progress=False, return_info=True, return_trace=True)
        else:
            s, rate, info = m.metropolis_hastings(lp, init, num_samples=40, proposal_scale=0.05,
                                                  random_seed=4, num_chains=16, return_info=True,
                                                  return_trace=True)
        prog = _trace.compile_model(lp, init)
        state = lib.mc_program_expr_jit(prog.handle)
    finally:
        lib.mc_debug_expr_jit(-1)
    return s, info, state


@pytest.mark.parametrize("algo", ["hmc", "nuts", "mh"])
@pytest.mark.parametrize("model", list(MODELS))
def test_jit_bit_identical_to_interpreter(gpu, model, algo):
    if algo != "hmc" and model not in ("logistic", "varying_slopes", "cauchy"):
        pytest.skip("HMC covers the model; NUTS / MH run on three")
    s0, i0, st0 = _run(algo, model, False)
    s1, i1, st1 = _run(algo, model, True)
    assert st0 == 0 and st1 == 1, (st0, st1)
    for name in s0:
        np.testing.assert_array_equal(np.asarray(s0[name]), np.asarray(s1[name]), err_msg=name)
    for k, v in i0.trace.items():
        np.testing.assert_array_equal(v, i1.trace[k], err_msg=k)
    np.testing.assert_array_equal(i0.step_size, i1.step_size)


def test_jit_throughput_beats_interpreter(gpu):
    """The reason for the JIT: logistic regression at N = 20 K, 64 chains, the
    compiled kernel at least 4x the interpreter's chain-steps/s."""
    import time

    import torch

    from mlx_mcmc_amd import _engine, _lib, _trace

    lib = _lib.load()
    lp, init = W.logistic_regression(W.ns_product(), 20000)
    rates = {}
    for jit in (False, True):
        lib.mc_debug_expr_jit(1 if jit else 0)
        try:
            prog = _trace.compile_model(lp, init)
            cs = _engine.ChainSet(prog, 64, prog.layout.flatten(init), 1e-3)
            smp = torch.empty((64, 1, prog.D), dtype=torch.float32, device=cs.device)
            cfg = dict(chain_offset=0, num_warmup=10 ** 6, num_samples=1, sample_begin=0,
                       sample_capacity=1, seed=0, step_size=1e-3, target_accept=0.8,
                       num_leapfrog_steps=10, adapt_step_size=False)
            cs.run_hmc(samples=smp, iter_begin=0, iter_count=1, **cfg)  # (compiles)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            cs.run_hmc(samples=smp, iter_begin=1, iter_count=4, **cfg)
            torch.cuda.synchronize()
            rates[jit] = 64 * 4 * 10 / (time.perf_counter() - t0)
        finally:
            lib.mc_debug_expr_jit(-1)
    print(f"logistic N=20K: interpreter {rates[False] / 1e6:.3f} M, JIT {rates[True] / 1e6:.3f} M "
          f"chain-steps/s")
    assert rates[True] >= 4 * rates[False], rates
