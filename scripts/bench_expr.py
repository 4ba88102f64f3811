"""Throughput of expression programs (MC_DIST_EXPR) against the fused terms
on the same model: HMC chain-leapfrog-steps/s of the kernel alone (HIP
events around the launches, L = 10, 256 chains), plus the host-side trace +
program build time.  The linear regression written two ways — the affine
fused loc and the same likelihood as a hand-written expression — plus the
two-predictor and logistic models."""
import os
import sys
import time
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__)))]
import numpy as np
import torch
import mlx_mcmc_amd as m
import mlx_mcmc_amd.core as mx
import workloads as W
from mlx_mcmc_amd import _engine, _lib, _trace

LIB = _lib.load()


def rate(lp, init, chains=256, L=10, eps=1e-3, iters=20, jit=-1, slices=0):
    """jit: -1 the default (expression terms compiled), 0 the interpreter;
    slices: 0 automatic (N = 100 K: the lane-resident kernel with the
    JIT-compiled LS_EXPR sweep), 1 the chain-per-workgroup tape."""
    LIB.mc_debug_expr_jit(jit)
    t0 = time.perf_counter()
    prog = _trace.compile_model(lp, init, slices=slices)
    t_build = time.perf_counter() - t0
    cs = _engine.ChainSet(prog, chains, prog.layout.flatten(init), eps, device=torch.device("cuda"))
    samples = torch.empty((chains, 1, prog.D), dtype=torch.float32, device="cuda")
    cfg = dict(chain_offset=0, num_warmup=10 ** 6, num_samples=1, sample_begin=0,
               sample_capacity=1, seed=0, step_size=eps, target_accept=0.8,
               num_leapfrog_steps=L, adapt_step_size=False)
    cs.run_hmc(samples=samples, iter_begin=0, iter_count=2, **cfg)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    cs.run_hmc(samples=samples, iter_begin=2, iter_count=iters, **cfg)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    cs.check_status()
    LIB.mc_debug_expr_jit(-1)
    kern = prog.slice_kernel
    if kern == "lanes" and LIB.mc_program_expr_jit(prog.handle) == 1 and any(
            t.dist == _lib.MC_DIST_EXPR for t in prog.model.terms):
        kern = f"lanes + JIT LS_EXPR, {prog.num_slices} slices"
    return chains * iters * L / (ms * 1e-3), t_build, kern


N = 100000
x, y = W.regression_data(N)
X, Y = mx.array(x), mx.array(y)


def fused(p):
    lp = m.Normal(0, 10).log_prob(p["a"]) + m.Normal(0, 10).log_prob(p["b"])
    lp = lp + m.HalfNormal(5).log_prob(p["sigma"])
    return lp + mx.sum(m.Normal(p["a"] + p["b"] * X, p["sigma"]).log_prob(Y))


def handwritten(p):
    lp = m.Normal(0, 10).log_prob(p["a"]) + m.Normal(0, 10).log_prob(p["b"])
    lp = lp + m.HalfNormal(5).log_prob(p["sigma"])
    z = (Y - (p["a"] + p["b"] * X)) / p["sigma"]
    return lp + mx.sum(-0.5 * mx.square(z) - mx.log(p["sigma"]) - 0.9189385)


init = {"a": np.float32(1.5), "b": np.float32(2.0), "sigma": np.float32(0.5)}
for name, f in (("affine fused", fused), ("hand-written expression", handwritten)):
    r, tb, k = rate(f, init)
    print(f"regression N={N} {name}: {r / 1e6:.3f} M chain-steps/s (kernel {k}; build {tb:.2f} s)")
# the varying-intercept regression alpha[g] + beta * x (G = 1000 groups of
# ~100 observations): the affine loc on the lane-resident kernel (lanes.h
# LS_AFF, 16 slices) and, for reference, on the tape (num_slices=1)
G = 1000
lpv, iv = W.varying_intercept(W.ns_product(), G, N)
xv, yv, gv = W.varying_intercept_data(G, N)
iv = dict(iv)
iv["alpha"] = np.array([yv[gv == k].mean() - 0.7 * xv[gv == k].mean() if np.any(gv == k) else 1.0
                        for k in range(G)], np.float32)
for sl, name in ((0, "lane-resident (auto)"), (1, "tape (num_slices=1)")):
    t0 = time.perf_counter()
    prog = _trace.compile_model(lpv, iv, slices=sl)
    tb = time.perf_counter() - t0
    cs = _engine.ChainSet(prog, 256, prog.layout.flatten(iv), 1e-3, device=torch.device("cuda"))
    smp = torch.empty((256, 1, prog.D), dtype=torch.float32, device="cuda")
    cfg = dict(chain_offset=0, num_warmup=10 ** 6, num_samples=1, sample_begin=0,
               sample_capacity=1, seed=0, step_size=1e-3, target_accept=0.8,
               num_leapfrog_steps=10, adapt_step_size=False)
    cs.run_hmc(samples=smp, iter_begin=0, iter_count=2, **cfg)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    it = 20 if sl == 0 else 2
    e0.record()
    cs.run_hmc(samples=smp, iter_begin=2, iter_count=it, **cfg)
    e1.record()
    torch.cuda.synchronize()
    cs.check_status()
    r = 256 * it * 10 / (e0.elapsed_time(e1) * 1e-3)
    print(f"varying intercept G={G} N={N} {name}: {r / 1e6:.3f} M chain-steps/s "
          f"(kernel {prog.slice_kernel}, {prog.num_slices} slices; build {tb:.2f} s)")
    del cs, smp, prog
lp, _ = W.two_predictor_regression(W.ns_product(), N)
i2 = {"a": np.float32(0.5), "b1": np.float32(1.2), "b2": np.float32(-0.8),
      "log_sigma": np.float32(-0.5)}
VARIANTS = ((0, 1, "tape, interpreter"), (-1, 1, "tape, JIT"), (-1, 0, "auto"))
for jit, sl, nm in VARIANTS:
    r, tb, k = rate(lp, i2, jit=jit, slices=sl)
    print(f"two-predictor N={N} expression ({nm}): {r / 1e6:.3f} M chain-steps/s "
          f"(kernel {k}; build {tb:.2f} s)")
lp, _ = W.logistic_regression(W.ns_product(), N)
for jit, sl, nm in VARIANTS:
    r, tb, k = rate(lp, {"a": np.float32(-0.3), "b": np.float32(1.1)}, jit=jit, slices=sl)
    print(f"logistic N={N} expression ({nm}): {r / 1e6:.3f} M chain-steps/s "
          f"(kernel {k}; build {tb:.2f} s)")


def nuts_rate(lp, init, slices, chains=256, eps=2e-3, iters=10, nuts_program=False):
    """NUTS leaf-steps/s (all chains) at a fixed step size: slices 0 = the
    sliced kernel (k_nuts_sl's run-time form JIT-compiled with the expression
    terms), 1 = the tape (k_nuts); nuts_program: the program nuts() runs
    (_trace.nuts_program: affine terms as expression terms)."""
    prog = _trace.compile_model(lp, init, slices=slices)
    if nuts_program:
        prog = _trace.nuts_program(prog, 10)
    kern = prog.nuts_kernel(10)
    cs = _engine.ChainSet(prog, chains, prog.layout.flatten(init), eps,
                          device=torch.device("cuda"))
    cfg = dict(chain_offset=0, num_warmup=10 ** 6, num_samples=0, sample_begin=0,
               sample_capacity=0, seed=0, step_size=eps, target_accept=0.8, max_tree_depth=10,
               adapt_step_size=False, slice_mode=0)
    cs.run_nuts(iter_begin=0, iter_count=2, **cfg)
    torch.cuda.synchronize()
    g0 = cs.scalars()["n_grad"].astype(np.int64).sum()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    cs.run_nuts(iter_begin=2, iter_count=iters, **cfg)
    e1.record()
    torch.cuda.synchronize()
    cs.check_status()
    leaves = cs.scalars()["n_grad"].astype(np.int64).sum() - g0
    return leaves / (e0.elapsed_time(e1) * 1e-3), kern


for name, f, start, eps in (
        ("logistic", W.logistic_regression, {"a": np.float32(-0.3), "b": np.float32(1.1)}, 2e-3),
        ("two-predictor", W.two_predictor_regression, i2, 1e-3)):
    lpn, _ = f(W.ns_product(), N)
    for sl in (0, 1):
        r, k = nuts_rate(lpn, start, sl, eps=eps)
        print(f"{name} N={N} NUTS (fixed eps {eps}): {r / 1e6:.3f} M leaf-steps/s (kernel {k})")

# a fused affine-loc regression: the tape, and the program nuts() runs (the
# affine term as an expression term on the sliced kernel)
start = {"a": np.float32(1.5), "b": np.float32(2.0), "sigma": np.float32(0.5)}
for label, conv in (("fused affine term, tape", False), ("nuts() program", True)):
    r, k = nuts_rate(fused, start, 0, eps=1e-3, nuts_program=conv)
    print(f"regression N={N} NUTS {label} (fixed eps 0.001): {r / 1e6:.3f} M leaf-steps/s "
          f"(kernel {k})")



def mh_rate(lp, init, chains=256, scale=2e-3, iters=200, mh_program=False):
    """Random-walk MH chain-iterations/s (all chains): the compiled program,
    or the one metropolis_hastings() runs (_trace.mh_program)."""
    prog = _trace.compile_model(lp, init)
    if mh_program:
        prog = _trace.mh_program(prog)
    kern = "sliced" if LIB.mc_program_mh_sliced(prog.handle) == 1 else "tape"
    cs = _engine.ChainSet(prog, chains, prog.layout.flatten(init), scale,
                          device=torch.device("cuda"))
    cfg = dict(chain_offset=0, num_warmup=0, num_samples=0, sample_begin=0,
               sample_capacity=0, seed=0)
    cs.run_mh(proposal_scale=scale, iter_begin=0, iter_count=20, **cfg)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    cs.run_mh(proposal_scale=scale, iter_begin=20, iter_count=iters, **cfg)
    e1.record()
    torch.cuda.synchronize()
    cs.check_status()
    return chains * iters / (e0.elapsed_time(e1) * 1e-3), kern


for label, conv in (("fused affine term", False), ("metropolis_hastings() program", True)):
    r, k = mh_rate(fused, start, mh_program=conv)
    print(f"regression N={N} MH {label}: {r / 1e6:.3f} M chain-iterations/s (kernel {k})")
