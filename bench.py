"""bench.py — leapfrog-steps/s (all chains) + ESS/s on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[2], SURVEY §8d "Large"): hierarchical Normal,
D = 1000 parameters (theta[997], mu, tau, sigma), N = 100,000 observations,
HMC with L = 20 leapfrog steps, 256 chains per GPU (configs[3] at N = 8: 2048
chains, 256/GPU; ESS sums and split R-hat over every rank's chains from
[2, D] f64 moment blocks all-reduced over RCCL, diagnostics.chain_diagnostics).
One *step* = one HMC iteration of every chain (L leapfrog steps, fused
gradient tape, accept, sample store) inside the persistent sampler kernel,
which is launched in chunks of --iters-per-launch iterations (default 50).

    python bench.py [--gpus N --steps K --warmup W]     (N > 1: spawns N rank processes)
    torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

Warmup W = untimed warmup iterations of the sampler (the reference's step-size
rule, Q4), preceded by --clock-warm-ms of untimed device work (default
--clock-warm-kind same: the sampler kernel on the measured chain set's own
buffers and workspace, its state then restored bit-exactly, so the timed
iterations compute exactly what they would without it; measured: cold, the
per-iteration time falls from 70-74 to 60 us over the first ~30 ms of sampler
work, profiles/r2/v17_clock_probe.json); K timed sampling iterations
bracketed by barrier + synchronize;
value = sum over ranks of chain-leapfrog-steps / max-over-ranks wall time.
The initial step size defaults to the one the reference's warmup rule reaches
on this model after the SURVEY's W = 500 (mean over 256 chains,
profiles/r1/v9_bench.json), so short driver runs (W = 5) sample with moving
chains instead of the blow-up regime of eps = 0.01.  Rank 0 prints one JSON
line; a cross-workgroup exchange timeout ends the run with a non-zero status
and no result line.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "leapfrog-steps/sec (all chains) + ESS/sec, 1000-dim Gaussian @1/2/4/8 GPUs"
FP32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 vector = f32-MFMA peak
HBM_PEAK_GBS = 8000.0
# mean step size over 256 chains after the reference's warmup rule (hmc.py:157-170)
# ran W = 500 iterations from eps0 = 0.01 on the Large model (profiles/r1/v9_bench.json)
CONVERGED_EPS = 6.1458e-4


def _ensure_pkg():
    import __graft_entry__ as ge

    return ge._ensure_pkg()


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)   # S = 1000
    ap.add_argument("--warmup", type=int, default=500)   #   and W = 500
    ap.add_argument("--shape", default="large", choices=["small", "medium", "large"])
    ap.add_argument("--chains", type=int, default=256, help="chains per GPU")
    ap.add_argument("--leapfrog", type=int, default=20)
    ap.add_argument("--step-size", type=float, default=CONVERGED_EPS,
                    help="initial step size (default: the reference warmup rule's converged "
                         "value on the Large model after W = 500, profiles/r1/v9_bench.json)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="budget of the CPU-oracle baseline sample (rank 0, N=1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-procs", type=int, default=-1,
                    help="processes of the aggregate CPU baseline (-1: min(15, cpu count): "
                         "the GPU box's CPU share is 16 and its process guard allows 16 "
                         "processes with the GPU device open, which torch's import in each "
                         "worker counts as, this one included; 0: skip)")
    ap.add_argument("--no-ess", action="store_true")
    ap.add_argument("--ess-draws", type=int, default=5000,
                    help="draws of the converged-ESS run (every rank runs its shard of the global "
                         "chains; untimed by the headline: fixed eps, R-hat checked); 0: skip")
    ap.add_argument("--ess-warmup", type=int, default=1000)
    ap.add_argument("--ess-step-size", type=float, default=None,
                    help="fixed step size of the converged-ESS run (default: the posterior "
                         "tests' value for the shape: large 2e-3, medium 5e-3, small 0.01)")
    ap.add_argument("--iters-per-launch", type=int, default=50,
                    help="HMC iterations per sampler launch (hmc() launches its persistent "
                         "kernel in chunks of 500, or once per phase without progress "
                         "output); 1 = one launch per step")
    ap.add_argument("--slices", type=int, default=0,
                    help="data slices per chain (0: the engine's automatic choice)")
    ap.add_argument("--slice-kernel", default="auto", choices=["auto", "interpreter", "lanes"],
                    help="kernel of the sliced program (csrc/lanes.h or csrc/sliced.h)")
    ap.add_argument("--gather", action="store_true",
                    help="also gather every rank's samples to rank 0 over RCCL (untimed)")
    ap.add_argument("--clock-warm-ms", type=float, default=500.0,
                    help="untimed device work before the sampler warmup (--clock-warm-kind; "
                         "the measured state is never changed by it): cold, the sampler's "
                         "first ~30 ms run 15-20 %% slower, so a short run (the driver's "
                         "--warmup 5) would otherwise time the cold kernel; 0: off")
    ap.add_argument("--clock-warm-kind", default="same", choices=["gemm", "sampler", "same"],
                    help="gemm: bf16 GEMMs; sampler: the sampler kernel on a throw-away chain "
                         "set of the same program (its own state, seed and sample buffer); "
                         "same: the sampler kernel on the measured chain set's buffers and "
                         "workspace, its state restored bit-exactly afterwards")
    ap.add_argument("--nuts-model", default="illcond", choices=["illcond", "hier"],
                    help="--workload nuts: illcond = BASELINE configs[4]'s 100-dim kappa = 1000 "
                         "Gaussian; hier = the hierarchical model of --shape (the README rows)")
    ap.add_argument("--nuts-step-size", type=float, default=None,
                    help="NUTS initial step size (dual averaging adapts it over the warmup; "
                         "default 0.1 illcond, 2e-3 hier)")
    ap.add_argument("--mh-scale", type=float, default=1e-3,
                    help="--workload mh: the random-walk proposal scale")
    ap.add_argument("--workload", default="hmc", choices=["hmc", "nuts", "mh"],
                    help="hmc: the headline (BASELINE configs[2]/[3]); nuts: BASELINE "
                         "configs[4] (NUTS depth 10 + dual averaging, 100-dim kappa = 1000 "
                         "Gaussian, 64 chains per GPU; a measurement line, not the headline)")
    args = ap.parse_args()
    if args.ess_step_size is None:
        args.ess_step_size = {"large": 2e-3, "medium": 5e-3, "small": 0.01}[args.shape]
    if args.workload == "nuts" and not any(a.startswith("--chains") for a in sys.argv[1:]):
        args.chains = 64
    if args.nuts_step_size is None:
        args.nuts_step_size = 0.1 if args.nuts_model == "illcond" else 2e-3
    return args


def cpu_model() -> str:
    """lscpu's model name of the host."""
    import subprocess

    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_single(G, N, L, step_size, budget_s, chain=0):
    """Time the CPU oracle (reference cost structure) on the same model, 1 chain, 1 thread."""
    import torch

    import workloads as W
    from oracle import philox as R
    from oracle import samplers as S

    torch.set_num_threads(1)
    lp, init = W.hierarchical(W.ns_oracle(), G, N)
    M = S.EagerModel(lp, init)
    q = M.flatten(init)
    steps = 0
    iters = 0
    t0 = time.perf_counter()
    # one HMC iteration = momentum, L two-gradient leapfrog steps, accept
    while time.perf_counter() - t0 < budget_s:
        p = R.momentum(0, chain, iters, M.D)
        H0 = M.hamiltonian(q, p)
        qp, pp = q, p
        for _ in range(L):
            qp, pp = M.leapfrog(qp, pp, step_size)
            steps += 1
        H1 = M.hamiltonian(qp, pp)
        if R.logf_u01(R.uniform(0, chain, iters, R.TAG_ACCEPT)) < -(H1 - H0):
            q = qp
        iters += 1
    dt = time.perf_counter() - t0
    return {"value": steps / dt, "iterations": iters, "seconds": dt}


def _cpu_worker(a):
    """One process of the aggregate CPU baseline (spawned: no GPU state)."""
    G, N, L, step_size, budget_s, seed = a
    import torch

    torch.set_num_threads(1)
    return cpu_single(G, N, L, step_size, budget_s, chain=seed)["value"]


def cpu_aggregate(G, N, L, step_size, budget_s, nproc):
    """nproc independent single-thread oracle processes, one
    chain each; aggregate chain-steps/s."""
    import multiprocessing as mp

    # the workers are CPU-only: hide the GPU from them (spawned children copy
    # the environment when the pool starts)
    hide = ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES")
    saved = {k: os.environ.get(k) for k in hide}
    for k in hide:
        os.environ[k] = ""
    try:
        ctx = mp.get_context("spawn")
        pool = ctx.Pool(nproc)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    # close + join (workers exit on their own) rather than the context
    # manager's terminate(): SIGTERMed workers print abort traces that would
    # hide a real abort in a profiler log
    try:
        vals = pool.map(_cpu_worker, [(G, N, L, step_size, budget_s, i) for i in range(nproc)])
    finally:
        pool.close()
        pool.join()
    return float(sum(vals))


def cpu_baseline(G, N, L, step_size, budget_s, nproc, gpu_value):
    """The `cpu_baseline` object: the oracle's HMC (reference cost structure:
    two gradients per leapfrog step, a Python iteration loop) on nproc
    single-thread processes (the baseline the >= 10x target
    is quoted against), plus one process alone (8d (i))."""
    one = cpu_single(G, N, L, step_size, budget_s)
    ncpu = os.cpu_count()
    out = {"unit": "leapfrog-steps/s", "kind": "port", "cpu_model": cpu_model(),
           "os_cpu_count": ncpu,
           "single_thread": {"value": one["value"], "cores": 1,
                             "gpu_over_cpu": gpu_value / one["value"],
                             "sample": (f"1 chain, 1 thread, {one['iterations']} iterations x "
                                        f"L={L}, {one['seconds']:.1f} s")}}
    if nproc > 0:
        agg = cpu_aggregate(G, N, L, step_size, budget_s / 2, nproc)
        out.update(value=agg, cores=nproc, gpu_over_cpu=gpu_value / agg,
                   sample=(f"oracle/samplers.py HMC restatement (torch-CPU autograd, 2 gradients "
                           f"per leapfrog step) on the same D={G + 3}, N={N} model at "
                           f"eps={step_size:.3g}, L={L}: {nproc} spawned single-thread "
                           f"processes, one chain each, {budget_s / 2:.1f} s each "
                           f"(SURVEY 8d (ii); the GPU box's CPU share is 16 of os.cpu_count()="
                           f"{ncpu}, and its process guard caps processes with the GPU device "
                           f"open at 16, this one included)"))
    else:
        out.update(value=one["value"], cores=1, gpu_over_cpu=gpu_value / one["value"],
                   sample=out["single_thread"]["sample"])
    return out


def kernel_label(prog, C):
    """The sampler kernel a launch runs (rocprof names it the same way)."""
    kind = prog.slice_kernel
    if kind == "lanes":
        name = "k_hmc_lf" if prog.lanes_fast else "k_hmc_lr"
        return f"{name} (S={prog.num_slices} slices, lane-resident)"
    if kind == "interpreter":
        return f"k_hmc_sl<{16 if C > 8 else 8}> (S={prog.num_slices} slices)"
    return f"k_hmc<{prog.waves_per_chain}>"


def pmc_traffic(shape, iters_per_launch):
    """HBM bytes per launch of `iters_per_launch` iterations from
    profiles/pmc_traffic.json (scripts/pmc_traffic.py): records keyed
    "<shape>@<iters per launch>" (HMC; "nuts-<model>[-<shape>]" and
    "mh-<shape>" for the other lines), measured at that launch size (a launch
    has fixed bytes — the slice blocks are loaded once per launch — so a
    record of another size is not rescaled).  (None, reason) when absent."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        data = json.load(open(path))
    except (OSError, ValueError):
        return None, "no profiles/pmc_traffic.json"
    key = f"{shape}@{iters_per_launch}"
    rec = data.get(key)
    if rec is None:
        return None, f"no PMC record for {key}"
    return rec.get("hbm_bytes_per_launch"), f"profiles/pmc_traffic.json[{key}] ({rec.get('profile', '')})"


def ess_block(samples, accept_n, K, elapsed):
    """ESS/s over the timed draws (reference rule, examples/06_nuts_comparison.py:22-41,
    summed over chains) — published only from chains that moved, with at least
    100 draws and split R-hat max <= 1.1; otherwise null with the reason.
    Under torch.distributed every rank passes its own shard: the per-element
    moment blocks are all-reduced (diagnostics.chain_diagnostics), so the
    result covers every rank's moving chains and every rank takes the same
    branch; `elapsed` is the max-over-ranks wall time."""
    import numpy as np
    import torch

    from mlx_mcmc_amd.diagnostics import chain_diagnostics
    from mlx_mcmc_amd.distributed import sum_over_ranks

    moving = np.nonzero(accept_n > 0)[0]
    n_moving = int(sum_over_ranks(float(moving.size), device=samples.device))
    n_all = int(sum_over_ranks(float(accept_n.size), device=samples.device))
    out = {"draws": K, "chains_used": n_moving, "frozen_chains": n_all - n_moving}
    if K < 100:
        out["ess_per_sec"] = None
        out["ess_null_reason"] = f"{K} timed draws < 100"
        return out
    if n_moving < 2:
        out["ess_per_sec"] = None
        out["ess_null_reason"] = "fewer than two chains accepted a proposal"
        return out
    idx = torch.from_numpy(moving).to(samples.device)
    d = chain_diagnostics(samples[:, :K, :].index_select(0, idx))
    rh = d["rhat"]
    out["rhat"] = {"max": float(np.nanmax(rh)), "median": float(np.nanmedian(rh)), "split": True}
    if d["n_constant"] or not np.isfinite(rh).all() or np.nanmax(rh) > 1.1:
        out["ess_per_sec"] = None
        out["ess_null_reason"] = (f"split R-hat max {np.nanmax(rh):.3g} > 1.1 over the {K} timed "
                                  f"draws of {n_moving} moving chains (and {d['n_constant']} "
                                  "constant series): the draws are not yet from the posterior")
        return out
    # (counted over every rank: each rank takes the same branch)
    if d["n_nonpositive_ess"] > 0:
        out["ess_per_sec"] = None
        out["ess_null_reason"] = (f"the reference ESS rule gives {d['n_nonpositive_ess']} "
                                  "non-positive per-chain ESS values (antithetic draws)")
        return out
    out["ess_per_sec"] = {"min": float(d["ess_sum"].min()) / elapsed,
                          "median": float(np.median(d["ess_sum"])) / elapsed,
                          "unit": "effective samples/s (sum over moving chains of every rank)"}
    return out


def converged_ess(prog, C, q0, dev, L, args, chain_offset=0, world=1):
    """ESS/s where the draws are from the posterior: the same kernel, model and
    chain count at the fixed step size of the posterior tests (eps = 2e-3,
    tests/test_gpu_posterior_exact.py: accept ~0.98), W = --ess-warmup,
    S = --ess-draws sampling iterations timed; reported only with split R-hat
    max <= 1.1.  ESS/s over the sampling seconds and over warmup + sampling
    (SURVEY 8d).  Multi-rank: rank r runs its shard of the global chains
    (chain_offset), the phases are bracketed by barriers and timed as the max
    over ranks, and ESS sums / R-hat come from the all-reduced moment blocks —
    so the line equals a one-rank run over the same global chains up to the
    f64 summation order."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from mlx_mcmc_amd import _engine
    from mlx_mcmc_amd.diagnostics import chain_diagnostics
    from mlx_mcmc_amd.distributed import max_over_ranks

    S, Wm, eps = args.ess_draws, args.ess_warmup, args.ess_step_size
    chains = _engine.ChainSet(prog, C, q0, eps, device=dev)
    samples = torch.empty((C, S, prog.D), dtype=torch.float32, device=dev)
    cfg = dict(chain_offset=chain_offset, num_warmup=Wm, num_samples=S, sample_begin=0,
               sample_capacity=S, seed=args.seed + 1, step_size=eps, target_accept=0.8,
               num_leapfrog_steps=L, adapt_step_size=False)

    def sync():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    sync()
    t0 = time.perf_counter()
    for it0 in range(0, Wm, 500):
        chains.run_hmc(samples=samples, iter_begin=it0, iter_count=min(500, Wm - it0), **cfg)
    sync()
    t1 = time.perf_counter()
    for it0 in range(Wm, Wm + S, 500):
        chains.run_hmc(samples=samples, iter_begin=it0, iter_count=min(500, Wm + S - it0), **cfg)
    sync()
    t2 = time.perf_counter()
    check(chains, "converged-ESS run")
    warm_s = max_over_ranks(t1 - t0, device=dev)
    samp_s = max_over_ranks(t2 - t1, device=dev)
    sc = chains.scalars()
    acc = np.array([np.sum(sc["n_accept"]), np.sum(sc["n_total"])], np.float64)
    if world > 1:
        from mlx_mcmc_amd.distributed import sum_over_ranks

        acc = np.array([sum_over_ranks(float(v), device=dev) for v in acc])
    d = chain_diagnostics(samples)
    rh = d["rhat"]
    out = {"step_size": eps, "warmup": Wm, "draws": S, "chains": C * world,
           "accept_rate": float(acc[0] / max(acc[1], 1.0)),
           "sampling_s": samp_s, "warmup_s": warm_s,
           "rhat": {"max": float(np.nanmax(rh)), "median": float(np.nanmedian(rh)), "split": True}}
    t0, t1, t2 = 0.0, warm_s, warm_s + samp_s
    if d["n_constant"] or not np.isfinite(rh).all() or np.nanmax(rh) > 1.1:
        out["ess_per_sec"] = None
        out["ess_null_reason"] = f"split R-hat max {np.nanmax(rh):.3g} > 1.1"
    elif d["n_nonpositive_ess"] > 0:
        # the reference rule (examples/06_nuts_comparison.py:22-41) keeps the
        # first autocorrelation below 0.05 even when it is strongly negative
        # (antithetic HMC draws), which makes n / (1 + 2 sum rho) negative;
        # counted over every rank, so every rank takes this branch together
        out["ess_per_sec"] = None
        out["ess_null_reason"] = (f"the reference ESS rule gives {d['n_nonpositive_ess']} "
                                  "non-positive per-chain ESS values (antithetic draws)")
    else:
        e = d["ess_sum"]
        out["ess_per_sec"] = {"min": float(e.min()) / (t2 - t1),
                              "median": float(np.median(e)) / (t2 - t1),
                              "min_over_warmup_and_sampling": float(e.min()) / (t2 - t0),
                              "unit": "effective samples/s (sum over chains, reference rule)"}
        out["ess_sum"] = {"min": float(e.min()), "median": float(np.median(e)),
                          "total": float(np.sum(e))}
        out["rhat"]["mean"] = float(np.nanmean(rh))
    del chains, samples
    return out


_STAGES = []


def stage(name):
    """MC_BENCH_STAGES=1: host timestamps of the bench's phases (stderr), to
    see the idle gaps before the timed region (the clock drops after ~3 ms)."""
    if os.environ.get("MC_BENCH_STAGES"):
        _STAGES.append((name, time.perf_counter()))


def print_stages():
    if _STAGES:
        t0 = _STAGES[0][1]
        print("stages (ms): " + ", ".join(f"{n} {1e3 * (t - t0):.2f}" for n, t in _STAGES),
              file=sys.stderr)


def check(chains, where):
    """A sliced launch whose cross-workgroup exchange timed out skipped work:
    report it and exit non-zero rather than publish a number for it."""
    from mlx_mcmc_amd import _lib

    try:
        chains.check_status()
    except _lib.EngineError as e:
        print(f"bench.py: sampler failed in the {where}: {e}", file=sys.stderr, flush=True)
        sys.exit(3)


def clock_warm(ms, dev, scratch=None):
    """Keep the device busy for `ms` milliseconds with work unrelated to the
    measured chains (the GPU raises its clock under sustained load).
    `scratch(n)` (kind "sampler"): n iterations of the same kernel on a
    throw-away chain set; otherwise bf16 GEMMs."""
    import torch

    if ms <= 0:
        return
    if scratch is not None:
        t0 = time.perf_counter()
        while (time.perf_counter() - t0) * 1e3 < ms:
            scratch(10)
            torch.cuda.synchronize()
        return
    a = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        for _ in range(10):
            a = (a @ a).clamp_(-1.0, 1.0)
        torch.cuda.synchronize()
    del a


def init_ranks():
    """One process per GPU (torchrun): RCCL over the node's GPUs.  With
    MC_DIST_BACKEND=gloo the ranks may share GPUs (rank r on GPU r % count): a
    rehearsal of the multi-rank path on a one-GPU box, collectives on host
    copies."""
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("MC_DIST_BACKEND", "nccl")
    gpu = local % max(1, torch.cuda.device_count()) if backend == "gloo" else local
    if world > 1:
        torch.cuda.set_device(gpu)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
    return world, rank, local, torch.device("cuda", gpu)


NUTS_D = 100
# SURVEY 8d unit for NUTS: one leaf (leapfrog step + gradient + Hamiltonian);
# algorithmic FP32 flops per leaf of the D-dim diagonal Gaussian: kicks and
# drift 6D, kinetic energy 2D, the Normal tape with a per-element scale 7D
# (d, d^2, 0.5 d^2, / var, c0 - log s, -, d / var), U-turn dot products at the
# merges <= 4D amortised
NUTS_FLOPS_PER_LEAF = 19 * NUTS_D


def nuts_model(args, ns):
    """(log_prob, init, D, flops per leaf, label) of the NUTS line's model."""
    import workloads as W

    if args.nuts_model == "illcond":
        lp, init = W.illcond_normal(ns, NUTS_D)
        return lp, init, NUTS_D, NUTS_FLOPS_PER_LEAF, f"D={NUTS_D} kappa=1000 Gaussian"
    G, N = W.SHAPES[args.shape]
    lp, init = W.hierarchical(ns, G, N)
    # a leaf = one leapfrog step: the gradient's 5N + 13D flops
    return (lp, init, G + 3, W.hierarchical_flops_per_step(G, N),
            f"hierarchical '{args.shape}' D={G + 3}, N={N}")


def nuts_cpu_baseline(budget_s, args):
    """The oracle's NUTS (reference cost structure: two gradients per leaf,
    recursive build_tree) on the same model, one chain, one thread: leaves/s."""
    import torch

    import workloads as W
    from oracle import samplers as S

    torch.set_num_threads(1)
    lp, init, D, _, label = nuts_model(args, W.ns_oracle())
    leaves, t0, runs = 0, time.perf_counter(), 0
    while time.perf_counter() - t0 < budget_s:
        r = S.nuts(lp, init, num_samples=20, num_warmup=20, step_size=args.nuts_step_size,
                   max_tree_depth=10, seed=runs)
        leaves += int(sum(r.trace["leaves"]))
        runs += 1
    dt = time.perf_counter() - t0
    return {"value": leaves / dt, "unit": "leaf-steps/s", "cores": 1, "kind": "port",
            "cpu_model": cpu_model(), "os_cpu_count": os.cpu_count(),
            "sample": (f"oracle/samplers.py NUTS restatement (torch-CPU autograd, 2 gradients per "
                       f"leaf), 1 chain, 1 thread: {runs} runs of 20 warmup + 20 sampling "
                       f"iterations (depth <= 10) on the same {label} model, {leaves} leaves "
                       f"in {dt:.1f} s (a run in progress at the budget's end finishes)")}


def nuts_kernel_name(prog) -> str:
    k = prog.nuts_kernel(10)
    if k == "sliced":
        return (f"k_nuts_sl (sliced lane-resident NUTS, one chain per wave, "
                f"{prog.num_slices} slices)")
    if k == "lanes":
        return ("k_nuts_lr (lane-resident, one chain per wave, register-only variant)"
                if prog.nuts_register_only(10) else "k_nuts_lr (lane-resident, one chain per wave)")
    return f"k_nuts<{prog.waves_per_chain}>"


def nuts_waves_per_chain(prog) -> int:
    k = prog.nuts_kernel(10)
    return prog.num_slices if k == "sliced" else (1 if k == "lanes" else prog.waves_per_chain)


def main_nuts(args):
    """BASELINE configs[4]: NUTS (depth 10, dual averaging) on the 100-dim
    kappa = 1000 Gaussian; value = leaves (leapfrog steps) of all chains per
    second over the timed sampling iterations."""
    import numpy as np
    import torch
    import torch.distributed as dist

    _ensure_pkg()
    import workloads as W
    from mlx_mcmc_amd import _engine, _trace
    from mlx_mcmc_amd.distributed import max_over_ranks, shard, sum_over_ranks

    world, rank, local, dev = init_ranks()
    C, K, Wm, B = args.chains, args.steps, args.warmup, max(1, args.iters_per_launch)
    lp_fn, init, D, flops_per_leaf, label = nuts_model(args, W.ns_product())
    prog = _trace.compile_model(lp_fn, init, slices=args.slices)
    eps0 = args.nuts_step_size
    chains = _engine.ChainSet(prog, C, prog.layout.flatten(init), eps0, device=dev)
    samples = torch.empty((C, max(K, 1), D), dtype=torch.float32, device=dev)
    chain_offset, _ = shard(C * world, world, rank)
    cfg = dict(chain_offset=chain_offset, num_warmup=Wm, num_samples=K, sample_begin=0,
               sample_capacity=K, seed=args.seed, step_size=eps0, target_accept=0.8,
               max_tree_depth=10, adapt_step_size=True, slice_mode=0)

    def launches(first, count):
        return [(first + i, min(B, count - i)) for i in range(0, count, B)]

    clock_warm(args.clock_warm_ms, dev)
    for it0, n in launches(0, Wm):
        chains.run_nuts(samples=samples, iter_begin=it0, iter_count=n, **cfg)
    torch.cuda.synchronize()
    g0 = chains.scalars()["n_grad"].astype(np.int64)
    stream = torch.cuda.current_stream()
    timed = launches(Wm, K)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in timed]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for (it0, n), (e0, e1) in zip(timed, ev):
        e0.record(stream)
        chains.run_nuts(samples=samples, iter_begin=it0, iter_count=n, **cfg)
        e1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    sc = chains.scalars()
    per = sc["n_grad"].astype(np.int64) - g0
    leaves = int(np.sum(per))
    full = [a.elapsed_time(b) for (a, b), (_, n) in zip(ev, timed) if n == B] or \
           [a.elapsed_time(b) for (a, b), _ in zip(ev, timed)]
    launch_ms = float(np.mean(full)) if K else float("nan")
    launch_ms_total = float(sum(a.elapsed_time(b) for a, b in ev))
    elapsed = max_over_ranks(elapsed, device=dev)
    leaves_all = int(sum_over_ranks(float(leaves), device=dev))   # every rank's chains
    # ESS/s of the timed draws (the metric's second half; every chain's
    # draws — a NUTS step always returns a state of its trajectory — with the
    # same R-hat gate as the HMC line; collective under torch.distributed)
    ess = ess_block(samples, np.ones(C, np.int64), K, elapsed)
    if rank == 0:
        value = leaves_all / elapsed
        # per launch: the timed leaves spread over the launches by their time
        leaves_per_launch = leaves * (launch_ms / launch_ms_total) if launch_ms_total else 0.0
        achieved = leaves_per_launch * flops_per_leaf / (launch_ms * 1e-3) / 1e12
        hier = args.nuts_model == "hier"
        traffic, traffic_src = pmc_traffic(
            f"nuts-{args.nuts_model}" + (f"-{args.shape}" if hier else ""), min(B, K))
        out = {
            "metric": ("leapfrog-steps/sec (all chains), NUTS " +
                       (label if hier else "100-dim kappa=1000 Gaussian")),
            "value": value, "unit": "leaf-steps/s", "n_gpus": world, "steps": K,
            "warmup": Wm, "ms_per_step": elapsed * 1e3 / max(K, 1), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": ("synthetic (fixed-seed hierarchical Normal data, SURVEY §8d)" if hier else
                     "synthetic (fixed kappa = 1000 diagonal scales, SURVEY §8d config 5)"),
            "config": {"workload": (f"NUTS depth 10 + dual averaging on the {label} model, "
                                    f"{C} chains per GPU" if hier else
                                    f"NUTS depth 10 + dual averaging (BASELINE configs[4]): "
                                    f"D={NUTS_D}, kappa=1000, {C} chains per GPU"),
                       "num_params": D, "max_tree_depth": 10, "chains_per_gpu": C,
                       "total_chains": C * world, "parallelism": f"chains sharded {C}/GPU"},
            "roofline": {
                "bound": "valu_fp32", "achieved": achieved, "peak": FP32_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": achieved / FP32_PEAK_TFLOPS, "traffic": traffic,
                "traffic_source": traffic_src,
                "kernel": nuts_kernel_name(prog),
                "launch_ms": launch_ms,
                "iters_per_launch": B, "flops_per_leaf": flops_per_leaf,
                "note": (f"{C} chains = {C * nuts_waves_per_chain(prog)} waves on 1024 SIMDs; "
                         + ("F = 5N + 13D flops per leaf (one gradient of the hierarchical "
                            "model)" if hier else "F = 19 D flops per leaf")
                         + " (SURVEY 8d unit: one leaf)")},
            "leaves": leaves_all, "leaves_rank0": leaves, "mean_tree_depth": float(np.mean(sc["depth_sum"] / np.maximum(
                sc["n_total"], 1))),
            # a launch lasts as long as its longest chain: the per-chain
            # leaves of the timed window (rank 0), and mean / max — the share
            # of the chain slots that stay busy (scripts/probe_nuts_balance.py)
            "chain_balance": {"min": int(per.min()), "median": float(np.median(per)),
                              "max": int(per.max()), "mean_over_max": float(per.mean() / max(per.max(), 1)),
                              "step_size_min": float(np.min(sc["step_size"])),
                              "step_size_median": float(np.median(sc["step_size"]))},
            "accept_stat_mean": float(np.mean(sc["alpha_sum"]) / max(Wm + K, 1)),
            "step_size": float(np.mean(sc["step_size"])),
            "clock_warm_ms": args.clock_warm_ms,
            "ess_per_sec": ess.pop("ess_per_sec"),
            "ess_timed": ess,
        }
        if world == 1 and not args.no_cpu_baseline:
            cb = nuts_cpu_baseline(min(args.cpu_seconds, 15.0), args)
            cb["gpu_over_cpu"] = value / cb["value"]
            out["cpu_baseline"] = cb
        print(json.dumps(out), flush=True)
    del chains, prog, samples
    torch.cuda.synchronize()
    if world > 1:
        dist.destroy_process_group()


def mh_cpu_baseline(budget_s, args, scale):
    """The oracle's MH (metropolis.py restated: one log density per
    iteration, torch CPU) on the same model, one chain, one thread."""
    import torch

    import workloads as W
    from oracle import samplers as S

    torch.set_num_threads(1)
    G, N = W.SHAPES[args.shape]
    lp, init = W.hierarchical(W.ns_oracle(), G, N)
    iters, t0, runs = 0, time.perf_counter(), 0
    while time.perf_counter() - t0 < budget_s:
        S.metropolis_hastings(lp, init, num_samples=20, proposal_scale=scale, random_seed=runs,
                              record=False)
        iters += 20
        runs += 1
    dt = time.perf_counter() - t0
    return {"value": iters / dt, "unit": "chain-iterations/s", "cores": 1, "kind": "port",
            "cpu_model": cpu_model(), "os_cpu_count": os.cpu_count(),
            "sample": (f"oracle/samplers.py metropolis_hastings (torch-CPU log density), 1 chain, "
                       f"1 thread: {runs} runs of 20 iterations on the same hierarchical "
                       f"'{args.shape}' model, {iters} iterations in {dt:.1f} s")}


def main_mh(args):
    """Random-walk Metropolis-Hastings (metropolis.py:6-101, the MCMC.run
    default) on the hierarchical model of --shape: value = chain-iterations
    (proposals evaluated) of all chains per second over the timed launches;
    a measurement line for the sliced MH kernel (k_mh_sl), not the headline."""
    import numpy as np
    import torch
    import torch.distributed as dist

    _ensure_pkg()
    import workloads as W
    from mlx_mcmc_amd import _engine, _lib, _trace
    from mlx_mcmc_amd.distributed import max_over_ranks, shard, sum_over_ranks

    world, rank, local, dev = init_ranks()
    C, K, Wm, B = args.chains, args.steps, args.warmup, max(1, args.iters_per_launch)
    G, N = W.SHAPES[args.shape]
    lp_fn, init = W.hierarchical(W.ns_product(), G, N)
    prog = _trace.compile_model(lp_fn, init, slices=args.slices)
    D = prog.D
    scale = args.mh_scale
    chains = _engine.ChainSet(prog, C, prog.layout.flatten(init), scale, device=dev)
    samples = torch.empty((C, max(K, 1), D), dtype=torch.float32, device=dev)
    chain_offset, _ = shard(C * world, world, rank)
    cfg = dict(chain_offset=chain_offset, num_warmup=Wm, num_samples=K, sample_begin=0,
               sample_capacity=K, seed=args.seed)

    def launches(first, count):
        return [(first + i, min(B, count - i)) for i in range(0, count, B)]

    clock_warm(args.clock_warm_ms, dev)
    for it0, n in launches(0, Wm):
        chains.run_mh(proposal_scale=scale, samples=samples, iter_begin=it0, iter_count=n, **cfg)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    timed = launches(Wm, K)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in timed]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for (it0, n), (e0, e1) in zip(timed, ev):
        e0.record(stream)
        chains.run_mh(proposal_scale=scale, samples=samples, iter_begin=it0, iter_count=n, **cfg)
        e1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    check(chains, "MH timed region")
    sc = chains.scalars()
    full = [a.elapsed_time(b) for (a, b), (_, n) in zip(ev, timed) if n == B] or \
           [a.elapsed_time(b) for (a, b), _ in zip(ev, timed)]
    launch_ms = float(np.mean(full)) if K else float("nan")
    iters_per_launch = min(B, K)
    elapsed = max_over_ranks(elapsed, device=dev)
    total = sum_over_ranks(float(C * K), device=dev)
    if rank == 0:
        value = total / elapsed
        # F = 3N + 10D flops per chain-iteration: the swept term's sum of
        # squares (d = x - theta, fma: 3 per element), the proposal (2 per
        # parameter), the direct term (~8 per parameter)
        flops = 3 * N + 10 * D
        achieved = C * iters_per_launch * flops / (launch_ms * 1e-3) / 1e12
        traffic, traffic_src = pmc_traffic(f"mh-{args.shape}", iters_per_launch)
        kern = ("k_mh_sl (sliced lane-resident MH, one chain per wave, "
                f"{prog.num_slices} slices)" if _lib.load().mc_program_mh_sliced(prog.handle) == 1
                else f"k_mh<{prog.waves_per_chain}>")
        out = {
            "metric": f"MH chain-iterations/sec (all chains), hierarchical '{args.shape}' D={D}, N={N}",
            "value": value, "unit": "chain-iterations/s", "n_gpus": world, "steps": K,
            "warmup": Wm, "ms_per_step": elapsed * 1e3 / max(K, 1), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (fixed-seed hierarchical Normal data, SURVEY §8d)",
            "config": {"workload": (f"random-walk MH (metropolis.py) on the hierarchical "
                                    f"'{args.shape}' model, proposal scale {scale}, {C} chains "
                                    f"per GPU"),
                       "num_params": D, "num_obs": N, "chains_per_gpu": C,
                       "total_chains": C * world, "parallelism": f"chains sharded {C}/GPU"},
            "roofline": {"bound": "valu_fp32", "achieved": achieved, "peak": FP32_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": achieved / FP32_PEAK_TFLOPS, "traffic": traffic,
                         "traffic_source": traffic_src,
                         "kernel": kern, "launch_ms": launch_ms,
                         "iters_per_launch": iters_per_launch, "flops_per_iteration": flops},
            "accept_rate": float(np.mean(sc["n_accept"] / np.maximum(sc["n_total"], 1))),
            "clock_warm_ms": args.clock_warm_ms,
        }
        if world == 1 and not args.no_cpu_baseline:
            cb = mh_cpu_baseline(min(args.cpu_seconds, 15.0), args, scale)
            cb["gpu_over_cpu"] = value / cb["value"]
            out["cpu_baseline"] = cb
        print(json.dumps(out), flush=True)
    del chains, prog, samples
    torch.cuda.synchronize()
    if world > 1:
        dist.destroy_process_group()


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_command(argv):
    """The command line one spawned rank runs: this script, same arguments."""
    return [sys.executable, os.path.abspath(__file__)] + list(argv)


def spawn_ranks(n, argv, cmd=None, poll_s=0.2):
    """`bench.py --gpus N` without a launcher: start N fresh rank processes
    (rank r on GPU r, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set per child,
    the same arguments) and wait for them.  The parent never imports torch or
    opens the device — every rank initialises HIP itself — so this is the
    torchrun layout (one process per GPU) by construction.  Rank 0's JSON line
    reaches stdout directly (the children inherit it; other ranks print no
    result line).  When a rank fails the others are stopped (they would wait
    in a collective for it) and the first non-zero status is returned."""
    import subprocess

    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), MC_BENCH_SPAWNED="1")
        procs.append(subprocess.Popen(cmd if cmd is not None else rank_command(argv), env=env))
    status = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 128 - rc
                print(f"bench.py: rank {procs.index(p)} exited with status {rc}; stopping the "
                      f"other ranks", file=sys.stderr, flush=True)
                for q in live:
                    q.terminate()
                for q in live:
                    try:
                        q.wait(timeout=20)
                    except subprocess.TimeoutExpired:
                        q.kill()
                        q.wait()
                live = []
        time.sleep(poll_s)
    return status


def resolve_world(args):
    """None when this process runs the bench itself; otherwise the exit status
    of the launch: `--gpus N > 1` with no WORLD_SIZE spawns N ranks
    (spawn_ranks); a WORLD_SIZE that disagrees with --gpus is an error (the
    line would report another GPU count than the one asked for)."""
    if args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr)
        return 2
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != args.gpus:
            print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws}: launch one process per "
                  f"GPU with the same count (torchrun --nproc-per-node {args.gpus}), or run "
                  f"without a launcher and let bench.py spawn the ranks", file=sys.stderr)
            return 2
        return None
    if args.gpus > 1:
        return spawn_ranks(args.gpus, sys.argv[1:])
    return None


def main():
    args = parse()
    status = resolve_world(args)
    if status is not None:
        sys.exit(status)
    if args.workload == "nuts":
        return main_nuts(args)
    if args.workload == "mh":
        return main_mh(args)
    import numpy as np
    import torch
    import torch.distributed as dist

    m = _ensure_pkg()
    import workloads as W
    from mlx_mcmc_amd import _engine, _trace
    from mlx_mcmc_amd.distributed import gather_to_root, max_over_ranks, shard

    world, rank, local, dev = init_ranks()

    G, N = W.SHAPES[args.shape]
    D = G + 3
    C = args.chains
    L = args.leapfrog
    K = args.steps
    Wm = args.warmup
    lp_fn, init = W.hierarchical(W.ns_product(), G, N)
    prog = _trace.compile_model(lp_fn, init, slices=args.slices, slice_kernel=args.slice_kernel)
    chains = _engine.ChainSet(prog, C, prog.layout.flatten(init), args.step_size, device=dev)
    samples = torch.empty((C, max(K, 1), D), dtype=torch.float32, device=dev)
    chain_offset, _ = shard(C * world, world, rank)   # weak scaling: C chains per GPU
    cfg = dict(chain_offset=chain_offset, num_warmup=Wm, num_samples=K, sample_begin=0,
               sample_capacity=K, seed=args.seed, step_size=args.step_size,
               target_accept=0.8, num_leapfrog_steps=L, adapt_step_size=True)

    # launches of B iterations (the last one shorter), in the warmup too, so
    # that a kernel-trace profile's average duration is the timed launches'
    B = max(1, args.iters_per_launch)

    def launches(first, count):
        return [(first + i, min(B, count - i)) for i in range(0, count, B)]

    scratch = None
    saved = None
    if args.clock_warm_kind == "same":
        saved = chains.state.clone()
        tmp = chains
    elif args.clock_warm_kind == "sampler":
        tmp = _engine.ChainSet(prog, C, prog.layout.flatten(init), args.step_size, device=dev)
    if args.clock_warm_kind != "gemm":
        tmp_s = torch.empty((C, 10, D), dtype=torch.float32, device=dev)
        tmp_cfg = dict(cfg, seed=args.seed + 7919, num_warmup=0, num_samples=10,
                       sample_capacity=10)

        def scratch(n):
            tmp.run_hmc(samples=tmp_s, iter_begin=0, iter_count=n, **tmp_cfg)
    stage("clock warm")
    clock_warm(args.clock_warm_ms, dev, scratch)
    stage("clock warm done")
    if scratch is not None:
        check(tmp, "clock warm")
        del tmp, tmp_s
    if saved is not None:
        chains.state.copy_(saved)   # the measured chains start from their initial state
        torch.cuda.synchronize()
        del saved
    stage("restored")
    # ---- untimed warmup (step-size adaptation) -------------------------------
    for it0, n in launches(0, Wm):
        chains.run_hmc(samples=samples, iter_begin=it0, iter_count=n, **cfg)
    torch.cuda.synchronize()
    stage("warmup done")
    check(chains, "warmup")
    stage("checked")

    # ---- timed region: K steps in launches of B ---------------------------------
    stream = torch.cuda.current_stream()
    timed = launches(Wm, K)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in timed]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    stage("t0")
    t0 = time.perf_counter()
    for (it0, n), (e0, e1) in zip(timed, ev):
        e0.record(stream)
        chains.run_hmc(samples=samples, iter_begin=it0, iter_count=n, **cfg)
        e1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    stage("t1")
    print_stages()
    check(chains, "timed region")
    # kernel time per launch from the largest launches of the timed region
    # (HIP events on the launch stream): a run of K < B iterations is one
    # K-iteration launch, and every field below describes that launch
    ipl = max((n for _, n in timed), default=0)
    full = [a.elapsed_time(b) for (a, b), (_, n) in zip(ev, timed) if n == ipl]
    launch_ms = float(np.mean(full)) if full else float("nan")
    each_ms = [round(a.elapsed_time(b), 4) for a, b in ev]
    iters_per_launch = max(ipl, 1)
    iter_ms = launch_ms / iters_per_launch
    elapsed = max_over_ranks(elapsed, device=dev)

    sc = chains.scalars()
    accept = float(np.mean(sc["n_accept"] / np.maximum(sc["n_total"], 1)))
    frozen = int(np.sum(sc["n_accept"] == 0)) if K else 0     # chains that never moved
    frozen = int(max_over_ranks(float(frozen), device=dev))
    eps = float(np.mean(sc["step_size"]))

    # ---- diagnostics on the device (not timed) ----------------------------------
    # ESS per (chain, element) with the reference rule and split R-hat over the
    # timed draws of the chains that moved (ess_block says when it is null)
    ess = None
    diag_ms = None
    # (every rank takes part: the moment blocks are all-reduced over RCCL)
    if not args.no_ess and K >= 1:
        td = time.perf_counter()
        ess = ess_block(samples, sc["n_accept"], K, elapsed)
        diag_ms = (time.perf_counter() - td) * 1e3
    ess_conv = None
    if not args.no_ess and args.ess_draws > 0:
        ess_conv = converged_ess(prog, C, prog.layout.flatten(init), dev, L, args,
                                 chain_offset=chain_offset, world=world)
    gather_ms = None
    if world > 1 and args.gather:
        tg = time.perf_counter()
        gather_to_root(samples)
        torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - tg) * 1e3

    if rank == 0:
        total_chains = C * world
        steps_total = total_chains * L * K
        value = steps_total / elapsed
        flops_per_launch = C * L * W.hierarchical_flops_per_step(G, N) * iters_per_launch
        achieved = flops_per_launch / (launch_ms * 1e-3) / 1e12
        traffic, traffic_src = pmc_traffic(args.shape, iters_per_launch)
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "leapfrog-steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": Wm,
            "ms_per_step": elapsed * 1e3 / max(K, 1),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (fixed-seed hierarchical Normal data, SURVEY §8d)",
            "config": {
                "workload": (f"hierarchical Normal '{args.shape}' HMC (BASELINE configs[2]/[3]): "
                             f"D={D}, N={N}, L={L}, {C} chains per GPU"),
                "num_params": D, "num_obs": N, "leapfrog_steps": L, "chains_per_gpu": C,
                "total_chains": total_chains, "parallelism": f"chains sharded {C}/GPU",
                "waves_per_chain": prog.waves_per_chain, "slices": prog.num_slices,
                "step_size0": args.step_size,
                "step_size0_note": (
                    "eps0 = the mean step size the reference's warmup rule (hmc.py:157-170) "
                    "reaches on this model after W = 500 from eps0 = 0.01 (SURVEY 8d's "
                    "setting), so short runs sample moving chains; HMC throughput does not "
                    "depend on eps (L = 20 leapfrog steps per iteration either way)"
                    if args.step_size == CONVERGED_EPS else "eps0 set on the command line"),
            },
            "roofline": {
                "bound": "valu_fp32", "achieved": achieved, "peak": FP32_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": achieved / FP32_PEAK_TFLOPS, "traffic": traffic,
                "kernel": kernel_label(prog, C),
                "iteration_ms": iter_ms,
                "launch_ms": launch_ms,
                "each_launch_ms": each_ms if len(each_ms) <= 25 else None,
                "iters_per_launch": iters_per_launch,
                "flops_per_launch": flops_per_launch,
                "note": ("FP32 VALU bound (SURVEY 8d: no dense contraction, no MFMA; vector FP32 "
                         "peak 157.3 TF); "
                         "F = 5N + 13D flops per chain-leapfrog-step, C*L per iteration, "
                         "iters_per_launch iterations per launch (the largest launch of the "
                         "timed region); launch_ms = HIP events around each such launch on "
                         "its stream, iteration_ms = launch_ms / iters_per_launch; "
                         "traffic = (2*FETCH_SIZE + WRITE_SIZE) per launch of this size from "
                         "profiles/pmc_traffic.json"),
                "traffic_source": traffic_src,
            },
            "accept_rate": accept, "step_size": eps,
            # the data every chain reads per step (8N bytes: y and the
            # group index), times chain-steps/s; chains share it through LDS/L2
            "per_chain_streamed_gbs": 8.0 * N * value / 1e9,
        }
        out["clock_warm_ms"] = args.clock_warm_ms
        out["clock_warm_kind"] = args.clock_warm_kind
        if gather_ms is not None:
            out["gather_ms"] = gather_ms
        out["frozen_chains"] = frozen
        if ess is not None:
            out["ess_per_sec"] = ess.pop("ess_per_sec")
            out["ess_timed"] = ess
            out["diagnostics_ms"] = diag_ms
        if ess_conv is not None:
            out["ess_converged"] = ess_conv
        if world == 1 and not args.no_cpu_baseline:
            nproc = args.cpu_procs if args.cpu_procs >= 0 else min(15, os.cpu_count() or 1)
            out["cpu_baseline"] = cpu_baseline(G, N, L, max(eps, 1e-4), args.cpu_seconds, nproc,
                                               value)
        print(json.dumps(out), flush=True)
    # release the device objects (program, chain state, workspace) before the
    # interpreter's exit handlers run, so nothing calls into HIP after a
    # profiler's teardown
    del chains, prog, samples
    torch.cuda.synchronize()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
