"""Which kernel each sampler runs for the workload models at a large data
size: HMC (the compiled program's slice kernel), NUTS (_trace.nuts_program)
and MH (_trace.mh_program) — to find models that still fall to the
chain-per-workgroup tape.
    python scripts/probe_kernels.py [N]"""
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__)))]
import __graft_entry__ as ge  # noqa: E402

ge._ensure_pkg()
import workloads as W  # noqa: E402
from mlx_mcmc_amd import _lib, _trace  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
ns = W.ns_product()
MODELS = {
    "linear_regression": lambda: W.linear_regression(ns, N),
    "linear_regression_exp": lambda: W.linear_regression_exp(ns, N),
    "two_predictor": lambda: W.two_predictor_regression(ns, N),
    "logistic": lambda: W.logistic_regression(ns, N),
    "huber": lambda: W.huber_regression(ns, N),
    "varying_intercept": lambda: W.varying_intercept(ns, 1000, N),
    "varying_slopes": lambda: W.varying_slopes(ns, 1000, N),
    "hierarchical": lambda: W.hierarchical(ns, 997, N),
    "hierarchical_reparam": lambda: W.hierarchical_reparam(ns, 997, N),
    "weighted_indexed": lambda: W.weighted_indexed(ns, 64, N),
    "tempered": lambda: W.tempered(ns, N),
    "cauchy": lambda: W.cauchy_location(ns, N),
    "gamma_beta": lambda: W.gamma_beta_regression(ns, N),
}
lib = _lib.load()
for name, mk in MODELS.items():
    try:
        lp, init = mk()
        prog = _trace.compile_model(lp, init)
        hmc = prog.slice_kernel
        nuts = _trace.nuts_program(prog, 10).nuts_kernel(10)
        mp = _trace.mh_program(prog)  # (kept alive while its handle is queried)
        mh = "sliced" if lib.mc_program_mh_sliced(mp.handle) == 1 else "tape"
        note = prog.kernel_note
        print(f"{name:22s} terms {len(prog.model.terms):2d} affine {prog.model.n_affines} "
              f"expr {prog.model.n_exprs}: HMC {hmc:10s} NUTS {nuts:7s} MH {mh:7s} {note[:70]}",
              flush=True)
    except Exception as e:  # noqa: BLE001
        print(f"{name:22s} error: {type(e).__name__}: {str(e)[:120]}", flush=True)

# the scalar-term conversion's program for the models still on the tape
for name in ("linear_regression_exp", "cauchy"):
    lp, init = MODELS[name]()
    prog = _trace.compile_model(lp, init)
    alt = _trace.affine_as_expressions(prog.model, True)
    p2 = _trace.Program(alt)
    print(f"{name} converted: terms {[(t.dist, t.n) for t in alt.terms]} HMC {p2.slice_kernel} "
          f"NUTS {p2.nuts_kernel(10)} MH {lib.mc_program_mh_sliced(p2.handle)} "
          f"note {p2.kernel_note!r}", flush=True)
