"""ctypes binding of libmcmc355.so (include/mcmc355.h).

The library is the product: there is no CPU fallback.  Loading fails loudly
when the shared object has not been built (``make -C mlx-mcmc_amd/csrc`` or
``__graft_entry__.build()``) and every sampling entry point raises
``EngineUnavailable`` when no ROCm device is visible.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.realpath(__file__))
LIB_PATH = os.path.join(_HERE, "libmcmc355.so")


class EngineUnavailable(RuntimeError):
    """Raised when the HIP engine cannot run (library missing or no GPU)."""


class EngineError(RuntimeError):
    """A negative MC_ERR_* return code from the C-ABI."""

    def __init__(self, code: int, message: str):
        super().__init__(f"libmcmc355 error {code}: {message}")
        self.code = code


# ---- C structs (must match include/mcmc355.h) -------------------------------
MC_OK = 0
MC_ERR_INVALID = -1
MC_ERR_UNSUPPORTED = -2
MC_ERR_HIP = -3
MC_ERR_NOMEM = -4

MC_DIST_NORMAL = 0
MC_DIST_HALFNORMAL = 1
MC_DIST_EXPONENTIAL = 2
MC_DIST_GAMMA = 3
MC_DIST_BETA = 4
MC_DIST_IDENTITY = 5
MC_DIST_EXPR = 6

# mc_expr_op (expression-term nodes)
(MC_EX_LEAF, MC_EX_ADD, MC_EX_SUB, MC_EX_MUL, MC_EX_DIV, MC_EX_NEG, MC_EX_EXP, MC_EX_LOG,
 MC_EX_SQRT, MC_EX_SQUARE, MC_EX_POW, MC_EX_ABS, MC_EX_LOG1P, MC_EX_TANH, MC_EX_SIGMOID,
 MC_EX_NORMAL_LP, MC_EX_HALFNORMAL_LP, MC_EX_EXPONENTIAL_LP, MC_EX_WHERE,
 MC_EX_GAMMA_LP, MC_EX_BETA_LP, MC_EX_GT, MC_EX_GE, MC_EX_LT, MC_EX_LE) = range(25)
MC_EXPR_MAX_NODES = 32

# mc_series_stats fields (include/mcmc355.h)
MC_ST_ESS, MC_ST_MEAN, MC_ST_M2, MC_ST_HMEAN0, MC_ST_HMEAN1, MC_ST_HM2_0, MC_ST_HM2_1 = range(7)
MC_ST_COUNT = 7

MC_OP_NONE = 0
MC_OP_CONST = 1
MC_OP_PSCALAR = 2
MC_OP_DATA = 3
MC_OP_PVEC = 4
MC_OP_GATHER = 5

MC_XF_NONE = 0
MC_XF_EXP = 1
MC_XF_LOG = 2

MC_RNG_TAG_MOMENTUM = 1
MC_RNG_TAG_ACCEPT = 2
MC_RNG_TAG_SLICE = 3
MC_RNG_TAG_DEPTH = 4
MC_RNG_TAG_MERGE = 5
MC_RNG_TAG_PROPOSAL = 6
MC_RNG_TAG_USER = 16


class McOperand(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int32),
        ("param_offset", ctypes.c_int32),
        ("pool_offset", ctypes.c_int64),
        ("value", ctypes.c_float),
        ("transform", ctypes.c_int32),
    ]


class McTerm(ctypes.Structure):
    _fields_ = [
        ("dist", ctypes.c_int32),
        ("affine", ctypes.c_int32),
        ("n", ctypes.c_int64),
        ("weight", ctypes.c_float),
        ("reserved1", ctypes.c_float),
        ("value", McOperand),
        ("loc", McOperand),
        ("scale", McOperand),
    ]


class McAffine(ctypes.Structure):
    """mc_affine: loc_i = loc_i + slope_i * x_i for a term with affine = k + 1."""
    _fields_ = [
        ("slope", McOperand),
        ("x", McOperand),
    ]


class McExprNode(ctypes.Structure):
    """mc_expr_node: op, argument nodes a, b, c (-1 unused), the leaf operand."""
    _fields_ = [
        ("op", ctypes.c_int32),
        ("a", ctypes.c_int32),
        ("b", ctypes.c_int32),
        ("c", ctypes.c_int32),
        ("leaf", McOperand),
    ]


class McExpr(ctypes.Structure):
    """mc_expr: nodes[first .. first + count) of one expression term."""
    _fields_ = [
        ("first", ctypes.c_int32),
        ("count", ctypes.c_int32),
    ]


class McChainScalars(ctypes.Structure):
    _fields_ = [
        ("step_size", ctypes.c_double),
        ("step_size_bar", ctypes.c_double),
        ("h_bar", ctypes.c_double),
        ("alpha_sum", ctypes.c_double),
        ("mu", ctypes.c_float),
        ("logp", ctypes.c_float),
        ("n_accept", ctypes.c_int32),
        ("n_total", ctypes.c_int32),
        ("warmup_accept", ctypes.c_int32),
        ("warmup_total", ctypes.c_int32),
        ("depth_sum", ctypes.c_int64),
        ("warmup_depth_sum", ctypes.c_int64),
        ("n_grad", ctypes.c_int64),
        ("n_divergent", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
    ]


class McRunConfig(ctypes.Structure):
    _fields_ = [
        ("num_chains", ctypes.c_int64),
        ("chain_offset", ctypes.c_int64),
        ("num_warmup", ctypes.c_int64),
        ("num_samples", ctypes.c_int64),
        ("iter_begin", ctypes.c_int64),
        ("iter_count", ctypes.c_int64),
        ("sample_begin", ctypes.c_int64),
        ("sample_capacity", ctypes.c_int64),
        ("seed", ctypes.c_uint64),
        ("step_size", ctypes.c_double),
        ("target_accept", ctypes.c_double),
        ("num_leapfrog_steps", ctypes.c_int32),
        ("max_tree_depth", ctypes.c_int32),
        ("adapt_step_size", ctypes.c_int32),
        ("slice_mode", ctypes.c_int32),
    ]


class McTrace(ctypes.Structure):
    _fields_ = [
        ("iter_begin", ctypes.c_int64),
        ("capacity", ctypes.c_int64),
        ("accepted", ctypes.c_void_p),
        ("accept_stat", ctypes.c_void_p),
        ("step_size", ctypes.c_void_p),
        ("energy", ctypes.c_void_p),
        ("tree_depth", ctypes.c_void_p),
        ("n_leapfrog", ctypes.c_void_p),
    ]


# (name, restype, argtypes) for every symbol include/mcmc355.h declares
_VP = ctypes.c_void_p
SIGNATURES = [
    ("mc_program_create", ctypes.c_int,
     [ctypes.POINTER(McTerm), ctypes.c_int32, ctypes.c_int32, ctypes.c_float,
      _VP, ctypes.c_int64, _VP, ctypes.c_int64, ctypes.POINTER(_VP)]),
    ("mc_program_create_affine", ctypes.c_int,
     [ctypes.POINTER(McTerm), ctypes.c_int32, ctypes.POINTER(McAffine), ctypes.c_int32,
      ctypes.c_int32, ctypes.c_float, _VP, ctypes.c_int64, _VP, ctypes.c_int64,
      ctypes.POINTER(_VP)]),
    ("mc_program_create_expr", ctypes.c_int,
     [ctypes.POINTER(McTerm), ctypes.c_int32, ctypes.POINTER(McAffine), ctypes.c_int32,
      ctypes.POINTER(McExpr), ctypes.c_int32, ctypes.POINTER(McExprNode), ctypes.c_int32,
      ctypes.c_int32, ctypes.c_float, _VP, ctypes.c_int64, _VP, ctypes.c_int64,
      ctypes.POINTER(_VP)]),
    ("mc_program_destroy", ctypes.c_int, [_VP]),
    ("mc_program_num_params", ctypes.c_int32, [_VP]),
    ("mc_program_waves_per_chain", ctypes.c_int32, [_VP]),
    ("mc_program_set_slices", ctypes.c_int, [_VP, ctypes.c_int32]),
    ("mc_program_num_slices", ctypes.c_int32, [_VP]),
    ("mc_program_set_slice_kernel", ctypes.c_int, [_VP, ctypes.c_int32]),
    ("mc_program_slice_kernel", ctypes.c_int32, [_VP]),
    ("mc_program_lanes_fast", ctypes.c_int32, [_VP]),
    ("mc_program_kernel_note", ctypes.c_char_p, [_VP]),
    ("mc_program_nuts_lanes", ctypes.c_int32, [_VP, ctypes.c_int32]),
    ("mc_logp_grad", ctypes.c_int, [_VP, ctypes.c_int64, _VP, _VP, _VP, _VP]),
    ("mc_dist_log_prob", ctypes.c_int,
     [ctypes.c_int32, ctypes.c_int64, _VP, ctypes.c_int32, _VP, ctypes.c_int32, _VP,
      ctypes.c_int32, _VP, _VP]),
    ("mc_state_bytes", ctypes.c_int64, [_VP, ctypes.c_int64]),
    ("mc_state_offsets", ctypes.c_int,
     [_VP, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
    ("mc_state_init", ctypes.c_int, [_VP, ctypes.c_int64, _VP, ctypes.c_double, _VP, _VP]),
    ("mc_hmc_workspace_bytes", ctypes.c_int64, [_VP, ctypes.c_int64]),
    ("mc_workspace_status", ctypes.c_int, [_VP, _VP, ctypes.c_int64, _VP]),
    ("mc_workspace_release", ctypes.c_int, [_VP]),
    ("mc_debug_exchange_fault", ctypes.c_int, [ctypes.c_int]),
    ("mc_debug_lanes_forms", ctypes.c_int, [ctypes.c_int]),
    ("mc_debug_lanes_fast", ctypes.c_int, [ctypes.c_int]),
    ("mc_debug_nuts_variant", ctypes.c_int, [ctypes.c_int]),
    ("mc_debug_nuts_sliced", ctypes.c_int, [ctypes.c_int]),
    ("mc_debug_xcd_local", ctypes.c_int, [ctypes.c_int]),
    ("mc_debug_workspace_xcd", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32),
                                              ctypes.POINTER(ctypes.c_int32)]),
    ("mc_debug_mh_sliced", ctypes.c_int, [ctypes.c_int]),
    ("mc_program_mh_sliced", ctypes.c_int32, [_VP]),
    ("mc_debug_expr_jit", ctypes.c_int, [ctypes.c_int]),
    ("mc_program_expr_jit", ctypes.c_int32, [_VP]),
    ("mc_debug_program_host_only", ctypes.c_int, [ctypes.c_int]),
    ("mc_debug_expr_jit_source", ctypes.c_int64, [_VP, ctypes.c_char_p, ctypes.c_int64]),
    ("mc_debug_expr_jit_compile", ctypes.c_int, [_VP, ctypes.c_char_p]),
    ("mc_debug_lane_plan_host", ctypes.c_int, [_VP, ctypes.c_int32]),
    ("mc_debug_expr_jit_lane_source", ctypes.c_int64, [_VP, ctypes.c_char_p, ctypes.c_int64]),
    ("mc_box_muller_host", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]),
    ("mc_logf_unit_host", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]),
    ("mc_hmc_run", ctypes.c_int,
     [_VP, ctypes.POINTER(McRunConfig), _VP, _VP, ctypes.POINTER(McTrace), _VP,
      ctypes.c_int64, _VP]),
    ("mc_nuts_workspace_bytes", ctypes.c_int64, [_VP, ctypes.c_int64, ctypes.c_int32]),
    ("mc_nuts_run", ctypes.c_int,
     [_VP, ctypes.POINTER(McRunConfig), _VP, _VP, ctypes.POINTER(McTrace), _VP,
      ctypes.c_int64, _VP]),
    ("mc_mh_workspace_bytes", ctypes.c_int64, [_VP, ctypes.c_int64]),
    ("mc_mh_run", ctypes.c_int,
     [_VP, ctypes.POINTER(McRunConfig), ctypes.c_double, _VP, _VP, ctypes.POINTER(McTrace), _VP,
      ctypes.c_int64, _VP]),
    ("mc_rng_fill", ctypes.c_int,
     [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
      ctypes.c_uint32, ctypes.c_int64, ctypes.c_int32, _VP, _VP]),
    ("mc_series_stats", ctypes.c_int,
     [ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, _VP, ctypes.c_int32, _VP, _VP]),
    ("mc_stats_reduce", ctypes.c_int,
     [ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, _VP, _VP, ctypes.c_int64, _VP, _VP]),
    ("mc_rhat", ctypes.c_int, [ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, _VP, _VP, _VP]),
    ("mc_pool_moments", ctypes.c_int,
     [ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, _VP, ctypes.c_int64, ctypes.c_int64, _VP,
      _VP]),
    ("mc_select_workspace_bytes", ctypes.c_int64, [ctypes.c_int32]),
    ("mc_select", ctypes.c_int,
     [ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, _VP, ctypes.c_int64, ctypes.c_int64,
      ctypes.c_int32, ctypes.POINTER(ctypes.c_int64), _VP, _VP, ctypes.c_int64, _VP]),
    ("mc_last_error", ctypes.c_char_p, []),
    ("mc_abi_version", ctypes.c_int32, []),
]

_lib = None


def load():
    """Load libmcmc355.so (torch first, so the process has one HIP runtime)."""
    global _lib
    if _lib is not None:
        return _lib
    import torch  # noqa: F401  (its libamdhip64 must be the one the library binds)

    if not os.path.exists(LIB_PATH):
        raise EngineUnavailable(
            f"{LIB_PATH} is not built; run `make -C mlx-mcmc_amd/csrc` "
            "(or __graft_entry__.build()) — there is no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    for name, res, args in SIGNATURES:
        try:
            fn = getattr(lib, name)
        except AttributeError:
            # (a test / diagnostic hook an older build lacks — A/B runs of
            # other builds, scripts/ab_lib.py; every product entry point is
            # required)
            if name.startswith("mc_debug_"):
                continue
            raise
        fn.restype = res
        fn.argtypes = args
    if lib.mc_abi_version() != 2:
        raise EngineUnavailable("libmcmc355.so ABI version mismatch")
    _lib = lib
    return lib


def check(rc: int) -> None:
    if rc != MC_OK:
        msg = load().mc_last_error()
        raise EngineError(rc, msg.decode() if msg else "")


def require_device():
    """Return the torch device the engine runs on; raise if there is none."""
    import torch

    load()
    if not torch.cuda.is_available():
        raise EngineUnavailable(
            "no ROCm GPU visible: the MI355X engine has no CPU fallback")
    return torch.device("cuda", torch.cuda.current_device())


def stream_handle():
    import torch

    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def ptr(t) -> ctypes.c_void_p:
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)
