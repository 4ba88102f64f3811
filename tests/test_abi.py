"""The C-ABI boundary without a GPU: the library loads, exports every symbol
include/mcmc355.h declares, its structs match the ctypes mirror, and argument
validation fails with the documented codes before touching the device."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from mlx_mcmc_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mcmc355.h")


def declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z0-9_]+\s*\**\s+(mc_[a-z0-9_]+)\s*\(",
                                 text, flags=re.M)))


def test_every_declared_symbol_is_exported():
    lib = _lib.load()
    names = declared_functions()
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), n
    assert {n for n, _, _ in _lib.SIGNATURES} == set(names)


def test_struct_layouts_match_header(tmp_path):
    src = tmp_path / "lay.c"
    src.write_text("""
#include <stdio.h>
#include <stddef.h>
#include "mcmc355.h"
#define O(T, f) printf("%s.%s %zu\\n", #T, #f, offsetof(T, f));
int main(void) {
  printf("mc_operand %zu\\nmc_term %zu\\nmc_chain_scalars %zu\\nmc_run_config %zu\\nmc_trace %zu\\nmc_affine %zu\\n",
         sizeof(mc_operand), sizeof(mc_term), sizeof(mc_chain_scalars), sizeof(mc_run_config),
         sizeof(mc_trace), sizeof(mc_affine));
  printf("mc_expr_node %zu\\nmc_expr %zu\\n", sizeof(mc_expr_node), sizeof(mc_expr));
  O(mc_expr_node, leaf) O(mc_expr, count)
  O(mc_term, affine) O(mc_affine, x) O(mc_term, value) O(mc_term, loc) O(mc_term, scale) O(mc_chain_scalars, logp)
  O(mc_chain_scalars, depth_sum) O(mc_chain_scalars, n_divergent) O(mc_run_config, seed)
  O(mc_run_config, step_size) O(mc_run_config, slice_mode) O(mc_trace, n_leapfrog)
  return 0;
}
""")
    exe = tmp_path / "lay"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                   check=True)
    out = dict(line.rsplit(" ", 1) for line in
               subprocess.run([str(exe)], capture_output=True, text=True).stdout.split("\n")
               if line)
    assert int(out["mc_operand"]) == ctypes.sizeof(_lib.McOperand)
    assert int(out["mc_term"]) == ctypes.sizeof(_lib.McTerm)
    assert int(out["mc_chain_scalars"]) == ctypes.sizeof(_lib.McChainScalars)
    assert int(out["mc_run_config"]) == ctypes.sizeof(_lib.McRunConfig)
    assert int(out["mc_trace"]) == ctypes.sizeof(_lib.McTrace)
    assert int(out["mc_affine"]) == ctypes.sizeof(_lib.McAffine)
    assert int(out["mc_expr_node"]) == ctypes.sizeof(_lib.McExprNode)
    assert int(out["mc_expr"]) == ctypes.sizeof(_lib.McExpr)
    for key, (cls, field) in {
        "mc_term.affine": (_lib.McTerm, "affine"), "mc_affine.x": (_lib.McAffine, "x"),
        "mc_expr_node.leaf": (_lib.McExprNode, "leaf"), "mc_expr.count": (_lib.McExpr, "count"),
        "mc_term.value": (_lib.McTerm, "value"), "mc_term.loc": (_lib.McTerm, "loc"),
        "mc_term.scale": (_lib.McTerm, "scale"),
        "mc_chain_scalars.logp": (_lib.McChainScalars, "logp"),
        "mc_chain_scalars.depth_sum": (_lib.McChainScalars, "depth_sum"),
        "mc_chain_scalars.n_divergent": (_lib.McChainScalars, "n_divergent"),
        "mc_run_config.seed": (_lib.McRunConfig, "seed"),
        "mc_run_config.step_size": (_lib.McRunConfig, "step_size"),
        "mc_run_config.slice_mode": (_lib.McRunConfig, "slice_mode"),
        "mc_trace.n_leapfrog": (_lib.McTrace, "n_leapfrog"),
    }.items():
        assert int(out[key]) == getattr(cls, field).offset, key


def test_validation_errors_before_device_work():
    lib = _lib.load()
    h = ctypes.c_void_p()
    terms = (_lib.McTerm * 1)()
    terms[0].dist = 7
    terms[0].n = 1
    rc = lib.mc_program_create(terms, 1, 2, 0.0, None, 0, None, 0, ctypes.byref(h))
    assert rc == _lib.MC_ERR_INVALID
    assert b"unknown distribution" in lib.mc_last_error()
    rc = lib.mc_program_create(terms, 1, 0, 0.0, None, 0, None, 0, ctypes.byref(h))
    assert rc == _lib.MC_ERR_INVALID and b"n_params" in lib.mc_last_error()
    # a gather index outside the parameter vector
    terms[0].dist = _lib.MC_DIST_NORMAL
    terms[0].n = 3
    terms[0].value.kind = _lib.MC_OP_CONST
    terms[0].loc.kind = _lib.MC_OP_GATHER
    terms[0].loc.param_offset = 0
    terms[0].loc.pool_offset = 0
    terms[0].scale.kind = _lib.MC_OP_CONST
    terms[0].scale.value = 1.0
    idx = np.array([0, 1, 5], np.int32)
    rc = lib.mc_program_create(terms, 1, 2, 0.0, None, 0, idx.ctypes.data_as(ctypes.c_void_p),
                               3, ctypes.byref(h))
    assert rc == _lib.MC_ERR_INVALID and b"out of range" in lib.mc_last_error()
    assert lib.mc_abi_version() == 2
    # host-side switch of the exchange kernels' timeout test hook
    assert lib.mc_debug_exchange_fault(0) == 0
    assert lib.mc_rng_fill(0, 0, 0, 0, 0, 0, 1, 9, None, None) == _lib.MC_ERR_INVALID


def test_product_fails_loudly_without_a_device():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a device is visible")
    import mlx_mcmc_amd as m

    with pytest.raises(_lib.EngineUnavailable):
        m.hmc(lambda p: m.Normal(0, 1).log_prob(p["x"]), {"x": 0.0}, num_samples=5,
              num_warmup=5, progress=False)
    with pytest.raises(_lib.EngineUnavailable):
        m.Normal(0, 1).log_prob(0.0)


def _expr_program(nodes, n=3, n_params=4, index=None, via_affine=False):
    """mc_program_create_expr on one expression term (host-side validation
    only: every case below fails before any device allocation)."""
    lib = _lib.load()
    h = ctypes.c_void_p()
    terms = (_lib.McTerm * 1)()
    terms[0].dist = _lib.MC_DIST_EXPR
    terms[0].n = n
    terms[0].weight = 1.0
    terms[0].affine = 1
    exprs = (_lib.McExpr * 1)()
    exprs[0].first, exprs[0].count = 0, len(nodes)
    carr = (_lib.McExprNode * max(1, len(nodes)))()
    for k, (op, a, b, c, leaf) in enumerate(nodes):
        carr[k].op, carr[k].a, carr[k].b, carr[k].c = op, a, b, c
        if leaf:
            for f, v in leaf.items():
                setattr(carr[k].leaf, f, v)
    data = np.arange(3, dtype=np.float32)
    idx = np.asarray(index if index is not None else [0, 0, 1], np.int32)
    dp, ip = data.ctypes.data_as(ctypes.c_void_p), idx.ctypes.data_as(ctypes.c_void_p)
    if via_affine:
        return lib.mc_program_create_affine(terms, 1, None, 0, n_params, 0.0, dp, 3, ip,
                                            idx.size, ctypes.byref(h)), lib.mc_last_error()
    rc = lib.mc_program_create_expr(terms, 1, None, 0, exprs, 1, carr, len(nodes), n_params, 0.0,
                                    dp, 3, ip, idx.size, ctypes.byref(h))
    return rc, lib.mc_last_error()


P0 = {"kind": _lib.MC_OP_PSCALAR, "param_offset": 0}
DATA = {"kind": _lib.MC_OP_DATA, "pool_offset": 0}
L, E = _lib.MC_EX_LEAF, _lib


@pytest.mark.parametrize("nodes,code,msg", [
    ([(L, -1, -1, -1, P0), (E.MC_EX_ADD, 0, -1, -1, None)], _lib.MC_ERR_INVALID,
     b"bad arguments"),                                                   # missing operand
    ([(L, -1, -1, -1, P0), (E.MC_EX_EXP, 1, -1, -1, None)], _lib.MC_ERR_INVALID,
     b"bad arguments"),                                                   # forward reference
    ([(L, -1, -1, -1, P0), (99, 0, -1, -1, None)], _lib.MC_ERR_INVALID, b"unknown op"),
    ([(L, -1, -1, -1, dict(P0, transform=_lib.MC_XF_EXP))], _lib.MC_ERR_INVALID,
     b"no transform"),
    ([(L, -1, -1, -1, {"kind": _lib.MC_OP_PSCALAR, "param_offset": 9})], _lib.MC_ERR_INVALID,
     b"out of range"),
    ([(L, -1, -1, -1, P0), (L, -1, -1, -1, DATA), (E.MC_EX_WHERE, 0, 1, 1, None)],
     _lib.MC_ERR_UNSUPPORTED, b"where mask"),                            # traced mask
    ([(L, -1, -1, -1, P0)] * 33, _lib.MC_ERR_UNSUPPORTED, b"1 .. 32 nodes"),
    # leaf ranges past the caller's pools (checked against n_data / n_index,
    # not the library's grown copies of them)
    ([(L, -1, -1, -1, {"kind": _lib.MC_OP_DATA, "pool_offset": 1})], _lib.MC_ERR_INVALID,
     b"data range out of pool"),
    ([(L, -1, -1, -1, {"kind": _lib.MC_OP_GATHER, "param_offset": 0, "pool_offset": 2})],
     _lib.MC_ERR_INVALID, b"index range out of pool"),
])
def test_expression_validation(nodes, code, msg):
    rc, err = _expr_program(nodes)
    assert rc == code and msg in err, (rc, err)


def test_expression_validation_gathers_and_entry_points():
    g0 = {"kind": _lib.MC_OP_GATHER, "param_offset": 0, "pool_offset": 0}
    g1 = {"kind": _lib.MC_OP_GATHER, "param_offset": 0, "pool_offset": 3}
    # two non-injective gathers through different index values
    rc, err = _expr_program([(L, -1, -1, -1, g0), (L, -1, -1, -1, g1),
                             (E.MC_EX_MUL, 0, 1, -1, None)], index=[0, 0, 1, 1, 1, 0])
    assert rc == _lib.MC_ERR_UNSUPPORTED and b"two different non-injective" in err
    # expression terms only through mc_program_create_expr
    rc, err = _expr_program([(L, -1, -1, -1, P0)], via_affine=True)
    assert rc == _lib.MC_ERR_INVALID and b"mc_program_create_expr" in err
