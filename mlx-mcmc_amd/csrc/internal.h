// internal.h — device-side program representation shared by the host code
// that builds it (api.hip) and the kernels that execute it (eval.h, hmc.h,
// nuts.h).  Not part of the C-ABI.
#pragma once
#include <stdint.h>
#include "../../include/mcmc355.h"

namespace mc {

// Operand of a fused term (see mc_operand in mcmc355.h).  `unique` is set by
// the program builder for GATHER operands whose index is injective inside the
// term (each parameter element receives at most one cotangent).
struct DevOperand {
    int32_t kind;
    int32_t poff;
    int64_t pool;
    float cval;
    int32_t unique;
    int32_t slot;     // PSCALAR: LDS slot of its per-wave partial cotangent
    int32_t xf;       // mc_transform_kind of a parameter operand (eval.h xf_*)
};

// Pass mask bits: which cotangents a sweep over the term accumulates.  Terms
// whose accumulating vector operands touch overlapping parameter ranges are
// swept once per conflict-free operand group (deterministic, no atomics).
enum : uint32_t {
    PASS_VALUE = 1u,
    PASS_LOC = 2u,
    PASS_SCALE = 4u,
    PASS_LP = 8u,
};

struct DevTerm {
    int32_t dist;
    int32_t primary;   // operand slot (0 value, 1 loc, 2 scale) of the
                       // non-injective GATHER the term is grouped by, or -1
    int64_t n;
    float weight;
    float c0;          // f32 normaliser: -0.5 log(2 pi)  [+ log 2 for HalfNormal]
    int32_t npass;
    uint32_t pass_masks;  // 4 bits per sweep: PASS_* of sweep p at bits 4p..4p+3
    int32_t prim_poff;    // param offset of the primary operand (no runtime
                          // indexing of op[]: it would force T into scratch)
    int32_t wave_task;    // >= 0: a small term with only broadcast-parameter
                          // cotangents, evaluated by this one wave while the
                          // other waves move on (-1: every wave)
    float clogs;          // CONST scale: f32 log(scale), precomputed
    float clg;            // Gamma / Beta with constant shapes: the gammaln
                          // normaliser (lgamma_norm), precomputed
    DevOperand op[3];  // value, loc, scale
    // ---- segment-tiled layout (primary >= 0) --------------------------------
    // Elements are grouped by the primary index into runs ("segments"), long
    // runs split into virtual segments; 64 virtual segments form a tile, one
    // per lane.  Every vector operand of the term is stored tiled: element u
    // of lane l of tile t lives at  tile_off[t] + (u/4)*256 + l*4 + u%4,
    // so a lane walks its own run with coalesced 16-byte loads.
    int32_t ntiles;
    int32_t nvirt;
    int32_t ncomb;        // > 0: segments were split, partials combined in order
    int32_t sync_before;  // a barrier is needed before this term's writes
    int64_t tile_base;    // index pool: per tile {off, len_pad, len_min}
    int64_t lane_base;    // index pool: per virtual segment {k, len}
    int64_t comb_base;    // index pool: per segment {k, vfirst, vcount}
    // ---- affine loc (mc_affine): loc_i = op[1]_i + ab_i * ax_i ----------------
    int32_t affine;       // 0 / 1
    int32_t pad_aff;
    DevOperand ab, ax;    // slope (CONST / PSCALAR), x (DATA / PVEC / GATHER)
    // ---- expression term (MC_DIST_EXPR): DevCtx::nodes[expr_base ..) --------
    int32_t expr_base;
    int32_t expr_n;       // nodes; the last is the root
};

// A node of an expression term (mc_expr_node).  `pass`: the sweep in which a
// vector leaf deposits its cotangents (leaves with overlapping parameter
// ranges deposit in different sweeps); `prim`: a leaf gathered through the
// term's non-injective index (segmented terms: value q[poff + k] of the
// lane's run, cotangent summed in a register and deposited once per run);
// prim = 1 + the leaf's row of split-run partials (0: not gathered so).
struct DevExprNode {
    int32_t op, a, b, c;
    int32_t pass, prim;
    DevOperand leaf;
};

struct DevCtx {
    const DevTerm* terms;
    const DevExprNode* nodes;  // expression-term nodes (may be null)
    int32_t n_terms;
    int32_t D;
    float lp_const;
    int32_t nslots;       // PSCALAR cotangent slots (+1 for log p)
    const float* data;
    const int32_t* index;
    int64_t sfin_base;    // index pool: {n_sparams, then per param {poff, first, count}},
                          // then the slot ids, grouped by parameter
};

// Per-launch constants shared by the sampler kernels.
struct RunArgs {
    mc_run_config cfg;
    int32_t dpad;          // D rounded up to 16 floats (arena stride unit)
    int32_t lds_floats;    // LDS floats per chain group
    int32_t scratch_floats;  // of which the evaluator's scratch (arena follows)
    int32_t data_lds;      // k_nuts: data-pool floats staged in LDS after the
                           // chain groups (0: the pool is read from global memory)
    int32_t fault;         // exchange kernels, test hook (mc_debug_exchange_fault):
                           // the grid's last workgroup exits at once, so the others
                           // of its chain block time out
};

struct TraceDev {
    int64_t iter_begin;
    int64_t capacity;
    uint8_t* accepted;
    float* accept_stat;
    double* step_size;
    float* energy;
    int32_t* tree_depth;
    int32_t* n_leapfrog;
};

constexpr int kMaxTreeDepth = 16;

}  // namespace mc
