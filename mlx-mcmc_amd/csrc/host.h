// host.h — internal host-side declarations shared by the translation units of
// libmcmc355.so (api.hip: program builder, planners, tape / diagnostics
// launches and the rest of the C-ABI; run_hmc.hip, run_mh.hip, run_nuts.hip:
// the sampler launches).  Helpers are `inline` so that every unit shares one
// definition (and one copy of the caches and workspace tag tables).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>
#include <type_traits>
#include <numeric>
#include <unordered_map>
#include <string>
#include <vector>


#include "eval.h"
#include "hmc.h"
#include "internal.h"
#include "lanes.h"
#include "lanes_fast.h"
#include "nuts_lanes.h"
#include "nuts_sliced.h"
#include "mh.h"
#include "nuts.h"
#include "philox.h"
#include "sliced.h"

using namespace mc;

// ---------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------
inline thread_local std::string g_last_error;

inline int fail(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

#define MC_HIP_TRY(expr)                                                                \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess)                                                           \
            return fail(MC_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_));      \
    } while (0)

// ---------------------------------------------------------------------------
// program
// ---------------------------------------------------------------------------
// Host copy of a sliced layout (sliced.h) and its device tables.
struct SlicePlan {
    int S = 1, Lp = 0, Pmax = 0, Dsh = 0, nitems = 0, sdata_floats = 0, nb_max = 0, combine = 0;
    std::vector<SlTerm> terms;
    std::vector<SlTerm> sterms;  // scalar terms (after the exchange)
    std::vector<float> data;
    std::vector<int32_t> index;
    std::vector<int64_t> blocks;
    std::vector<int32_t> gidx;
    SlTerm* d_terms = nullptr;
    SlTerm* d_sterms = nullptr;
    float* d_data = nullptr;
    int32_t* d_index = nullptr;
    int64_t* d_blocks = nullptr;
    int32_t* d_gidx = nullptr;
};

// Host copy of the lane-resident layout (lanes.h) and its device tables.
struct LanePlan {
    int ok = 0;          // the sliced program qualifies
    int rs = 1;          // register slots per lane (1, 2 or 4)
    int sdata_floats = 0;
    int S = 0, Dsh = 0, nitems = 0;  // slice geometry (S = 1: an unsliced program, no exchange)
    int32_t shl[kLrMaxShared] = {0, 0, 0, 0};  // shared parameters by ordinal
    int32_t n_generic = 0;  // scalar terms that are not "own" priors
    int fast = 0;        // fast form: only swept / direct terms and own priors (k_hmc_lf)
    int form = -1;       // the fast form's LF_* bits when every slice has the same terms
                         // and distinct shared roles (compile-time k_hmc_lf), else -1
    int32_t shxf[kLrMaxShared] = {0, 0, 0, 0};  // transforms of the shared parameters
    float shid[kLrMaxShared] = {0.f, 0.f, 0.f, 0.f};  // raw identity weights (k_hmc_lf)
    int rep = 1;         // lanes per private parameter (lanes.h LrCtx::rep)
    std::vector<int32_t> rng;  // [S][64][4] lane RNG plan (lanes_fast.h lf_rng_*), or empty
    int32_t* d_rng = nullptr;
    int has_xf = 0;      // a shared parameter is transformed, or an identity term
                         // (no NUTS lanes, no term interpreter)
    int has_expr = 0;    // LS_EXPR terms: only the JIT-compiled k_hmc_lr runs the plan
                         // (jit.hip); without it the program runs on the tape
    int nuts_expr = 0;   // LS_EXPR terms beside a fast form (every other term swept /
                         // direct, every scalar term an own prior): the JIT-compiled
                         // run-time form of k_nuts_sl takes the program
    std::string why;     // why it does not qualify
    std::vector<LrTerm> terms;
    std::vector<float> data;
    std::vector<int64_t> blocks;
    std::vector<int32_t> gidx;
    std::vector<LrSterm> sterms;
    LrTerm* d_terms = nullptr;
    LrSterm* d_sterms = nullptr;
    float* d_data = nullptr;
    int64_t* d_blocks = nullptr;
    int32_t* d_gidx = nullptr;
};

struct mc_program {
    int32_t D = 0;
    float lp_const = 0.0f;
    int32_t wpc = 1;
    int32_t nslots = 1;
    int64_t sfin_base = 0;
    int64_t max_n = 0;
    std::vector<DevTerm> terms;
    DevTerm* d_terms = nullptr;
    std::vector<DevExprNode> nodes;  // expression-term nodes (DevTerm::expr_base)
    bool ex = false;                 // has expression terms: the EX kernel instantiations
    DevExprNode* d_nodes = nullptr;
    float* d_data = nullptr;
    int32_t* d_index = nullptr;
    // terms as validated (before the chain-per-workgroup tiling) and the host
    // pools they point into: the input of the slice planner
    std::vector<DevTerm> raw;
    std::vector<float> h_data;
    std::vector<int32_t> h_index;
    SlicePlan sl;
    LanePlan lr;
    int32_t slice_kernel = 0;  // 0 automatic, 1 term interpreter, 2 lane-resident
    // why the automatic plan did not reach the lane-resident kernel ("" when it
    // did or was not asked to): mc_program_kernel_note
    std::string note;
    // the expression-term JIT's compiled kernels (jit.hip JitState), created
    // at the first launch that uses them
    mutable void* jit = nullptr;
};

inline DevCtx ctx_of(const mc_program* p) {
    DevCtx c;
    c.terms = p->d_terms;
    c.nodes = p->d_nodes;
    c.n_terms = (int32_t)p->terms.size();
    c.D = p->D;
    c.lp_const = p->lp_const;
    c.nslots = p->nslots;
    c.data = p->d_data;
    c.index = p->d_index;
    c.sfin_base = p->sfin_base;
    return c;
}

inline SlCtx slctx_of(const mc_program* p) {
    SlCtx c;
    std::memset(&c, 0, sizeof(c));
    const SlicePlan& P = p->sl;
    c.terms = P.d_terms;
    c.data = P.d_data;
    c.index = P.d_index;
    c.blocks = P.d_blocks;
    c.gidx = P.d_gidx;
    c.n_terms = (int32_t)p->raw.size();
    c.S = P.S;
    c.Lp = P.Lp;
    c.Pmax = P.Pmax;
    c.Dsh = P.Dsh;
    c.D = p->D;
    c.nitems = P.nitems;
    c.sdata_floats = P.sdata_floats;
    c.lp_const = p->lp_const;
    c.combine = P.combine;
    c.sterms = P.d_sterms;
    c.n_sterms = (int32_t)P.sterms.size();
    return c;
}
static constexpr int kSlLdsBudget = 150 * 1024;
inline bool has_affine(const mc_program* p) {
    for (const DevTerm& t : p->raw)
        if (t.affine) return true;
    return false;
}
inline bool has_expr(const mc_program* p) {
    for (const DevTerm& t : p->raw)
        if (t.dist == MC_DIST_EXPR) return true;
    return false;
}
// Transformed parameter operands and identity terms (the reparameterised
// models of mc_transform_kind).
inline bool has_transform(const mc_program* p) {
    for (const DevTerm& t : p->raw) {
        if (t.dist == MC_DIST_IDENTITY) return true;
        for (int a = 0; a < 3; ++a)
            if (t.op[a].xf != MC_XF_NONE) return true;
        if (t.affine && (t.ab.xf != MC_XF_NONE || t.ax.xf != MC_XF_NONE)) return true;
    }
    return false;
}
// ... whose transforms all act on broadcast (PSCALAR) parameters and whose
// identity terms are scalar: the lane-resident kernel k_hmc_lr runs them
// (lanes.h LrCtx::shxf); anything else runs on the chain-per-workgroup kernels.
inline bool transform_on_shared_only(const mc_program* p) {
    for (const DevTerm& t : p->raw) {
        if (t.affine && (t.ab.xf != MC_XF_NONE || t.ax.xf != MC_XF_NONE)) return false;
        for (int a = 0; a < 3; ++a)
            if (t.op[a].xf != MC_XF_NONE && t.op[a].kind != MC_OP_PSCALAR) return false;
        if (t.dist == MC_DIST_IDENTITY && t.op[0].kind != MC_OP_PSCALAR &&
            t.op[0].kind != MC_OP_CONST)
            return false;
    }
    return true;
}
// Affine terms the lane-resident kernels take (lanes.h LS_AFF): Normal, value
// data, loc private (a parameter vector or gather), shared or constant, slope
// shared or constant, x data, no transform on the slope or x.  Any other
// affine term (x a parameter vector: the non-centred mu + tau * z) keeps the
// program on the chain-per-workgroup kernels.
inline bool affine_lanes_ok(const mc_program* p) {
    for (const DevTerm& t : p->raw) {
        if (!t.affine) continue;
        if (t.dist != MC_DIST_NORMAL || t.op[0].kind != MC_OP_DATA) return false;
        if (t.ax.kind != MC_OP_DATA || t.ax.xf != MC_XF_NONE) return false;
        if (!(t.ab.kind == MC_OP_PSCALAR || t.ab.kind == MC_OP_CONST) || t.ab.xf != MC_XF_NONE)
            return false;
        const int k1 = t.op[1].kind, k2 = t.op[2].kind;
        if (!(k1 == MC_OP_PVEC || k1 == MC_OP_GATHER || k1 == MC_OP_PSCALAR || k1 == MC_OP_CONST))
            return false;
        if (!(k2 == MC_OP_PSCALAR || k2 == MC_OP_CONST)) return false;
    }
    return true;
}
// Expression terms the lane-resident kernel takes (lanes.h LS_EXPR, code
// generated per program by the expression JIT): leaves data, broadcast
// parameters and constants only — no parameter vectors or gathers — with at
// least one data array and at most kLrExprData of them, one pass.  Every term
// of the program must qualify (else the program stays on the tape kernels).
inline bool expr_lanes_ok(const mc_program* p) {
    if (const char* e = std::getenv("MC_EXPR_LANES"))  // 0: the tape (A/B, tests)
        if (e[0] == '0') return false;
    for (const DevTerm& t : p->raw) {
        if (t.dist != MC_DIST_EXPR) continue;
        if (t.primary >= 0 || t.npass != 1 || t.expr_n < 1) return false;
        std::vector<int64_t> arrays;  // distinct data arrays (one LDS tile each)
        for (int k = 0; k < t.expr_n; ++k) {
            const DevExprNode& d = p->nodes[t.expr_base + k];
            if (d.op != MC_EX_LEAF) continue;
            if (d.prim) return false;
            if (d.leaf.kind == MC_OP_DATA) {
                if (std::find(arrays.begin(), arrays.end(), d.leaf.pool) == arrays.end())
                    arrays.push_back(d.leaf.pool);
            } else if (d.leaf.kind != MC_OP_CONST && d.leaf.kind != MC_OP_PSCALAR) {
                return false;
            }
        }
        if (arrays.empty() || (int)arrays.size() > kLrExprData) return false;
    }
    return true;
}
// The term interpreter (k_hmc_sl) takes neither transformed operands, affine
// locs nor expression terms: such sliced programs run on the lane-resident
// kernels only (or, expression terms without the JIT, on the tape).
inline bool interp_ok(const mc_program* p) {
    return !has_transform(p) && !has_affine(p) && !has_expr(p);
}

inline LrCtx lrctx_of(const mc_program* p) {
    LrCtx c;
    std::memset(&c, 0, sizeof(c));
    const LanePlan& L = p->lr;
    c.terms = L.d_terms;
    c.data = L.d_data;
    c.blocks = L.d_blocks;
    c.gidx = L.d_gidx;
    c.sterms = L.d_sterms;
    c.n_terms = (int32_t)p->raw.size();
    c.n_sterms = (int32_t)L.sterms.size();
    c.n_sterms_generic = L.n_generic;
    c.S = L.S;
    c.Dsh = L.Dsh;
    c.D = p->D;
    c.nitems = L.nitems;
    c.sdata_floats = L.sdata_floats;
    c.lp_const = p->lp_const;
    for (int k = 0; k < kLrMaxShared; ++k) {
        c.shl[k] = L.shl[k];
        c.shxf[k] = L.shxf[k];
        c.shid[k] = L.shid[k];
    }
    c.has_xf = L.has_xf;
    c.rep = L.rep;
    c.rng = (const int4*)L.d_rng;
    return c;
}
// ---------------------------------------------------------------------------
// geometry helpers
// ---------------------------------------------------------------------------
inline int cpb_of(int wpc) { return wpc >= 4 ? 1 : 4 / wpc; }
inline int block_of(int wpc) { return 64 * wpc * cpb_of(wpc); }
inline int32_t dpad_of(int32_t D) { return (D + 15) / 16 * 16; }
static constexpr int64_t kLdsArenaBudget = 64 * 1024;  // keep >= 2 workgroups per CU

inline int scratch_of(const mc_program* p) {
    // keep every chain group's region 16-byte aligned
    return (group_scratch_floats(p->wpc, p->nslots) + 3) / 4 * 4;
}
inline int64_t hmc_lds_floats(const mc_program* p, bool lds_arena) {
    return scratch_of(p) + (lds_arena ? 5 * (int64_t)dpad_of(p->D) : 0);
}
inline bool hmc_use_lds(const mc_program* p) {
    return cpb_of(p->wpc) * hmc_lds_floats(p, true) * 4 <= kLdsArenaBudget;
}

template <typename K>
inline hipError_t allow_lds(K kernel, size_t bytes) {
    if (bytes <= 64 * 1024) return hipSuccess;
    // the attribute is a per-(kernel, device) maximum: the largest value set so
    // far is cached and a launch needing no more skips the call (it costs host
    // time on every launch otherwise; launch functions run once per chunk of
    // iterations).  A launch needing more raises it — never lowers it, so a
    // later large launch of the same instantiation is never refused.
    static std::mutex mu;
    static std::map<std::pair<const void*, int>, size_t> max_set;
    int dev = 0;
    (void)hipGetDevice(&dev);
    const auto key = std::make_pair(reinterpret_cast<const void*>(kernel), dev);
    std::lock_guard<std::mutex> lk(mu);
    auto it = max_set.find(key);
    if (it != max_set.end() && bytes <= it->second) return hipSuccess;
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e == hipSuccess) max_set[key] = bytes;
    return e;
}

inline TraceDev trace_of(const mc_trace* t) {
    TraceDev d;
    std::memset(&d, 0, sizeof(d));
    if (t) {
        d.iter_begin = t->iter_begin;
        d.capacity = t->capacity;
        d.accepted = t->accepted;
        d.accept_stat = t->accept_stat;
        d.step_size = t->step_size;
        d.energy = t->energy;
        d.tree_depth = t->tree_depth;
        d.n_leapfrog = t->n_leapfrog;
    } else {
        d.capacity = 0;
    }
    return d;
}

// The instantiation of a chain-per-workgroup launcher for a program: waves
// per chain (1, 4 or 8), LDS arena or not, expression terms or not (EX).
template <typename F>
inline int dispatch_tape(const mc_program* p, bool lds, F&& f) {
    using T_ = std::true_type;
    using F_ = std::false_type;
    auto ex = [&](auto w, auto l) { return p->ex ? f(w, l, T_{}) : f(w, l, F_{}); };
    auto arena = [&](auto w) { return lds ? ex(w, T_{}) : ex(w, F_{}); };
    switch (p->wpc) {
        case 1: return arena(std::integral_constant<int, 1>{});
        case 4: return arena(std::integral_constant<int, 4>{});
        default: return arena(std::integral_constant<int, 8>{});
    }
}
// ---------------------------------------------------------------------------
// HMC / NUTS launches
// ---------------------------------------------------------------------------
inline int check_cfg(const mc_program* p, const mc_run_config* cfg, void* state) {
    if (!p || !cfg || !state) return fail(MC_ERR_INVALID, "NULL program/config/state");
    if (cfg->num_chains < 0 || cfg->iter_count < 0 || cfg->iter_begin < 0 ||
        cfg->num_warmup < 0 || cfg->num_samples < 0)
        return fail(MC_ERR_INVALID, "negative count in config");
    if (cfg->chain_offset < 0 || cfg->chain_offset + cfg->num_chains > (int64_t)UINT32_MAX)
        return fail(MC_ERR_INVALID, "chain ids must fit in 32 bits");
    if (cfg->iter_begin + cfg->iter_count > (int64_t)UINT32_MAX)
        return fail(MC_ERR_INVALID, "iteration ids must fit in 32 bits");
    return MC_OK;
}

// ---- same-XCD exchange (sliced.h granule_store_xcd) ---------------------------
// The exchange kernels place a block's S slices at workgroups w with equal
// w % 8 when the grid allows (grid % 8 == 0 and (grid / 8) % S == 0); with
// the device dealing workgroups round-robin over its 8 XCDs (observed on
// MI355X, not an architectural guarantee) those share an XCD, and records
// can stay in its L2.  xcd_round_robin(grid) checks that dealing once per
// (device, grid size): a probe launch records each workgroup's XCC id and
// every residue class mod 8 must name one XCD.  MC_XCD_LOCAL=0 in the
// environment (or mc_debug_xcd_local(0)) turns the L2-resident exchange off.
// The kernels check the placement again before their first publish.
inline int g_xcd_local = -1;  // mc_debug_xcd_local; -1: MC_XCD_LOCAL from the environment
bool xcd_round_robin(int64_t grid, int S);  // (run_hmc.hip)

// ---- sliced launches ---------------------------------------------------------
inline int device_cus() {
    static int cached[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
    if (cached[dev] == 0) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return 0;
        cached[dev] = n;
    }
    return cached[dev];
}
// Exchange kernels (k_hmc_sl, k_hmc_lr with S >= 2) spin on records of the
// other workgroups of their chain block, so every workgroup of a launch must
// be resident at once.  An occupancy query of the same kernel, block size and
// LDS caps the grid at what the device holds: a launch that cannot be
// co-resident fails fast with MC_ERR_UNSUPPORTED.  They are then launched
// plainly: on a device shared with other work that keeps some of the grid
// out, the spin times out and the launch reports MC_ERR_TIMEOUT with the
// stranded block's state unchanged (mc_workspace_status).  (Round 2 also
// offered cooperative launches behind an environment switch: ~50 us more per
// launch on MI355X, profiles/r2/v17_coop_ab.json, and a crash in torch's HIP
// exit handlers under rocprofv3 whose cause was not found — removed.)
template <typename... KA, typename... A>
inline hipError_t launch_exchange(void (*k)(KA...), int64_t grid, int block, size_t lds,
                                  hipStream_t st, A&&... a) {
    hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(block), lds, st,
                       std::decay_t<KA>(std::forward<A>(a))...);
    return hipGetLastError();
}
// workgroups of kernel k (block threads, lds bytes) the device holds at once
template <typename K>
inline int64_t resident_capacity(K k, int block, size_t lds) {
    // cached per (kernel, device, block, LDS): the occupancy query is a host
    // call on every exchange launch otherwise
    static std::mutex mu;
    static std::map<std::tuple<const void*, int, int, size_t>, int64_t> cache;
    int dev = 0;
    (void)hipGetDevice(&dev);
    const auto key = std::make_tuple(reinterpret_cast<const void*>(k), dev, block, lds);
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = cache.find(key);
        if (it != cache.end()) return it->second;
    }
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(k), block,
                                                     lds) != hipSuccess)
        return -1;
    const int64_t cap = (int64_t)n * device_cus();
    std::lock_guard<std::mutex> lk(mu);
    cache[key] = cap;
    return cap;
}
inline int g_exchange_fault = 0;  // mc_debug_exchange_fault
inline bool sliced(const mc_program* p) { return p->sl.S >= 2 && p->sl.d_terms != nullptr; }
// an unsliced program planned onto the lane-resident kernel (one slice)
inline bool lanes1(const mc_program* p) { return p->sl.S < 2 && p->lr.ok && p->lr.S == 1; }
inline int sl_nb_for(const mc_program* p, int64_t C) {
    return (p->sl.nb_max >= 16 && C > 8) ? 16 : 8;
}
// chain blocks per launch: every workgroup of a launch must be resident at
// once (the slices of a block wait for each other), one workgroup per CU
inline int64_t sl_groups_per_launch(const mc_program* p, int64_t C) {
    const int nb = sl_nb_for(p, C);
    const int64_t groups = (C + nb - 1) / nb;
    const int64_t cap = std::max<int64_t>(1, device_cus() / p->sl.S);
    return std::min(groups, cap);
}
static constexpr int64_t kSlStatusBytes = 256;
// waves per workgroup of the lane-resident kernel: 8 (16 chains, two waves per
// SIMD) for up to 16 slices... 4 (8 chains, one wave per SIMD) for <= 8 slices
// one slice: one wave per workgroup (no exchange, so no block structure to
// keep; a lone wave per CU does not share the scalar unit or LDS with others)
inline int lr_nw(const mc_program* p) { return p->lr.S == 1 ? 1 : (p->lr.S <= 8 ? 4 : 8); }
inline int64_t lr_groups_per_launch(const mc_program* p, int64_t C) {
    const int nb = 2 * lr_nw(p);
    const int64_t groups = (C + nb - 1) / nb;
    if (p->lr.S == 1) return groups;  // no exchange: no co-residency needed
    const int64_t cap = std::max<int64_t>(1, device_cus() / p->lr.S);
    return std::min(groups, cap);
}
inline int64_t sl_workspace_bytes(const mc_program* p, int64_t C) {
    if (lanes1(p)) return kSlStatusBytes;
    const int nb = sl_nb_for(p, C);
    int64_t x = 2 * sl_groups_per_launch(p, C) * p->sl.S * (int64_t)p->sl.nitems * nb * 8;
    if (p->lr.ok)  // either kernel may run on the same workspace (lanes.h: one
                   // 128-byte line per (wave, slice) record)
        x = std::max(x, 2 * lr_groups_per_launch(p, C) * lr_nw(p) * p->sl.S * 128);
    return kSlStatusBytes + x;
}
// A lane plan with expression terms (LanePlan::has_expr) runs only the
// JIT-compiled k_hmc_lr (its LS_EXPR sweep is generated per program,
// jit.hip gen_lane_term); when the JIT is off or its compilation failed the
// launch returns kLanesNoJit and the caller runs the program on the tape.
constexpr int kLanesNoJit = 1000;
inline bool use_lanes(const mc_program* p, const mc_run_config* cfg) {
    return p->lr.ok && p->slice_kernel != 1 && cfg->num_leapfrog_steps > 0;
}

// Exchange tags of the lane-resident kernel continue across launches on one
// workspace: a process-wide counter per workspace address hands every launch
// a fresh tag range, so the granule lines need clearing only the first time
// the library sees a workspace (or after it is released, reused by another
// kernel, or the 32-bit counter would wrap) — not ahead of every launch.
inline std::mutex g_ws_mu;
struct WsTags {
    uint32_t epoch;    // last tag handed out
    uint64_t cleared;  // bytes of the workspace cleared when its tags started
};
inline std::unordered_map<const void*, WsTags> g_ws_epoch;
// workspaces whose last launch was an exchange kernel (k_hmc_sl / k_hmc_lr):
// only those hold a status word for mc_workspace_status
inline std::unordered_map<const void*, char> g_ws_status;
inline void ws_forget(const void* ws) {
    std::lock_guard<std::mutex> lk(g_ws_mu);
    g_ws_epoch.erase(ws);
    g_ws_status.erase(ws);
}
inline void ws_mark_status(const void* ws) {
    std::lock_guard<std::mutex> lk(g_ws_mu);
    g_ws_status[ws] = 1;
}
inline bool ws_has_status(const void* ws) {
    std::lock_guard<std::mutex> lk(g_ws_mu);
    return g_ws_status.count(ws) != 0;
}
// Reserve `need` tags on ws, whose launch uses `bytes` of it: *base = first
// tag - 1; returns true if the workspace must be cleared first — the first
// time, when the tags would wrap, or when the launch uses more of it than was
// cleared (a larger layout after mc_program_set_slices / set_slice_kernel
// would otherwise read stale words beyond the cleared range).
inline bool ws_reserve(const void* ws, uint64_t need, uint64_t bytes, uint32_t* base) {
    std::lock_guard<std::mutex> lk(g_ws_mu);
    auto it = g_ws_epoch.find(ws);
    const bool clear = it == g_ws_epoch.end() || (uint64_t)it->second.epoch + need >= 0xFFFFFFF0ull ||
                       bytes > it->second.cleared;
    *base = clear ? 0u : it->second.epoch;
    const uint64_t cleared = clear ? bytes : it->second.cleared;
    g_ws_epoch[ws] = WsTags{(uint32_t)(*base + need), cleared};
    return clear;
}



// the fast-form kernel (lanes_fast.h) for programs that qualify, unless
// MC_LANES_FAST=0 in the environment (A/B timing against k_hmc_lr)
inline int g_lanes_fast = -1;  // mc_debug_lanes_fast; -1: MC_LANES_FAST from the environment
inline bool lanes_fast_enabled() {
    if (g_lanes_fast < 0) {
        const char* e = std::getenv("MC_LANES_FAST");
        g_lanes_fast = (e && e[0] == '0') ? 0 : 1;
    }
    return g_lanes_fast == 1;
}

// compile-time forms of k_hmc_lf: MC_LANES_FORM=0 in the environment or
// mc_debug_lanes_forms(0) selects the run-time form kernel (A/B timing, tests)
inline int g_lanes_forms = -1;
inline bool lanes_forms_enabled() {
    if (g_lanes_forms < 0) {
        const char* e = std::getenv("MC_LANES_FORM");
        g_lanes_forms = (e && e[0] == '0') ? 0 : 1;
    }
    return g_lanes_forms == 1;
}

#ifdef MC_STAMPS
// diagnostic build only: copy out / reset the section stamp accumulators of
// the unit that defines these (eval.h's __device__ accumulators exist once per
// translation unit): mc_debug_stamps / _wg for the HMC kernels (run_hmc.hip),
// mc_debug_stamps_nuts / _nuts_wg for the NUTS kernels (run_nuts.hip)
#define MC_STAMPS_EXPORT(NAME, WGNAME)                                                   \
    extern "C" int NAME(unsigned long long* acc, unsigned long long* cnt, int reset) {     \
        if (acc) MC_HIP_TRY(hipMemcpyFromSymbol(acc, HIP_SYMBOL(mc_stamp_acc),              \
                                                sizeof(mc_stamp_acc)));                    \
        if (cnt) MC_HIP_TRY(hipMemcpyFromSymbol(cnt, HIP_SYMBOL(mc_stamp_cnt),              \
                                                sizeof(mc_stamp_cnt)));                    \
        if (reset) {                                                                       \
            unsigned long long z[16 * 32] = {0};                                           \
            MC_HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(mc_stamp_acc), z, sizeof(z)));          \
            MC_HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(mc_stamp_cnt), z, sizeof(z)));          \
            std::vector<unsigned long long> zw(1024 * 16, 0);                               \
            MC_HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(mc_stamp_wg), zw.data(), zw.size() * 8)); \
        }                                                                                  \
        return MC_OK;                                                                      \
    }                                                                                      \
    extern "C" int WGNAME(unsigned long long* wg) {                                        \
        MC_HIP_TRY(hipMemcpyFromSymbol(wg, HIP_SYMBOL(mc_stamp_wg), 1024 * 16 * 8));          \
        return MC_OK;                                                                      \
    }
#endif

// lane-resident HMC launches, one translation unit per register-slot count
// (run_lanes_rs*.hip)
int hmc_lanes_rs1(const mc_program*, const mc_run_config*, void*, float*, const mc_trace*, void*,
                  hipStream_t);
int hmc_lanes_rs2(const mc_program*, const mc_run_config*, void*, float*, const mc_trace*, void*,
                  hipStream_t);
int hmc_lanes_rs4(const mc_program*, const mc_run_config*, void*, float*, const mc_trace*, void*,
                  hipStream_t);
