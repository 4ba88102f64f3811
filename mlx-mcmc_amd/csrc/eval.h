// eval.h — the fused reverse-mode tape: log density + gradient of a program
// of distribution terms, evaluated by one chain group (WPC wavefronts).
//
// Replaces, per gradient evaluation, the reference's
//   grad_log_prob -> mx.grad(log_prob_fn)      (kernels/hmc.py:53-67,
//                                               kernels/nuts.py:76-87)
//   Normal.log_prob      (distributions/normal.py:49-56)
//   HalfNormal.log_prob  (distributions/halfnormal.py:43-63)
//   mx.sum over the likelihood (e.g. tests/test_hmc.py:196)
// with one sweep per term: forward value and hand-written VJP in the same
// loop, cotangents reduced in registers / LDS in a fixed order (no float
// atomics, so every evaluation is bit-reproducible).
//
// Two element mappings:
//   strided    element i -> thread i mod T (coalesced), for terms without a
//              non-injective gather;
//   segmented  terms gathered through a sorted group index (hierarchical
//              likelihoods): each lane owns one run of one group in a
//              host-built tiled layout, keeps theta_group in a register and
//              sums the group's cotangent in a register (csrc/api.hip
//              build_segments).
// Terms with a broadcast (uniform) scale accumulate moments per lane —
// count, sum d, sum d^2 with d = value - loc — and form log p and every
// cotangent from them once per lane: the per-element work is 3 VALU ops and
// there is no per-element division.  This is the same arithmetic as the
// per-element formulas up to fp32 rounding order.
#pragma once
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif
#include "internal.h"

#define MC_DEV __device__ __forceinline__

namespace mc {

// The program tables (terms, tile/lane/finalize tables) are read-only for the
// whole launch: reading them through the constant address space lets the
// compiler use scalar (SMEM) loads for wave-uniform fields instead of vector
// loads that it must re-issue after every store it cannot disambiguate.
#define MC_CONST __attribute__((address_space(4)))
// ---- diagnostic stamps (separate build with -DMC_STAMPS; never in the
// product library): wave 0 of workgroup 0 accumulates s_memtime deltas per
// section into mc_stamp_acc, read back with mc_debug_stamps().
#ifdef MC_STAMPS
__device__ unsigned long long mc_stamp_acc[16 * 32];  // [wave][section]
__device__ unsigned long long mc_stamp_cnt[16 * 32];
__device__ unsigned long long mc_stamp_wg[1024 * 16];  // [workgroup][section 0..15], wave 0
struct StampClock {
    unsigned long long last;
};
MC_DEV unsigned long long mc_now() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
// per-workgroup accumulators in LDS (a global read-modify-write per stamp
// would be waited for by every later barrier and inflate those sections)
MC_DEV unsigned long long* mc_stamp_lds() {
    __shared__ unsigned long long acc[2 * 16 * 32];
    return acc;
}
MC_DEV void stamp_init() {
    unsigned long long* a = mc_stamp_lds();
    for (int i = threadIdx.x; i < 2 * 16 * 32; i += blockDim.x) a[i] = 0;
    __syncthreads();
}
MC_DEV void stamp(StampClock& c, int sec) {
    const unsigned long long t = mc_now();
    if ((threadIdx.x & 63) == 0 && threadIdx.x < 16 * 64) {
        unsigned long long* a = mc_stamp_lds();
        a[(threadIdx.x >> 6) * 32 + sec] += t - c.last;
        a[512 + (threadIdx.x >> 6) * 32 + sec] += 1;
    }
    c.last = mc_now();
}
MC_DEV void stamp_flush() {
    if (threadIdx.x == 0 && blockIdx.x < 1024) {
        const unsigned long long* a = mc_stamp_lds();
        for (int s = 0; s < 16; ++s) mc_stamp_wg[blockIdx.x * 16 + s] += a[s];
    }
    if (blockIdx.x == 0 && (threadIdx.x & 63) == 0 && threadIdx.x < 16 * 64) {
        const unsigned long long* a = mc_stamp_lds();
        const int w = threadIdx.x >> 6;
        for (int s = 0; s < 32; ++s) {
            mc_stamp_acc[w * 32 + s] += a[w * 32 + s];
            mc_stamp_cnt[w * 32 + s] += a[512 + w * 32 + s];
        }
    }
}
#define MC_STAMP_INIT stamp_init();
#define MC_STAMP_FLUSH stamp_flush();
#define MC_STAMP_DECL StampClock mc_clk{mc_now()};
#define MC_STAMP(sec) stamp(mc_clk, sec)
#else
#define MC_STAMP_DECL
#define MC_STAMP(sec)
#define MC_STAMP_INIT
#define MC_STAMP_FLUSH
#endif

template <typename T>
MC_DEV const MC_CONST T* cptr(const T* p) {
    return (const MC_CONST T*)p;
}

// A term descriptor read field by field from the constant address space
// (uniform index -> scalar loads into SGPRs).
MC_DEV DevOperand load_op(const MC_CONST DevOperand* p) {
    DevOperand o;
    o.kind = p->kind;
    o.poff = p->poff;
    o.pool = p->pool;
    o.cval = p->cval;
    o.unique = p->unique;
    o.slot = p->slot;
    o.xf = p->xf;
    return o;
}

MC_DEV DevTerm load_term(const MC_CONST DevTerm* p) {
    DevTerm t;
    t.dist = p->dist;
    t.primary = p->primary;
    t.n = p->n;
    t.weight = p->weight;
    t.c0 = p->c0;
    t.npass = p->npass;
    t.pass_masks = p->pass_masks;
    t.prim_poff = p->prim_poff;
    t.wave_task = p->wave_task;
    t.clogs = p->clogs;
    t.clg = p->clg;
    t.op[0] = load_op(&p->op[0]);
    t.op[1] = load_op(&p->op[1]);
    t.op[2] = load_op(&p->op[2]);
    t.ntiles = p->ntiles;
    t.nvirt = p->nvirt;
    t.ncomb = p->ncomb;
    t.sync_before = p->sync_before;
    t.tile_base = p->tile_base;
    t.lane_base = p->lane_base;
    t.comb_base = p->comb_base;
    t.affine = p->affine;
    if (t.affine) {
        t.ab = load_op(&p->ab);
        t.ax = load_op(&p->ax);
    }
    t.expr_base = p->expr_base;
    t.expr_n = p->expr_n;
    return t;
}

// Wave-wide float sum, bit-identical in every lane.  Inside each 16-lane row
// a DPP butterfly (quad_perm xor 1, xor 2, half-row mirror, row mirror: each
// stage adds a pair in both orders, and fp add is commutative) leaves the row
// sum in all 16 lanes; the four row sums are then added in fixed order from
// SGPRs.  ~4 DPP adds + 4 readlanes, no LDS traffic.
template <int CTRL>
MC_DEV float dpp_row(float x) {
    return __int_as_float(
        __builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}
MC_DEV float wave_sum(float x) {
    x += dpp_row<0xB1>(x);   // quad_perm [1,0,3,2]
    x += dpp_row<0x4E>(x);   // quad_perm [2,3,0,1]
    x += dpp_row<0x141>(x);  // row_half_mirror
    x += dpp_row<0x140>(x);  // row_mirror
    const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 0));
    const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 16));
    const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 32));
    const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 48));
    return ((r0 + r1) + r2) + r3;
}
// N wave_sums side by side (bit-identical to wave_sum of each): the N DPP
// chains interleave, so a lone wave waits for one chain's latency.
template <int N>
MC_DEV void wave_sumN(float (&x)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) x[i] += dpp_row<0xB1>(x[i]);
#pragma unroll
    for (int i = 0; i < N; ++i) x[i] += dpp_row<0x4E>(x[i]);
#pragma unroll
    for (int i = 0; i < N; ++i) x[i] += dpp_row<0x141>(x[i]);
#pragma unroll
    for (int i = 0; i < N; ++i) x[i] += dpp_row<0x140>(x[i]);
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x[i]), 0));
        const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x[i]), 16));
        const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x[i]), 32));
        const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x[i]), 48));
        x[i] = ((r0 + r1) + r2) + r3;
    }
}
MC_DEV void wave_sum2(float (&x)[2]) { wave_sumN<2>(x); }

// A chain group: WPC wavefronts that together own one chain.  With WPC == 1
// several chains share a workgroup and never use the workgroup barrier.
template <int WPC>
struct Group {
    static constexpr int T = 64 * WPC;
    int tid;
    float* red;   // LDS scratch, WPC floats (sum())
    float* sred;  // LDS: per-wave partials of the broadcast-parameter cotangents
                  // and of log p, [slot][wave]

    MC_DEV void sync() const {
        if constexpr (WPC == 1) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        } else {
            __syncthreads();
        }
    }

    MC_DEV float sum(float x) const {
        x = wave_sum(x);
        if constexpr (WPC == 1) {
            return x;
        } else {
            if ((tid & 63) == 0) red[tid >> 6] = x;
            __syncthreads();
            float t = red[0];
#pragma unroll
            for (int w = 1; w < WPC; ++w) t += red[w];
            __syncthreads();
            return t;
        }
    }
};

// Deposit a wave's partial of cotangent slot `slot` (no barrier: the slots are
// summed in a fixed order once per evaluation, see eval_lp_grad).
template <int WPC>
MC_DEV void flush_slot(const Group<WPC>& G, int slot, float x) {
    x = wave_sum(x);
    if ((G.tid & 63) == 0) G.sred[slot * WPC + (G.tid >> 6)] = x;
}

// The same for a wave task: the one wave owns every entry of the slot.
template <int WPC>
MC_DEV void flush_slot_task(const Group<WPC>& G, int slot, float x) {
    x = wave_sum(x);
    const int lane = G.tid & 63;
    if (lane < WPC) G.sred[slot * WPC + lane] = (lane == 0) ? x : 0.0f;
}

// LDS scratch of a chain group beyond the reduction slots: the per-virtual-
// segment partial cotangents of a split segmented term (<= 4T floats).
struct SegScratch {
    float* vpart;
};

struct ElemOut {
    float lp, dv, dm, ds;
};

// normal.py:49-56:  lp = (log_norm - log(scale)) - (0.5 * (v - loc)^2) / scale^2
// VJP: d/dv = -(v-loc)/var, d/dloc = (v-loc)/var, d/dscale = (v-loc)^2/(var*s) - 1/s
MC_DEV ElemOut elem_normal(float c0, float v, float m, float s, float logs) {
    const float var = s * s;
    const float d = v - m;
    const float d2 = d * d;
    ElemOut o;
    o.lp = (c0 - logs) - (0.5f * d2) / var;
    const float t = d / var;
    o.dv = -t;
    o.dm = t;
    o.ds = d2 / (var * s) - 1.0f / s;
    return o;
}

// halfnormal.py:43-63: where(v >= 0, (log2 + log_norm - log s) - 0.5 v^2/s^2, -inf);
// the VJP of mx.where sends no cotangent through the -inf branch.
MC_DEV ElemOut elem_halfnormal(float c0, float v, float s, float logs) {
    ElemOut o;
    if (v >= 0.0f) {
        const float var = s * s;
        const float v2 = v * v;
        o.lp = (c0 - logs) - (0.5f * v2) / var;
        o.dv = -(v / var);
        o.ds = v2 / (var * s) - 1.0f / s;
    } else {
        o.lp = -__builtin_inff();
        o.dv = 0.0f;
        o.ds = 0.0f;
    }
    o.dm = 0.0f;
    return o;
}

// exponential.py:48-71: where(v >= 0, log(rate) - rate * v, -inf); operand
// slot 2 is the rate.
MC_DEV ElemOut elem_exponential(float v, float r, float logr) {
    ElemOut o;
    if (v >= 0.0f) {
        o.lp = logr - r * v;
        o.dv = -r;
        o.ds = 1.0f / r - v;
    } else {
        o.lp = -__builtin_inff();
        o.dv = 0.0f;
        o.ds = 0.0f;
    }
    o.dm = 0.0f;
    return o;
}

// gamma.py:48-59,61-88 (slots: value, alpha, beta):
//   log_norm = alpha * log(beta) - f32(gammaln(alpha))
//   where(v > 0, log_norm + (alpha - 1) * log(v) - beta * v, -inf)
// gammaln is the reference's host scipy value: it carries no gradient.
MC_DEV ElemOut elem_gamma(float v, float a, float b, float logb, float lga) {
    ElemOut o;
    if (v > 0.0f) {
        const float lv = logf(v);
        const float lnorm = a * logb - lga;
        o.lp = (lnorm + (a - 1.0f) * lv) - b * v;
        o.dv = (a - 1.0f) / v - b;
        o.dm = logb + lv;
        o.ds = a / b - v;
    } else {
        o.lp = -__builtin_inff();
        o.dv = o.dm = o.ds = 0.0f;
    }
    return o;
}

// beta.py:45-57,59-91 (slots: value, alpha, beta):
//   where(0 < v < 1, (alpha-1) log v + (beta-1) log(1-v) - logB(alpha, beta), -inf)
// logB from host scipy gammaln in the reference: no gradient.
MC_DEV ElemOut elem_beta(float v, float a, float b, float lbeta) {
    ElemOut o;
    if (v > 0.0f && v < 1.0f) {
        const float lv = logf(v);
        const float l1v = logf(1.0f - v);
        o.lp = ((a - 1.0f) * lv + (b - 1.0f) * l1v) - lbeta;
        o.dv = (a - 1.0f) / v - (b - 1.0f) / (1.0f - v);
        o.dm = lv;
        o.ds = l1v;
    } else {
        o.lp = -__builtin_inff();
        o.dv = o.dm = o.ds = 0.0f;
    }
    return o;
}

// An identity term (MC_DIST_IDENTITY): the value itself, cotangent 1.
MC_DEV ElemOut elem_identity(float v) {
    ElemOut o;
    o.lp = v;
    o.dv = 1.0f;
    o.dm = o.ds = 0.0f;
    return o;
}

// The fused distributions a kernel build evaluates (bit d: MC_DIST d): all
// of them, but the expression JIT (jit.hip gen_source) compiles only its
// program's, so that Gamma / Beta's float64 gammaln stays out of kernels that
// never run it.
#ifndef MC_JIT_DISTS
#define MC_JIT_DISTS 0x3Fu
#endif
constexpr bool dist_on(int d) { return ((MC_JIT_DISTS >> d) & 1u) != 0; }

// Every distribution: logs = f32 log of operand slot 2 (scale / rate / beta;
// unused by Beta), lg = the gammaln normaliser (Gamma, Beta; see lgamma_norm).
MC_DEV ElemOut elem_eval(int dist, float c0, float v, float m, float s, float logs, float lg) {
    switch (dist) {
        case MC_DIST_NORMAL:
            if constexpr (dist_on(MC_DIST_NORMAL)) return elem_normal(c0, v, m, s, logs);
            break;
        case MC_DIST_HALFNORMAL:
            if constexpr (dist_on(MC_DIST_HALFNORMAL)) return elem_halfnormal(c0, v, s, logs);
            break;
        case MC_DIST_EXPONENTIAL:
            if constexpr (dist_on(MC_DIST_EXPONENTIAL)) return elem_exponential(v, s, logs);
            break;
        case MC_DIST_GAMMA:
            if constexpr (dist_on(MC_DIST_GAMMA)) return elem_gamma(v, m, s, logs, lg);
            break;
        case MC_DIST_IDENTITY:
            if constexpr (dist_on(MC_DIST_IDENTITY)) return elem_identity(v);
            break;
        default:
            if constexpr (dist_on(MC_DIST_BETA)) return elem_beta(v, m, s, lg);
            break;
    }
    return ElemOut{0.0f, 0.0f, 0.0f, 0.0f};
}

// The gammaln normaliser as the reference forms it (float64 scipy gammaln of
// the float32 shapes, rounded once): Gamma lgamma(alpha); Beta
// lgamma(alpha) + lgamma(beta) - lgamma(alpha + beta).
__host__ __device__ inline float lgamma_norm(int dist, float a, float b) {
    if (dist == MC_DIST_GAMMA) return (float)lgamma((double)a);
    if (dist == MC_DIST_BETA)
        return (float)(lgamma((double)a) + lgamma((double)b) - lgamma((double)a + (double)b));
    return 0.0f;
}

// lgamma_norm in a kernel: compiled only where Gamma / Beta are (dist_on)
MC_DEV float lg_norm_dev(int dist, float a, float b) {
    if constexpr (!dist_on(MC_DIST_GAMMA) && !dist_on(MC_DIST_BETA)) return 0.0f;
    return lgamma_norm(dist, a, b);
}

// Does the normaliser vary per element (a vector shape operand)?
MC_DEV bool lg_per_element(int dist, int k1, int k2) {
    const bool v1 = k1 == MC_OP_DATA || k1 == MC_OP_PVEC || k1 == MC_OP_GATHER;
    const bool v2 = k2 == MC_OP_DATA || k2 == MC_OP_PVEC || k2 == MC_OP_GATHER;
    return (dist == MC_DIST_GAMMA && v1) || (dist == MC_DIST_BETA && (v1 || v2));
}

MC_DEV bool is_vec(int kind) {
    return kind == MC_OP_DATA || kind == MC_OP_PVEC || kind == MC_OP_GATHER;
}

// Transformed parameter operands (mc_transform_kind): the f32 value a term
// reads, and the VJP applied to its cotangent c as mx.grad's would be
// (exp: c * exp(x), from the forward value y; log: c / x).
MC_DEV float xf_apply(int xf, float x) {
    return xf == MC_XF_EXP ? expf(x) : (xf == MC_XF_LOG ? logf(x) : x);
}
MC_DEV float xf_chain(int xf, float c, float x, float y) {
    return xf == MC_XF_EXP ? c * y : (xf == MC_XF_LOG ? c / x : c);
}
// A PSCALAR operand's cotangent partial through its transform.
MC_DEV float xf_chain_scalar(const DevOperand& o, float c, const float* q) {
    if (o.xf == MC_XF_NONE) return c;
    const float x = q[o.poff];
    return xf_chain(o.xf, c, x, xf_apply(o.xf, x));
}

MC_DEV float uniform_value(const DevOperand& o, const float* q) {
    if (o.kind == MC_OP_PSCALAR) return xf_apply(o.xf, q[o.poff]);
    if (o.kind == MC_OP_CONST) return o.cval;
    return 0.0f;
}

// Per-lane moments of d = value - loc (Normal) or of the value (HalfNormal)
// for a term with a broadcast scale.
struct Moments {
    float cnt, s1, s2;
    bool neg;  // HalfNormal: some value < 0 (log p = -inf)
};

// log p and the broadcast-operand cotangents from the moments (per lane).
MC_DEV void finish_moments(const DevTerm& T, uint32_t mask, float s, float logs,
                           const Moments& M, float& lp_acc, float& pv, float& pm, float& ps) {
    const float w = T.weight;
    const float var = s * s;
    if (mask & PASS_LP) {
        const float lpt = M.neg ? -__builtin_inff() : (M.cnt * (T.c0 - logs) - (0.5f * M.s2) / var);
        lp_acc += w * lpt;
    }
    if ((mask & PASS_VALUE) && T.op[0].kind == MC_OP_PSCALAR) pv += -(w * (M.s1 / var));
    if ((mask & PASS_LOC) && T.op[1].kind == MC_OP_PSCALAR) pm += w * (M.s1 / var);
    if ((mask & PASS_SCALE) && T.op[2].kind == MC_OP_PSCALAR)
        ps += w * (M.s2 / (var * s) - M.cnt / s);
}

// ---------------------------------------------------------------------------
// strided mapping
// ---------------------------------------------------------------------------
// VK / LK: 0 broadcast, 1 DATA, 2 PVEC.  Broadcast scale.
template <int DIST, int VK, int LK>
MC_DEV void strided_uscale(const DevTerm& T, const DevCtx& P, const float* q, float* g, int tid,
                           int nthr, uint32_t mask, float uv, float um, float var, Moments& M) {
    const float* vd = (VK == 1) ? P.data + T.op[0].pool : (VK == 2 ? q + T.op[0].poff : nullptr);
    const float* ld = (LK == 1) ? P.data + T.op[1].pool : (LK == 2 ? q + T.op[1].poff : nullptr);
    float* gv = (VK == 2 && (mask & PASS_VALUE)) ? g + T.op[0].poff : nullptr;
    float* gl = (LK == 2 && (mask & PASS_LOC)) ? g + T.op[1].poff : nullptr;
    const float w = T.weight;
    const int64_t n = T.n;
    const float inv_var = 1.0f / var;
    float s1 = 0.0f, s2 = 0.0f, cnt = 0.0f;
    bool neg = false;
    for (int64_t i = tid; i < n; i += nthr) {
        const float v = (VK == 0) ? uv : vd[i];
        if constexpr (DIST == MC_DIST_NORMAL) {
            const float m = (LK == 0) ? um : ld[i];
            const float d = v - m;
            s2 = fmaf(d, d, s2);
            s1 += d;
            if (VK == 2 && gv) gv[i] += -(w * d) * inv_var;
            if (LK == 2 && gl) gl[i] += (w * d) * inv_var;
        } else {
            if (v >= 0.0f) {
                s2 = fmaf(v, v, s2);
                s1 += v;
                cnt += 1.0f;
                if (VK == 2 && gv) gv[i] += -(w * v) * inv_var;
            } else {
                neg = true;
            }
        }
    }
    if constexpr (DIST == MC_DIST_NORMAL) {
        cnt = (tid < n) ? (float)((n - 1 - tid) / nthr + 1) : 0.0f;
    }
    M.s1 += s1;
    M.s2 += s2;
    M.cnt += cnt;
    M.neg = M.neg || neg;
}

MC_DEV int fast_kind(const DevOperand& o) {
    const int kind = o.kind;
    if (o.xf != MC_XF_NONE && is_vec(kind)) return -1;  // transformed vector: generic path
    return kind == MC_OP_DATA ? 1 : (kind == MC_OP_PVEC ? 2 : (is_vec(kind) ? -1 : 0));
}

MC_DEV float fetch(const DevOperand& o, int64_t i, float uni, const float* q, const DevCtx& P) {
    switch (o.kind) {
        case MC_OP_DATA:
            return P.data[o.pool + i];
        case MC_OP_PVEC:
            return xf_apply(o.xf, q[o.poff + i]);
        case MC_OP_GATHER:
            return xf_apply(o.xf, q[o.poff + P.index[o.pool + i]]);
        default:
            return uni;
    }
}

// Accumulate a per-element cotangent for operand o (never the primary).
MC_DEV void accum(const DevOperand& o, int64_t i, float c, float& scalar_part, float* g,
                  const float* q, const DevCtx& P) {
    switch (o.kind) {
        case MC_OP_PSCALAR:
            scalar_part += c;  // (its transform: at the slot flush, xf_chain_scalar)
            break;
        case MC_OP_PVEC: {
            const int64_t j = o.poff + i;
            if (o.xf != MC_XF_NONE) c = xf_chain(o.xf, c, q[j], xf_apply(o.xf, q[j]));
            g[j] += c;
            break;
        }
        case MC_OP_GATHER: {
            const int64_t j = o.poff + P.index[o.pool + i];
            if (o.xf != MC_XF_NONE) c = xf_chain(o.xf, c, q[j], xf_apply(o.xf, q[j]));
            g[j] += c;
            break;
        }
        default:
            break;
    }
}

// Generic per-element path (vector scale, injective gathers): full formulas.
// Affine loc (T.affine): m = loc + slope * x per element (the reference's two
// f32 ops), and the loc cotangent cm also flows to the slope (cm * x, partial
// pb) and to x (cm * slope).
MC_DEV void strided_generic(const DevTerm& T, const DevCtx& P, const float* q, float* g, int tid,
                            int nthr, uint32_t mask, float uv, float um, float us, float ulogs,
                            float ulg, float& lp_acc, float& pv, float& pm, float& ps,
                            float& pb) {
    const bool scale_vec = is_vec(T.op[2].kind);
    const bool lgv = lg_per_element(T.dist, T.op[1].kind, T.op[2].kind);
    const float w = T.weight;
    const bool aff = T.affine != 0;
    const float ub = aff ? uniform_value(T.ab, q) : 0.0f;
    float dummy = 0.0f;
    for (int64_t i = tid; i < T.n; i += nthr) {
        const float v = fetch(T.op[0], i, uv, q, P);
        float m = fetch(T.op[1], i, um, q, P);
        float xa = 0.0f;
        if (aff) {
            xa = fetch(T.ax, i, 0.0f, q, P);
            m = m + ub * xa;
        }
        const float s = fetch(T.op[2], i, us, q, P);
        const float logs = scale_vec ? logf(s) : ulogs;
        const float lg = lgv ? lg_norm_dev(T.dist, m, s) : ulg;
        const ElemOut e = elem_eval(T.dist, T.c0, v, m, s, logs, lg);
        if (mask & PASS_LP) lp_acc += w * e.lp;
        if (mask & PASS_VALUE) accum(T.op[0], i, w * e.dv, pv, g, q, P);
        if (mask & PASS_LOC) {
            const float cm = w * e.dm;
            accum(T.op[1], i, cm, pm, g, q, P);
            if (aff) {
                pb += cm * xa;
                accum(T.ax, i, cm * ub, dummy, g, q, P);
            }
        }
        if (mask & PASS_SCALE) accum(T.op[2], i, w * e.ds, ps, g, q, P);
    }
}

// ---------------------------------------------------------------------------
// segmented mapping (terms grouped by a sorted, non-injective gather)
// ---------------------------------------------------------------------------
MC_DEV int64_t seg_elem(int off, int u, int lane) {
    return (int64_t)off + (u >> 2) * 256 + lane * 4 + (u & 3);
}

// Fast path: Normal, broadcast scale, primary in slot PV (0 value, 1 loc),
// the other of value/loc a DATA vector.  Per element: d, d^2 FMA, sum d.
template <int WPC, int PV>
MC_DEV void seg_normal_uscale(const DevTerm& T, const DevCtx& P, const float* q, float* g,
                              const Group<WPC>& G, uint32_t mask, float var, Moments& M,
                              float* vpart) {
    const int wave = G.tid >> 6;
    const int lane = G.tid & 63;
    const DevOperand& od = T.op[1 - PV];
    const MC_CONST int* tiles = cptr(P.index) + T.tile_base;
    const int* lanes = P.index + T.lane_base;
    const float* data = P.data + od.pool;
    const bool acc_prim = (mask & (1u << PV)) != 0;
    const bool split = T.ncomb > 0;
    const float w = T.weight;
    float s1_all = 0.0f, s2_all = 0.0f, cnt_all = 0.0f;
    // software pipeline over this wave's tiles: the next tile's lane record is
    // loaded while the current tile streams, and a tile's first data batch is
    // issued before its dependent theta read.
    int t = wave;
    int2 rec_n = make_int2(0, 0);
    if (t < T.ntiles && t * 64 + lane < T.nvirt)
        rec_n = reinterpret_cast<const int2*>(lanes)[t * 64 + lane];
    for (; t < T.ntiles; t += WPC) {
        const int off = tiles[3 * t];
        const int lpad = tiles[3 * t + 1];
        const int lmin = tiles[3 * t + 2];
        const int v = t * 64 + lane;
        const bool valid = v < T.nvirt;
        const int k = rec_n.x;
        const int len = rec_n.y;
        const int tn = t + WPC;
        rec_n = make_int2(0, 0);
        if (tn < T.ntiles && tn * 64 + lane < T.nvirt)
            rec_n = reinterpret_cast<const int2*>(lanes)[tn * 64 + lane];
        const float th = q[T.prim_poff + k];
        const float4* base = reinterpret_cast<const float4*>(data + off) + lane;
        float s1 = 0.0f, s2 = 0.0f;
        const int full4 = lmin >> 2;
        float s1b = 0.0f, s2b = 0.0f;  // two accumulator chains
        auto acc4 = [&](const float4 x) {
            const float d0 = PV == 1 ? x.x - th : th - x.x;
            const float d1 = PV == 1 ? x.y - th : th - x.y;
            const float d2 = PV == 1 ? x.z - th : th - x.z;
            const float d3 = PV == 1 ? x.w - th : th - x.w;
            s2 = fmaf(d0, d0, s2);
            s1 += d0;
            s2b = fmaf(d1, d1, s2b);
            s1b += d1;
            s2 = fmaf(d2, d2, s2);
            s1 += d2;
            s2b = fmaf(d3, d3, s2b);
            s1b += d3;
        };
        // batches of kBatch independent 16-byte loads in flight per lane; the
        // next batch is issued before the current one is consumed
        constexpr int kBatch = 4;
        const int nb = full4 / kBatch;
        float4 cur[kBatch];
        if (nb > 0) {
#pragma unroll
            for (int b = 0; b < kBatch; ++b) cur[b] = base[b * 64];
        }
        for (int bi = 0; bi < nb; ++bi) {
            float4 nxt[kBatch];
            const bool more = bi + 1 < nb;
            if (more) {
#pragma unroll
                for (int b = 0; b < kBatch; ++b) nxt[b] = base[((bi + 1) * kBatch + b) * 64];
            }
#pragma unroll
            for (int b = 0; b < kBatch; ++b) acc4(cur[b]);
            if (more) {
#pragma unroll
                for (int b = 0; b < kBatch; ++b) cur[b] = nxt[b];
            }
        }
        int u4 = nb * kBatch;
        if (u4 < full4) {
            const int r = full4 - u4;
            float4 x[kBatch];
#pragma unroll
            for (int b = 0; b < kBatch; ++b)
                if (b < r) x[b] = base[(u4 + b) * 64];
#pragma unroll
            for (int b = 0; b < kBatch; ++b)
                if (b < r) acc4(x[b]);
            u4 = full4;
        }
        for (; 4 * u4 < lpad; ++u4) {
            const float4 x = base[u4 * 64];
            const float xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if (4 * u4 + e < len) {
                    const float d = PV == 1 ? xs[e] - th : th - xs[e];
                    s2 = fmaf(d, d, s2);
                    s1 += d;
                }
            }
        }
        s1 += s1b;
        s2 += s2b;
        if (!valid) {  // lanes past the last virtual segment read padding
            s1 = 0.0f;
            s2 = 0.0f;
        }
        s1_all += s1;
        s2_all += s2;
        cnt_all += (float)len;
        if (valid && acc_prim) {
            const float c = PV == 1 ? w * (s1 / var) : -(w * (s1 / var));
            if (split) vpart[v] = c;
            else g[T.prim_poff + k] += c;
        }
    }
    M.s1 += s1_all;
    M.s2 += s2_all;
    M.cnt += cnt_all;
}

MC_DEV float seg_fetch(const DevOperand& o, int64_t e, float uni, float prim, bool is_prim,
                       const float* q, const DevCtx& P) {
    if (is_prim) return prim;
    switch (o.kind) {
        case MC_OP_DATA:
            return P.data[o.pool + e];
        case MC_OP_GATHER:
            return xf_apply(o.xf, q[o.poff + P.index[o.pool + e]]);
        default:
            return uni;
    }
}

// Generic segmented path: full per-element formulas.
template <int WPC>
MC_DEV void seg_generic(const DevTerm& T, const DevCtx& P, const float* q, float* g,
                        const Group<WPC>& G, uint32_t mask, float uv, float um, float us,
                        float ulogs, float ulg, float& lp_acc, float& pv, float& pm, float& ps,
                        float& pb, float* vpart) {
    const int wave = G.tid >> 6;
    const int lane = G.tid & 63;
    const int a = T.primary;
    const int prim_poff = T.prim_poff;
    const MC_CONST int* tiles = cptr(P.index) + T.tile_base;
    const int* lanes = P.index + T.lane_base;
    const bool acc_prim = (mask & (1u << a)) != 0;
    const bool split = T.ncomb > 0;
    const bool scale_vec = is_vec(T.op[2].kind);
    const bool lgv = lg_per_element(T.dist, a == 1 ? MC_OP_PVEC : T.op[1].kind,
                                    a == 2 ? MC_OP_PVEC : T.op[2].kind);
    const float w = T.weight;
    const bool aff = T.affine != 0;  // loc = (gathered) loc + slope * x, x data (tiled)
    const float ub = aff ? uniform_value(T.ab, q) : 0.0f;
    const int prim_xf = a == 0 ? T.op[0].xf : (a == 1 ? T.op[1].xf : T.op[2].xf);
    for (int t = wave; t < T.ntiles; t += WPC) {
        const int off = tiles[3 * t];
        const int lpad = tiles[3 * t + 1];
        const int v = t * 64 + lane;
        const bool valid = v < T.nvirt;
        const int k = valid ? lanes[2 * v] : 0;
        const int len = valid ? lanes[2 * v + 1] : 0;
        const float thx = q[prim_poff + k];
        const float th = xf_apply(prim_xf, thx);
        float cp = 0.0f;
        for (int u = 0; u < lpad; ++u) {
            if (u < len) {
                const int64_t e = seg_elem(off, u, lane);
                const float vv = seg_fetch(T.op[0], e, uv, th, a == 0, q, P);
                float m = seg_fetch(T.op[1], e, um, th, a == 1, q, P);
                const float xa = aff ? P.data[T.ax.pool + e] : 0.0f;
                if (aff) m = m + ub * xa;
                const float s = seg_fetch(T.op[2], e, us, th, a == 2, q, P);
                const float logs = (scale_vec || a == 2) ? logf(s) : ulogs;
                const float lg = lgv ? lg_norm_dev(T.dist, m, s) : ulg;
                const ElemOut o = elem_eval(T.dist, T.c0, vv, m, s, logs, lg);
                if (mask & PASS_LP) lp_acc += w * o.lp;
                if (mask & PASS_VALUE) {
                    if (a == 0) cp += w * o.dv;
                    else accum(T.op[0], e, w * o.dv, pv, g, q, P);
                }
                if (mask & PASS_LOC) {
                    const float cm = w * o.dm;
                    if (a == 1) cp += cm;
                    else accum(T.op[1], e, cm, pm, g, q, P);
                    if (aff) pb += cm * xa;
                }
                if (mask & PASS_SCALE) {
                    if (a == 2) cp += w * o.ds;
                    else accum(T.op[2], e, w * o.ds, ps, g, q, P);
                }
            }
        }
        if (valid && acc_prim) {
            cp = xf_chain(prim_xf, cp, thx, th);
            if (split) vpart[v] = cp;
            else g[prim_poff + k] += cp;
        }
    }
}

// ---------------------------------------------------------------------------
// expression terms (MC_DIST_EXPR, include/mcmc355.h mc_expr_node): the
// elementwise MLX expressions mx.grad differentiates in the reference
// (hmc.py:53-67), one f32 rounding per op, reverse mode per element.
// ---------------------------------------------------------------------------
constexpr int kExMaxNodes = MC_EXPR_MAX_NODES;

// The fused-term evaluation paths of eval_term (the strided moment sums per
// operand-kind code 0..11 — MC_JIT_SU bits — and the other three paths): a
// build compiles every one; the expression JIT (jit.hip) only those its
// program's fused terms take.
enum : uint32_t {
    MC_PATH_STRIDED_GENERIC = 1u,
    MC_PATH_SEG_NORMAL = 2u,
    MC_PATH_SEG_GENERIC = 4u,
};
#ifndef MC_JIT_PATHS
#define MC_JIT_PATHS 7u
#endif
#ifndef MC_JIT_SU
#define MC_JIT_SU 0xFFFu
#endif

// Division in expression nodes: the reciprocal unit's 1/y refined by one
// Newton step of the quotient, q + (x - y q) / y ~ q + (x - y q) r — within
// an ulp of the IEEE quotient (the residual x - y q is exact in an FMA),
// at 5 VALU beside the reciprocal instead of the ~10 of the scaled IEEE
// sequence (v_div_scale / v_div_fmas / v_div_fixup).  An element loop's
// uniform divisor keeps its reciprocal in a register.  v_div_fixup_f32
// replaces the quotient by the IEEE result where an operand is special (a
// zero or infinite divisor, infinite or NaN operands).  Divisors beyond 2^126
// in magnitude (their reciprocal is subnormal) are outside its range.
MC_DEV float ex_div(float x, float y) {
    const float r = __builtin_amdgcn_rcpf(y);
    const float q = x * r;
    const float e = __builtin_fmaf(-y, q, x);
    return __builtin_amdgcn_div_fixupf(__builtin_fmaf(e, r, q), y, x);
}

// exp and log in expression nodes: the transcendental unit (v_exp_f32 /
// v_log_f32, base 2) with the conversion to base e done in extended
// precision where it matters, ~1-2 ulp (ocml's expf / logf: ~1 ulp, about
// twice the instructions for their range and subnormal handling).
//   exp: t = x log2(e) rounded, its residual x log2(e) - t from an FMA plus
//        the low part of log2(e); exp2(t) (1 + residual ln 2).  Infinite or
//        zero exp2(t) (|x| beyond the range, +-inf) is returned as is.
//        Subnormal results are the unit's.
//   log: log2 of the argument (a subnormal one scaled by 2^32 first) times
//        ln 2; 0 -> -inf, negative -> NaN, inf -> inf.
MC_DEV float ex_exp(float x) {
    const float L = 1.44269502162933349609375f;     // f32 log2(e)
    const float Llo = 1.925963033500011079e-8f;      // log2(e) - L
    const float t = x * L;
    const float lo = __builtin_fmaf(x, L, -t) + x * Llo;
    const float r = __builtin_amdgcn_exp2f(t);
    const float c = lo * 0.693147180559945309f;
    return (r == 0.0f || __builtin_isinf(r)) ? r : __builtin_fmaf(r, c, r);
}
MC_DEV float ex_log(float x) {
    const bool sub = x < 1.17549435e-38f;  // subnormal, zero or negative
    const float r = __builtin_amdgcn_logf(sub ? x * 4294967296.0f : x);
    return (sub ? r - 32.0f : r) * 0.693147180559945309f;
}

// log(1 + x) from the rounded sum u = 1 + x: log(u) * (x / (u - 1))
// (the quotient corrects the rounding of u; exact for u - 1 == x), x where
// u rounds to 1, and log(u) for u = inf.  A few ulp, branch-free, against
// log1pf's ~40 instructions.
MC_DEV float ex_log1p(float x) {
    const float u = 1.0f + x;
    const float d = u - 1.0f;
    const float l = ex_log(u);
    const float r = __builtin_isinf(u) ? l : l * ex_div(x, d);
    return d == 0.0f ? x : r;
}

// The distribution nodes' element formulas: elem_normal / elem_halfnormal /
// elem_exponential's operations with their divisions through ex_div.
MC_DEV ElemOut ex_normal(float c0, float v, float m, float s, float logs) {
    const float var = s * s;
    const float d = v - m;
    const float d2 = d * d;
    ElemOut o;
    o.lp = (c0 - logs) - ex_div(0.5f * d2, var);
    const float t = ex_div(d, var);
    o.dv = -t;
    o.dm = t;
    o.ds = ex_div(d2, var * s) - ex_div(1.0f, s);
    return o;
}
MC_DEV ElemOut ex_halfnormal(float c0, float v, float s, float logs) {
    ElemOut o;
    if (v >= 0.0f) {
        const float var = s * s;
        const float v2 = v * v;
        o.lp = (c0 - logs) - ex_div(0.5f * v2, var);
        o.dv = -ex_div(v, var);
        o.ds = ex_div(v2, var * s) - ex_div(1.0f, s);
    } else {
        o.lp = -__builtin_inff();
        o.dv = 0.0f;
        o.ds = 0.0f;
    }
    o.dm = 0.0f;
    return o;
}
MC_DEV ElemOut ex_exponential(float v, float r, float logr) {
    ElemOut o;
    if (v >= 0.0f) {
        o.lp = logr - r * v;
        o.dv = -r;
        o.ds = ex_div(1.0f, r) - v;
    } else {
        o.lp = -__builtin_inff();
        o.dv = 0.0f;
        o.ds = 0.0f;
    }
    o.dm = 0.0f;
    return o;
}

// Gamma(a, b).log_prob(v) and Beta(a, b).log_prob(v) nodes (elem_gamma /
// elem_beta's operations, divisions and logs through ex_div / ex_log): the
// gammaln normaliser is the reference's host scipy value of the current
// float32 shapes — float64 lgamma rounded once — and carries no cotangent
// (gamma.py:48-59, beta.py:45-57), so the shape cotangents are log b + log v
// and log v / log(1 - v).  Outside the support: -inf, no cotangents (where).
MC_DEV float ex_gamma_lp(float v, float a, float b) {
    if (!(v > 0.0f)) return -__builtin_inff();
    const float lga = (float)lgamma((double)a);
    return ((a * ex_log(b) - lga) + (a - 1.0f) * ex_log(v)) - b * v;
}
MC_DEV void ex_gamma_grad(float v, float a, float b, float& dv, float& da, float& db) {
    if (!(v > 0.0f)) {
        dv = da = db = 0.0f;
        return;
    }
    dv = ex_div(a - 1.0f, v) - b;
    da = ex_log(b) + ex_log(v);
    db = ex_div(a, b) - v;
}
MC_DEV float ex_beta_lp(float v, float a, float b) {
    if (!(v > 0.0f && v < 1.0f)) return -__builtin_inff();
    const float lbeta = (float)(lgamma((double)a) + lgamma((double)b) - lgamma((double)a + (double)b));
    return ((a - 1.0f) * ex_log(v) + (b - 1.0f) * ex_log(1.0f - v)) - lbeta;
}
MC_DEV void ex_beta_grad(float v, float a, float b, float& dv, float& da, float& db) {
    if (!(v > 0.0f && v < 1.0f)) {
        dv = da = db = 0.0f;
        return;
    }
    dv = ex_div(a - 1.0f, v) - ex_div(b - 1.0f, 1.0f - v);
    da = ex_log(v);
    db = ex_log(1.0f - v);
}

// Forward value of a non-leaf node (x, y, z: its argument values; c0: the
// distribution nodes' f32 normaliser, as elem_normal / elem_halfnormal).
// Divisions go through ex_div, exp / log / log1p through ex_exp / ex_log /
// ex_log1p; sqrt / pow / tanh are ocml's.
MC_DEV float ex_fwd(int op, float x, float y, float z, float c0) {
    switch (op) {
        case MC_EX_ADD: return x + y;
        case MC_EX_SUB: return x - y;
        case MC_EX_MUL: return x * y;
        case MC_EX_DIV: return ex_div(x, y);
        case MC_EX_NEG: return -x;
        case MC_EX_EXP: return ex_exp(x);
        case MC_EX_LOG: return ex_log(x);
        case MC_EX_SQRT: return sqrtf(x);
        case MC_EX_SQUARE: return x * x;
        case MC_EX_POW: return powf(x, y);
        case MC_EX_ABS: return fabsf(x);
        case MC_EX_LOG1P: return ex_log1p(x);
        case MC_EX_TANH: return tanhf(x);
        case MC_EX_SIGMOID: return ex_div(1.0f, 1.0f + ex_exp(-x));
        case MC_EX_NORMAL_LP: return ex_normal(c0, x, y, z, ex_log(z)).lp;
        case MC_EX_HALFNORMAL_LP: return ex_halfnormal(c0, x, z, ex_log(z)).lp;
        case MC_EX_EXPONENTIAL_LP: return ex_exponential(x, z, ex_log(z)).lp;
        case MC_EX_WHERE: return x != 0.0f ? y : z;
        case MC_EX_GAMMA_LP: return ex_gamma_lp(x, y, z);
        case MC_EX_BETA_LP: return ex_beta_lp(x, y, z);
        // comparisons: 1 / 0 masks (false for a NaN operand, as mx.greater's);
        // their reverse step is zero (ex_bwd's default)
        case MC_EX_GT: return x > y ? 1.0f : 0.0f;
        case MC_EX_GE: return x >= y ? 1.0f : 0.0f;
        case MC_EX_LT: return x < y ? 1.0f : 0.0f;
        case MC_EX_LE: return x <= y ? 1.0f : 0.0f;
        default: return 0.0f;
    }
}

// Reverse step of a non-leaf node with value v and cotangent c: the
// cotangents of its arguments (mx.grad's VJPs: exp c*v, log c/x, sqrt
// c/(2v), pow c*y*x^(y-1) and c*v*log x, tanh c*(1-v^2), sigmoid
// c*v*(1-v); where: nothing to the mask, c to the branch taken).
MC_DEV void ex_bwd(int op, float x, float y, float z, float v, float c, float c0, float& dx,
                   float& dy, float& dz) {
    dx = dy = dz = 0.0f;
    switch (op) {
        case MC_EX_ADD: dx = c; dy = c; break;
        case MC_EX_SUB: dx = c; dy = -c; break;
        case MC_EX_MUL: dx = c * y; dy = c * x; break;
        case MC_EX_DIV: dx = ex_div(c, y); dy = -ex_div(c * x, y * y); break;
        case MC_EX_NEG: dx = -c; break;
        case MC_EX_EXP: dx = c * v; break;
        case MC_EX_LOG: dx = ex_div(c, x); break;
        case MC_EX_SQRT: dx = ex_div(c, 2.0f * v); break;
        case MC_EX_SQUARE: dx = c * (2.0f * x); break;
        case MC_EX_POW:
            dx = c * (y * powf(x, y - 1.0f));
            dy = c * (v * logf(x));
            break;
        case MC_EX_ABS: dx = x > 0.0f ? c : (x < 0.0f ? -c : 0.0f); break;
        case MC_EX_LOG1P: dx = ex_div(c, 1.0f + x); break;
        case MC_EX_TANH: dx = c * (1.0f - v * v); break;
        case MC_EX_SIGMOID: dx = c * (v * (1.0f - v)); break;
        case MC_EX_NORMAL_LP: {
            const ElemOut e = ex_normal(c0, x, y, z, ex_log(z));
            dx = c * e.dv;
            dy = c * e.dm;
            dz = c * e.ds;
            break;
        }
        case MC_EX_HALFNORMAL_LP: {
            const ElemOut e = ex_halfnormal(c0, x, z, ex_log(z));
            dx = c * e.dv;
            dz = c * e.ds;
            break;
        }
        case MC_EX_EXPONENTIAL_LP: {
            const ElemOut e = ex_exponential(x, z, ex_log(z));
            dx = c * e.dv;
            dz = c * e.ds;
            break;
        }
        case MC_EX_WHERE:
            if (x != 0.0f) dy = c;
            else dz = c;
            break;
        case MC_EX_GAMMA_LP:
        case MC_EX_BETA_LP: {
            float gv, ga, gb;
            if (op == MC_EX_GAMMA_LP) ex_gamma_grad(x, y, z, gv, ga, gb);
            else ex_beta_grad(x, y, z, gv, ga, gb);
            dx = c * gv;
            dy = c * ga;
            dz = c * gb;
            break;
        }
        default: break;
    }
}

// ---- two elements at once (the expression JIT's paired element code) -------
// The same operations as ex_fwd / ex_bwd on a pair of elements: the plain
// arithmetic packed (v_pk_add_f32 / v_pk_mul_f32 / v_pk_fma_f32 round every
// lane exactly as the scalar instruction), the transcendental unit, the
// fix-ups and the selects per component.  So each component is bit-identical
// to the scalar path's result for its element.
typedef float exf2 __attribute__((ext_vector_type(2)));

MC_DEV exf2 ex2_fma(exf2 a, exf2 b, exf2 c) { return __builtin_elementwise_fma(a, b, c); }
MC_DEV exf2 ex2_div(exf2 x, exf2 y) {
    const exf2 r = {__builtin_amdgcn_rcpf(y.x), __builtin_amdgcn_rcpf(y.y)};
    const exf2 q = x * r;
    const exf2 e = ex2_fma(-y, q, x);
    const exf2 q1 = ex2_fma(e, r, q);
    return exf2{__builtin_amdgcn_div_fixupf(q1.x, y.x, x.x),
                __builtin_amdgcn_div_fixupf(q1.y, y.y, x.y)};
}
MC_DEV exf2 ex2_exp(exf2 x) {
    const float L = 1.44269502162933349609375f;
    const float Llo = 1.925963033500011079e-8f;
    const exf2 t = x * L;
    const exf2 lo = ex2_fma(x, exf2{L, L}, -t) + x * Llo;
    const exf2 r = {__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
    const exf2 c = lo * 0.693147180559945309f;
    const exf2 f = ex2_fma(r, c, r);
    return exf2{(r.x == 0.0f || __builtin_isinf(r.x)) ? r.x : f.x,
                (r.y == 0.0f || __builtin_isinf(r.y)) ? r.y : f.y};
}
MC_DEV exf2 ex2_log(exf2 x) {
    const bool sx = x.x < 1.17549435e-38f, sy = x.y < 1.17549435e-38f;
    const exf2 xs = x * exf2{sx ? 4294967296.0f : 1.0f, sy ? 4294967296.0f : 1.0f};
    const exf2 r = {__builtin_amdgcn_logf(xs.x), __builtin_amdgcn_logf(xs.y)};
    return exf2{sx ? r.x - 32.0f : r.x, sy ? r.y - 32.0f : r.y} * 0.693147180559945309f;
}
MC_DEV exf2 ex2_log1p(exf2 x) {
    const exf2 u = 1.0f + x;
    const exf2 d = u - 1.0f;
    const exf2 l = ex2_log(u);
    const exf2 r = l * ex2_div(x, d);
    return exf2{d.x == 0.0f ? x.x : (__builtin_isinf(u.x) ? l.x : r.x),
                d.y == 0.0f ? x.y : (__builtin_isinf(u.y) ? l.y : r.y)};
}
MC_DEV exf2 ex2_each(float (*f)(float), exf2 x) { return exf2{f(x.x), f(x.y)}; }
// ex_normal's operations on a pair (every component rounds as the scalar
// path): log density, and the value / loc / scale cotangent factors.
MC_DEV exf2 ex2_normal_lp(float c0, exf2 v, exf2 m, exf2 s) {
    const exf2 var = s * s;
    const exf2 d = v - m;
    const exf2 d2 = d * d;
    return (c0 - ex2_log(s)) - ex2_div(0.5f * d2, var);
}
MC_DEV void ex2_normal_grad(exf2 v, exf2 m, exf2 s, exf2& dv, exf2& dm, exf2& ds) {
    const exf2 var = s * s;
    const exf2 d = v - m;
    const exf2 d2 = d * d;
    const exf2 t = ex2_div(d, var);
    dv = -t;
    dm = t;
    ds = ex2_div(d2, var * s) - ex2_div(exf2{1.0f, 1.0f}, s);
}

MC_DEV exf2 ex2_fwd(int op, exf2 x, exf2 y, exf2 z, float c0) {
    switch (op) {
        case MC_EX_ADD: return x + y;
        case MC_EX_SUB: return x - y;
        case MC_EX_MUL: return x * y;
        case MC_EX_DIV: return ex2_div(x, y);
        case MC_EX_NEG: return -x;
        case MC_EX_EXP: return ex2_exp(x);
        case MC_EX_LOG: return ex2_log(x);
        case MC_EX_SQUARE: return x * x;
        case MC_EX_LOG1P: return ex2_log1p(x);
        case MC_EX_SIGMOID: return ex2_div(exf2{1.0f, 1.0f}, 1.0f + ex2_exp(-x));
        case MC_EX_NORMAL_LP: return ex2_normal_lp(c0, x, y, z);
        default:  // the rest per component through the scalar path
            return exf2{ex_fwd(op, x.x, y.x, z.x, c0), ex_fwd(op, x.y, y.y, z.y, c0)};
    }
}
MC_DEV void ex2_bwd(int op, exf2 x, exf2 y, exf2 z, exf2 v, exf2 c, float c0, exf2& dx, exf2& dy,
                    exf2& dz) {
    dx = dy = dz = exf2{0.0f, 0.0f};
    switch (op) {
        case MC_EX_ADD: dx = c; dy = c; break;
        case MC_EX_SUB: dx = c; dy = -c; break;
        case MC_EX_MUL: dx = c * y; dy = c * x; break;
        case MC_EX_DIV: dx = ex2_div(c, y); dy = -ex2_div(c * x, y * y); break;
        case MC_EX_NEG: dx = -c; break;
        case MC_EX_EXP: dx = c * v; break;
        case MC_EX_LOG: dx = ex2_div(c, x); break;
        case MC_EX_SQUARE: dx = c * (2.0f * x); break;
        case MC_EX_LOG1P: dx = ex2_div(c, 1.0f + x); break;
        case MC_EX_TANH: dx = c * (1.0f - v * v); break;
        case MC_EX_SIGMOID: dx = c * (v * (1.0f - v)); break;
        case MC_EX_NORMAL_LP: {
            exf2 gv, gm, gs;
            ex2_normal_grad(x, y, z, gv, gm, gs);
            dx = c * gv;
            dy = c * gm;
            dz = c * gs;
            break;
        }
        default: {
            float ax, ay, az, bx, by, bz;
            ex_bwd(op, x.x, y.x, z.x, v.x, c.x, c0, ax, ay, az);
            ex_bwd(op, x.y, y.y, z.y, v.y, c.y, c0, bx, by, bz);
            dx = exf2{ax, bx};
            dy = exf2{ay, by};
            dz = exf2{az, bz};
            break;
        }
    }
}

// One expression term.  Strided (element i -> thread i mod nthr) or, with a
// non-injective gather (T.primary >= 0), per (virtual) segment of the
// segment-tiled layout (build_segments_ops), the gathered leaves read
// q[poff + k] and sum their cotangent in `part` over the run; runs split
// into virtual segments (few groups, T.ncomb > 0) leave one partial per
// gathered leaf in vpart (row prim - 1), added in order per group after a
// barrier, as the fused terms' are.  Vector leaves deposit in their pass only (sweeps separated by a
// group barrier: deterministic, no atomics); broadcast (PSCALAR) leaves sum
// per thread and flush to their cotangent slots after pass 0.
// NMAX: the node arrays' size.  Terms of <= 16 nodes run the NMAX = 16
// instantiation inlined into the (EX) kernel, whose value / adjoint /
// partial arrays the compiler keeps in registers (uniform dynamic indices:
// indirect register moves); larger terms run NMAX = 32, whose arrays live in
// scratch memory (slower per node: every argument read waits for a scratch
// load; 3 x 32 VGPRs are not affordable).
template <int WPC, bool VALUE_ONLY, int NMAX>
MC_DEV void eval_expr_n(const DevTerm& T, const DevCtx& P, const float* q, float* g,
                        const Group<WPC>& G, bool task, int tid, int nthr, float& lp_acc,
                        float* vpart) {
    const MC_CONST DevExprNode* N = cptr(P.nodes) + T.expr_base;
    const int nn = T.expr_n;
    const float w = T.weight;
    const bool seg = T.primary >= 0;
    const bool split = seg && T.ncomb > 0;
    float val[NMAX], adj[NMAX], part[NMAX];
    // the node descriptors, read once per term: lane k of these registers
    // holds node k (packed op / arguments / flags, leaf offsets, constant);
    // a node visit reads them with readlane into SGPRs (re-reading them from
    // constant memory per node and element cost ~20 scalar loads per element)
    int dcode = 0, dpoff = 0, dpool = 0;
    float dcval = 0.0f;
    {
        const int ln = G.tid & 63;
        if (ln < nn) {
            const MC_CONST DevExprNode* d = N + ln;
            dcode = (d->op & 31) | ((d->a + 1) << 5) | ((d->b + 1) << 11) | ((d->c + 1) << 17) |
                    ((d->prim != 0 ? 1 : 0) << 23) | ((d->pass & 15) << 24) | ((d->leaf.kind & 7) << 28);
            dpoff = d->leaf.poff;
            dpool = (int)d->leaf.pool;
            dcval = d->leaf.cval;
        }
    }
    auto code = [&](int k) { return __builtin_amdgcn_readlane(dcode, k); };
    auto cop = [](int d) { return d & 31; };
    auto carg = [](int d, int sh) { return ((d >> sh) & 63) - 1; };
    auto cprim = [](int d) { return ((d >> 23) & 1) != 0; };
    auto cpass = [](int d) { return (d >> 24) & 15; };
    auto ckind = [](int d) { return (d >> 28) & 7; };
    auto cval_of = [&](int k) {
        return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dcval), k));
    };
    const int npass = VALUE_ONLY ? 1 : T.npass;
    for (int pass = 0; pass < npass; ++pass) {
        for (int k = 0; k < nn; ++k) part[k] = 0.0f;
        // element e (strided index, or tiled position), run parameter kr
        auto element = [&](int64_t e, int kr) {
            for (int k = 0; k < nn; ++k) {
                const int d = code(k);
                const int op = cop(d);
                float v;
                if (op == MC_EX_LEAF) {
                    const int kind = ckind(d);
                    const int poff = __builtin_amdgcn_readlane(dpoff, k);
                    if (cprim(d)) {
                        v = q[poff + kr];
                    } else if (kind == MC_OP_CONST) {
                        v = cval_of(k);
                    } else if (kind == MC_OP_PSCALAR) {
                        v = q[poff];
                    } else if (kind == MC_OP_DATA) {
                        v = P.data[__builtin_amdgcn_readlane(dpool, k) + e];
                    } else if (kind == MC_OP_PVEC) {
                        v = q[poff + e];
                    } else {
                        v = q[poff + P.index[__builtin_amdgcn_readlane(dpool, k) + e]];
                    }
                } else {
                    const int a = carg(d, 5), b = carg(d, 11), c = carg(d, 17);
                    v = ex_fwd(op, val[a], b >= 0 ? val[b] : 0.0f, c >= 0 ? val[c] : 0.0f,
                               cval_of(k));
                }
                val[k] = v;
            }
            if (pass == 0) lp_acc += w * val[nn - 1];
            if constexpr (VALUE_ONLY) return;
            for (int k = 0; k < nn; ++k) adj[k] = -0.0f;  // (-0 + x == x: jit.hip gen_term)
            adj[nn - 1] = w;
            for (int k = nn - 1; k >= 0; --k) {
                const float ck = adj[k];
                const int d = code(k);
                const int op = cop(d);
                if (op == MC_EX_LEAF) {
                    const int kind = ckind(d);
                    if (kind == MC_OP_PSCALAR || cprim(d)) {
                        part[k] += ck;
                    } else if ((kind == MC_OP_PVEC || kind == MC_OP_GATHER) && cpass(d) == pass) {
                        const int poff = __builtin_amdgcn_readlane(dpoff, k);
                        const int64_t j =
                            kind == MC_OP_PVEC
                                ? (int64_t)poff + e
                                : (int64_t)poff + P.index[__builtin_amdgcn_readlane(dpool, k) + e];
                        g[j] += ck;
                    }
                    continue;
                }
                const int a = carg(d, 5), b = carg(d, 11), c = carg(d, 17);
                float dx, dy, dz;
                ex_bwd(op, val[a], b >= 0 ? val[b] : 0.0f, c >= 0 ? val[c] : 0.0f, val[k], ck,
                       cval_of(k), dx, dy, dz);
                adj[a] += dx;
                if (b >= 0) adj[b] += dy;
                if (c >= 0) adj[c] += dz;
            }
        };
        if (!seg) {
            for (int64_t i = tid; i < T.n; i += nthr) element(i, 0);
        } else {
            const int wave = G.tid >> 6;
            const int lane = G.tid & 63;
            const MC_CONST int* tiles = cptr(P.index) + T.tile_base;
            const int* lanes = P.index + T.lane_base;
            for (int t = wave; t < T.ntiles; t += WPC) {
                const int off = tiles[3 * t];
                const int v = t * 64 + lane;
                const bool valid = v < T.nvirt;
                const int kr = valid ? lanes[2 * v] : 0;
                const int len = valid ? lanes[2 * v + 1] : 0;
                for (int k = 0; k < nn; ++k)
                    if (N[k].prim) part[k] = 0.0f;
                for (int u = 0; u < len; ++u) element(seg_elem(off, u, lane), kr);
                if (!VALUE_ONLY && valid) {
                    for (int k = 0; k < nn; ++k) {
                        if (!N[k].prim || N[k].pass != pass) continue;
                        if (split) vpart[(N[k].prim - 1) * T.nvirt + v] = part[k];
                        else g[N[k].leaf.poff + kr] += part[k];
                    }
                }
            }
            if (!VALUE_ONLY && split) {
                // split runs: each group's virtual-segment partials in order
                G.sync();
                const int* comb = P.index + T.comb_base;
                for (int c = G.tid; c < T.ncomb; c += G.T) {
                    const int kc = comb[3 * c], vf = comb[3 * c + 1], vc = comb[3 * c + 2];
                    for (int k = 0; k < nn; ++k) {
                        if (!N[k].prim || N[k].pass != pass) continue;
                        const float* vp = vpart + (N[k].prim - 1) * T.nvirt;
                        float sum = vp[vf];
                        for (int j = 1; j < vc; ++j) sum += vp[vf + j];
                        g[N[k].leaf.poff + kc] += sum;
                    }
                }
            }
        }
        if (!VALUE_ONLY && pass == 0) {
            for (int k = 0; k < nn; ++k) {
                if (N[k].op != MC_EX_LEAF || N[k].leaf.kind != MC_OP_PSCALAR) continue;
                if (task) flush_slot_task(G, N[k].leaf.slot, part[k]);
                else flush_slot(G, N[k].leaf.slot, part[k]);
            }
        }
        if (!VALUE_ONLY && pass + 1 < npass) G.sync();
    }
}

#ifdef MC_JIT
// The program's expression terms compiled to straight-line code (jit.hip:
// generated per program, compiled by hiprtc into the tape kernels' EX
// instantiations): the same operations in the same order as eval_expr_n's
// node walk, so the results are bit-identical to the interpreter's.
template <int WPC, bool VALUE_ONLY>
MC_DEV void mc_jit_expr(const DevTerm& T, const DevCtx& P, const float* q, float* g,
                        const Group<WPC>& G, bool task, int tid, int nthr, float& lp_acc,
                        float* vpart);
#endif

// (only in the EX kernel instantiations: the node arrays would otherwise
// raise the register count of every tape kernel.  Both variants are inlined:
// a call in a kernel turned every uniform branch of it into an exec-masked
// one — all 19 op cases of every node executed for every element, 20x slower)
template <int WPC, bool VALUE_ONLY>
MC_DEV void eval_expr(const DevTerm& T, const DevCtx& P, const float* q, float* g,
                      const Group<WPC>& G, bool task, int tid, int nthr, float& lp_acc,
                      float* vpart) {
#ifdef MC_JIT
    mc_jit_expr<WPC, VALUE_ONLY>(T, P, q, g, G, task, tid, nthr, lp_acc, vpart);
    return;
#endif
    if (T.expr_n <= 16)
        eval_expr_n<WPC, VALUE_ONLY, 16>(T, P, q, g, G, task, tid, nthr, lp_acc, vpart);
    else
        eval_expr_n<WPC, VALUE_ONLY, kExMaxNodes>(T, P, q, g, G, task, tid, nthr, lp_acc, vpart);
}

// ---------------------------------------------------------------------------
// VALUE_ONLY: the forward tape alone (Metropolis-Hastings, mh.h) — every
// sweep keeps only its PASS_LP work and nothing is written to g.
// EX: the program holds expression terms (separate kernel instantiations, so
// programs without them keep the register budget they had).
template <int WPC, bool VALUE_ONLY = false, bool EX = false>
MC_DEV void eval_term(const DevTerm& T, const DevCtx& P, const float* q, float* g,
                      const Group<WPC>& G, float& lp_acc, const SegScratch& S) {
    MC_STAMP_DECL
    const bool task = T.wave_task >= 0;
    if (task && (G.tid >> 6) != T.wave_task) return;  // another wave owns it
    const int tid = task ? (G.tid & 63) : G.tid;
    const int nthr = task ? 64 : G.T;
    if constexpr (EX) {
        if (T.dist == MC_DIST_EXPR) {
            eval_expr<WPC, VALUE_ONLY>(T, P, q, g, G, task, tid, nthr, lp_acc, S.vpart);
            return;
        }
    }
    // (a JIT build names the fused-term paths its program takes, jit.hip
    // gen_source: the others are compiled out — registers and code)
    constexpr uint32_t su_codes = MC_JIT_SU;
    constexpr uint32_t paths = MC_JIT_PATHS;
    if constexpr (paths == 0 && su_codes == 0) return;
    const float uv = uniform_value(T.op[0], q);
    const float um = uniform_value(T.op[1], q);
    const float us = uniform_value(T.op[2], q);
    const bool scale_vec = is_vec(T.op[2].kind);
    const float ulogs =
        scale_vec ? 0.0f : (T.op[2].kind == MC_OP_CONST ? T.clogs : logf(us));
    const float var = us * us;
    const bool normal = (T.dist == MC_DIST_NORMAL);
    const bool moment_dist = normal || T.dist == MC_DIST_HALFNORMAL;
    // the gammaln normaliser when it is the same for every element
    const float ulg = lg_per_element(T.dist, T.op[1].kind, T.op[2].kind)
                          ? 0.0f
                          : ((T.op[1].kind == MC_OP_PSCALAR || T.op[2].kind == MC_OP_PSCALAR)
                                 ? lg_norm_dev(T.dist, um, us)
                                 : T.clg);

    MC_STAMP(20);
    for (int pass = 0; pass < T.npass; ++pass) {
        const uint32_t mask =
            ((T.pass_masks >> (4 * pass)) & 0xFu) & (VALUE_ONLY ? PASS_LP : 0xFu);
        if (VALUE_ONLY && mask == 0) continue;  // uniform: no writes, no barrier needed
        float pv = 0.0f, pm = 0.0f, ps = 0.0f, pb = 0.0f;
        Moments M = {0.0f, 0.0f, 0.0f, false};
        bool moments = false;

        if (T.primary < 0) {
            const int fv = fast_kind(T.op[0]);
            const int fl = normal ? fast_kind(T.op[1]) : 0;
            if (moment_dist && !scale_vec && fv >= 0 && fl >= 0 && !T.affine) {
                moments = true;
                const int code = normal ? (fv * 3 + fl) : (9 + fv);
                switch (code) {
#define MC_SU(c, D_, V_, L_)                                                                \
    case c:                                                                                 \
        if constexpr ((su_codes >> c) & 1u)                                                 \
            strided_uscale<D_, V_, L_>(T, P, q, g, tid, nthr, mask, uv, um, var, M);        \
        break;
                    MC_SU(0, MC_DIST_NORMAL, 0, 0)
                    MC_SU(1, MC_DIST_NORMAL, 0, 1)
                    MC_SU(2, MC_DIST_NORMAL, 0, 2)
                    MC_SU(3, MC_DIST_NORMAL, 1, 0)
                    MC_SU(4, MC_DIST_NORMAL, 1, 1)
                    MC_SU(5, MC_DIST_NORMAL, 1, 2)
                    MC_SU(6, MC_DIST_NORMAL, 2, 0)
                    MC_SU(7, MC_DIST_NORMAL, 2, 1)
                    MC_SU(8, MC_DIST_NORMAL, 2, 2)
                    MC_SU(9, MC_DIST_HALFNORMAL, 0, 0)
                    MC_SU(10, MC_DIST_HALFNORMAL, 1, 0)
                    MC_SU(11, MC_DIST_HALFNORMAL, 2, 0)
#undef MC_SU
                    default:
                        break;
                }
            } else if constexpr ((paths & MC_PATH_STRIDED_GENERIC) != 0) {
                strided_generic(T, P, q, g, tid, nthr, mask, uv, um, us, ulogs, ulg, lp_acc, pv,
                                pm, ps, pb);
            }
        } else {
            float* vpart = S.vpart;
            const int other_kind = T.primary == 1 ? T.op[0].kind : T.op[1].kind;
            const int prim_xf = T.primary == 0 ? T.op[0].xf : (T.primary == 1 ? T.op[1].xf
                                                                                  : T.op[2].xf);
            const bool fast = normal && !scale_vec && T.primary <= 1 && other_kind == MC_OP_DATA &&
                              !T.affine && prim_xf == MC_XF_NONE;
            if (fast) {
                moments = true;
                if constexpr ((paths & MC_PATH_SEG_NORMAL) != 0) {
                    if (T.primary == 1)
                        seg_normal_uscale<WPC, 1>(T, P, q, g, G, mask, var, M, vpart);
                    else
                        seg_normal_uscale<WPC, 0>(T, P, q, g, G, mask, var, M, vpart);
                }
            } else if constexpr ((paths & MC_PATH_SEG_GENERIC) != 0) {
                seg_generic<WPC>(T, P, q, g, G, mask, uv, um, us, ulogs, ulg, lp_acc, pv, pm,
                                 ps, pb, vpart);
            }
            if (T.ncomb > 0 && (mask & (1u << T.primary))) {
                // split segments: add the virtual partials in order
                G.sync();
                const int prim_poff = T.prim_poff;
                const int* comb = P.index + T.comb_base;
                for (int c = G.tid; c < T.ncomb; c += G.T) {
                    const int k = comb[3 * c], vf = comb[3 * c + 1], vc = comb[3 * c + 2];
                    float s = vpart[vf];
                    for (int j = 1; j < vc; ++j) s += vpart[vf + j];
                    g[prim_poff + k] += s;
                }
            }
        }
        MC_STAMP(21);
        if (moments) finish_moments(T, mask, us, ulogs, M, lp_acc, pv, pm, ps);

        // broadcast-parameter cotangents: per-wave partials into their slots
        auto flush = [&](int slot, float x) {
            if (task) flush_slot_task(G, slot, x);
            else flush_slot(G, slot, x);
        };
        // (a transformed parameter's partial through its VJP first)
        if ((mask & PASS_VALUE) && T.op[0].kind == MC_OP_PSCALAR)
            flush(T.op[0].slot, xf_chain_scalar(T.op[0], pv, q));
        if ((mask & PASS_LOC) && T.op[1].kind == MC_OP_PSCALAR)
            flush(T.op[1].slot, xf_chain_scalar(T.op[1], pm, q));
        if ((mask & PASS_SCALE) && T.op[2].kind == MC_OP_PSCALAR)
            flush(T.op[2].slot, xf_chain_scalar(T.op[2], ps, q));
        if ((mask & PASS_LOC) && T.affine && T.ab.kind == MC_OP_PSCALAR)
            flush(T.ab.slot, xf_chain_scalar(T.ab, pb, q));
        if (!VALUE_ONLY && pass + 1 < T.npass) G.sync();  // passes exist because their writes overlap
        MC_STAMP(22);
    }
}

// Log density at q and its gradient into g (g may not alias q; unused and may
// be NULL with VALUE_ONLY).  Every thread
// of the group returns the same value.  Barriers: one after zeroing g (skipped
// when the caller zeroed it in its own sweep), one before a term whose vector
// writes overlap an earlier term's since the last barrier (host-computed
// sync_before), one before and one after the fixed-order slot reduction.
template <int WPC, bool VALUE_ONLY = false, bool EX = false>
MC_DEV float eval_lp_grad(const DevCtx& P, const float* q, float* g, const Group<WPC>& G,
                          const SegScratch& S, bool g_zeroed = false) {
    MC_STAMP_DECL
    if (!VALUE_ONLY && !g_zeroed) {
        for (int j = G.tid; j < P.D; j += G.T) g[j] = 0.0f;
        G.sync();
    }
    float lp_acc = 0.0f;
    const MC_CONST DevTerm* terms = cptr(P.terms);
    for (int t = 0; t < P.n_terms; ++t) {
        const DevTerm T = load_term(terms + t);
        if (!VALUE_ONLY && T.sync_before) G.sync();
        MC_STAMP(2 + 2 * (t < 7 ? t : 7));
        eval_term<WPC, VALUE_ONLY, EX>(T, P, q, g, G, lp_acc, S);
        MC_STAMP(3 + 2 * (t < 7 ? t : 7));
    }
    const int lp_slot = P.nslots - 1;
    flush_slot(G, lp_slot, lp_acc);
    G.sync();
    MC_STAMP(18);
    // broadcast parameters: sum their slots in (slot, wave) order
    const MC_CONST int* fin = cptr(P.index) + P.sfin_base;
    const int nsp = fin[0];
    const MC_CONST int* ids = fin + 1 + 3 * nsp;
    for (int i = G.tid; i < (VALUE_ONLY ? 0 : nsp); i += G.T) {
        const int poff = fin[1 + 3 * i], first = fin[2 + 3 * i], cnt = fin[3 + 3 * i];
        float t = 0.0f;
        for (int c = 0; c < cnt; ++c) {
            const float* sl = G.sred + ids[first + c] * WPC;
            float u = sl[0];
#pragma unroll
            for (int w = 1; w < WPC; ++w) u += sl[w];
            t = (c == 0) ? u : t + u;
        }
        g[poff] += t;
    }
    const float* ls = G.sred + lp_slot * WPC;
    float lp = ls[0];
#pragma unroll
    for (int w = 1; w < WPC; ++w) lp += ls[w];
    G.sync();
    MC_STAMP(19);
    return lp + P.lp_const;
}

// LDS floats of a chain group's evaluator scratch: reduction slots (16),
// segment partials (4T), cotangent slots (nslots x WPC).
__host__ __device__ constexpr int group_scratch_floats(int wpc, int nslots) {
    return 16 + 4 * 64 * wpc + nslots * wpc;
}

template <int WPC>
MC_DEV void carve_group(float* base, Group<WPC>& G, SegScratch& S) {
    G.red = base;
    S.vpart = base + 16;
    G.sred = base + 16 + 4 * 64 * WPC;
}

}  // namespace mc
