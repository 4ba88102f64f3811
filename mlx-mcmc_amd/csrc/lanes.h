// lanes.h — lane-resident sliced HMC: the work split of k_hmc_sl (sliced.h;
// reference hmc.py:7-206 per chain), with every chain's state in registers.
//
//   * A workgroup evaluates one data slice for a block of 16 chains; wave w
//     owns chains 2w and 2w+1 and runs their whole trajectory on its own: no
//     workgroup barrier inside the iteration loop.
//   * Each private parameter of the slice (theta_g with its groups'
//     observations) is dealt to one (lane, slot): lane j keeps q, p, grad of
//     its <= RS private parameters for both chains in VGPRs, and every term's
//     elements of that parameter are tiled so that lane j streams them
//     (element u of (slot r, lane j) at toff[r] + (u/4)*256 + 4j + u%4 of the
//     operand's region of the slice block, in LDS).  The gradient of a private
//     parameter is complete inside the lane.
//   * The broadcast ("shared") parameters (mu, tau, sigma) are replicated in
//     every lane of every slice: q, p, grad and their derived scale values
//     (1/x, 1/x^2, log x) are registers too.
//   * Per element both chains are advanced with packed FP32 (v_pk_add_f32 /
//     v_pk_fma_f32): d = x - theta, s1 += d, s2 = fma(d, d, s2) — three
//     instructions per element for two chains.
//   * Once per leapfrog step each wave publishes its two chains' records (log
//     p partial, shared-cotangent partials, kinetic partials) as tagged 8-byte
//     granules and polls the 16 slices' records of the same two chains; a
//     16-lane DPP row sums each item in a fixed tree (identical in every
//     slice), so all replicas of a shared parameter stay bit-identical and
//     every slice takes the same accept decision.  The scalar terms (priors of
//     the shared parameters) are then added in term order.
// Eligibility (host planner, api.hip plan_lanes): S <= 16, <= kLrMaxShared
// shared parameters, <= 64 * kLrMaxSlots private parameters per slice, and
// every per-element parameter operand private.  Results equal k_hmc_sl's up
// to fp32 summation order; runs are bit-reproducible and independent of how
// chains are split over launches or GPUs.
#pragma once
#include "sliced.h"

namespace mc {

constexpr int kLrMaxSlots = 4;   // private parameters per lane
constexpr int kLrMaxShared = 4;  // broadcast parameters
constexpr int kLrMaxNB = 16;     // chains per block: up to 8 waves x 2 chains
constexpr int kLrSlices = 16;    // max slices (one 16-lane DPP row per item)
constexpr int kLrExprData = 6;   // data leaves of a lane-resident expression term

// One term restricted to one slice.
struct LrTerm {
    int32_t dist;
    int32_t mode;     // 0: broadcast scale (moment sums), 1: per-element formula
    int32_t pp;       // operand slot of the per-element parameter, or -1 (chunk term)
    int32_t nslot;    // slots with elements (chunk term: 1)
    float weight, c0;
    float clogs, cinv, cinv2;  // CONST scale: f32 log(scale), 1/scale, 1/scale^2
    float clg;                 // Gamma / Beta with constant shapes: gammaln normaliser
    int32_t kind[3];  // SK_* of value, loc, scale
    int32_t jsh[3];   // SK_SHARED: shared ordinal
    int32_t doff[3];  // SK_DATA: float offset of the operand's tiled region (slice block)
    float cval[3];    // SK_CONST
    int32_t toff[kLrMaxSlots];   // per slot: tile offset inside an operand region
    int32_t lmin4[kLrMaxSlots];  // per slot: min (over lanes with elements) length / 4
    int32_t len_off;             // int32 [nslot][64] run lengths (slice block)
    int32_t sig;                 // LS_*: a specialised form, or LS_GENERIC
    // LS_AFF (affine loc: loc + b * x): the slope's kind (SK_SHARED / SK_CONST),
    // shared ordinal and constant, and the float offset of x's tile (its
    // elements tiled as the value's)
    int32_t kb, jb;
    float cb;
    int32_t xoff;
    // LS_EXPR (an expression term, MC_DIST_EXPR, over data, broadcast
    // parameters and constants): its node range in the program's node table
    // and the float offsets of its data leaves' tiles, in node order (tiled as
    // a chunk term's value)
    int32_t expr_base, expr_n;
    int32_t eoff[kLrExprData];
};

// Specialised term forms (Normal, broadcast scale, moment sums) with their
// operand kinds fixed at compile time: (value, loc, scale).
enum : int32_t {
    LS_GENERIC = 0,
    LS_DATA_PP_SH = 1,   // y ~ Normal(theta[g], sigma)        grouped likelihood
    LS_DATA_PP_C = 2,    // y ~ Normal(theta[g], const)
    LS_PP_SH_SH = 3,     // theta ~ Normal(mu, tau)            hierarchical prior
    LS_PP_C_C = 4,       // theta ~ Normal(const, const)
    LS_PP_DATA_SH = 5,   // theta ~ Normal(m_data, tau)
    LS_DATA_SH_SH = 6,   // y ~ Normal(mu, sigma)              chunked likelihood
    LS_DSCALE = 7,       // theta ~ Normal(m, s_i), y_i ~ Normal(theta_g, s_i): a per-element
                         // data scale (tiles of 1/s^2 and log s), one of value / loc private
    LS_AFF = 8,          // y ~ Normal(loc + b * x, sigma): an affine loc (mc_affine) over
                         // data x; loc private (alpha[g]), shared or constant, b shared or
                         // constant, a broadcast scale (lr_affine_term)
    LS_EXPR = 9,         // an expression term over data, broadcast parameters and
                         // constants (a GLM likelihood: logistic, two-predictor ...): its
                         // element code is generated and compiled per program by the
                         // expression JIT (jit.hip gen_lane_term, mc_jit_lane_expr)
};

// A scalar term (constants and shared parameters only), compact for LDS.
struct LrSterm {
    int32_t dist;
    int32_t kinds;  // SK_* of value | loc << 4 | scale << 8
    int32_t jsh;    // shared ordinals: value | loc << 4 | scale << 8
    float c0;
    float cval[3];
    float clogs;    // CONST scale: f32 log(scale)
    float clg;      // gammaln normaliser (constant shapes)
    float wn;       // weight * element count
    int32_t own;    // a prior of one shared parameter: value shared, Normal /
                    // HalfNormal with constant loc and scale
    float cinv;     // CONST scale: 1/scale
    int32_t raw;    // bit a: shared operand a reads the raw parameter of a
                    // transformed one (LrCtx::shxf; an identity term's log-Jacobian)
    int32_t pad[3];
};

struct LrCtx {
    const LrTerm* terms;    // [S][n_terms], the slice's active terms first
    const float* data;      // slice blocks
    const int64_t* blocks;  // per slice {data offset, floats, active terms, swept terms}
    const int32_t* gidx;    // [S][kLrMaxSlots][64]: global parameter of (slot, lane), -1
    const LrSterm* sterms;  // scalar terms (constants / shared parameters only)
    int32_t n_terms;
    int32_t n_sterms;
    int32_t n_sterms_generic;  // scalar terms that are not "own" priors
    int32_t S;
    int32_t Dsh;
    int32_t D;
    int32_t nitems;         // record per chain: lp, Dsh cotangents, K0, K1
    int32_t sdata_floats;   // LDS floats of a slice block (the scalar terms follow)
    float lp_const;
    int32_t shl[kLrMaxShared];  // global index of shared parameter k
    int32_t shxf[kLrMaxShared];  // its mc_transform_kind: every slice term (and
                                 // every scalar-term operand without the raw
                                 // bit) reads xf(q) (mx.exp(log_sigma) ...)
    float shid[kLrMaxShared];    // k_hmc_lf: the weights of the identity terms
                                 // over the raw parameter (its log-Jacobian)
    int32_t has_xf;              // a transform or an identity term (k_hmc_lf)
    const int4* rng;             // [S][64] lane RNG plan (lf_rng_*), or nullptr
    int32_t rep;                 // lanes per private parameter (1, 2, 4, 8 or 16):
                                 // a parameter's elements are split over the
                                 // `rep` lanes of its group (lanes j & ~(rep-1)
                                 // .. + rep-1), every lane of the group holds
                                 // its q, p, g; the group leader alone counts it
                                 // in kinetic energies, U-turn dots and stores
};

typedef float f2 __attribute__((ext_vector_type(2)));

// Sum over the `rep` lanes of this lane's group (rep in {1, 2, 4, 8, 16},
// uniform): an xor / mirror butterfly of DPP row operations, so every lane of
// a group computes the same additions in the same order and holds the same
// bits (a + b == b + a in IEEE arithmetic).  The private gradients of a
// replicated layout (LrCtx::rep) are the sums of the lanes' partials.
template <int LEVELS>
MC_DEV void grp_levels(float& a, float& b) {
    // quad_perm [1,0,3,2] (lanes 2i <-> 2i+1), quad_perm [2,3,0,1] (the halves
    // of a quad), row_half_mirror (the quads of 8 lanes), row_mirror (the
    // halves of a 16-lane row); two independent chains interleaved
    if (LEVELS >= 1) { a += dpp_row<0xB1>(a); b += dpp_row<0xB1>(b); }
    if (LEVELS >= 2) { a += dpp_row<0x4E>(a); b += dpp_row<0x4E>(b); }
    if (LEVELS >= 3) { a += dpp_row<0x141>(a); b += dpp_row<0x141>(b); }
    if (LEVELS >= 4) { a += dpp_row<0x140>(a); b += dpp_row<0x140>(b); }
}
// two values at once (one uniform switch, straight-line code per case)
MC_DEV void grp_sum2(float& a, float& b, int rep) {
    switch (rep) {
        case 2: grp_levels<1>(a, b); break;
        case 4: grp_levels<2>(a, b); break;
        case 8: grp_levels<3>(a, b); break;
        case 16: grp_levels<4>(a, b); break;
        default: break;
    }
}

MC_DEV f2 pk_fma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

// Wave-uniform read of lane `lane`'s value (lane is uniform).
MC_DEV float rl(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}
// A [kLrMaxShared] register array indexed by a per-lane or uniform ordinal.
MC_DEV float pick4(const float (&a)[kLrMaxShared], int k) {
    float v = a[0];
#pragma unroll
    for (int kk = 1; kk < kLrMaxShared; ++kk) v = (k == kk) ? a[kk] : v;
    return v;
}
// k is wave-uniform: a branch on it (an indexed store would put the array in
// scratch, selects would cost 4 adds per call)
MC_DEV void add4(float (&a)[kLrMaxShared][2], int k, int c, float x) {
    k = __builtin_amdgcn_readfirstlane(k);
    if (k == 0) {
        if (c) a[0][1] += x; else a[0][0] += x;
    } else if (k == 1) {
        if (c) a[1][1] += x; else a[1][0] += x;
    } else if (k == 2) {
        if (c) a[2][1] += x; else a[2][0] += x;
    } else {
        if (c) a[3][1] += x; else a[3][0] += x;
    }
}

// Moment sums of one lane's run for both chains (packed): DC bit 0 value is
// data, bit 1 loc is data; vv / mm the chains' non-data operand values.
template <int DC>
MC_DEV void lr_moments(const float* xv, const float* xm, int len, int lmin4, f2 vv, f2 mm,
                       f2& s1, f2& s2) {
    f2 a1 = {0.0f, 0.0f}, a2 = {0.0f, 0.0f};
    auto elem = [&](float x, float y) {
        f2 d;
        if (DC == 0) d = vv - mm;
        else if (DC == 1) d = (f2){x, x} - mm;
        else if (DC == 2) d = vv - (f2){y, y};
        else { const float t = x - y; d = (f2){t, t}; }
        a1 += d;
        a2 = pk_fma(d, d, a2);
    };
    int u4 = 0;
    for (; u4 + 4 <= lmin4; u4 += 4) {
        float4 a[4], c[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            a[q] = c[q] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (DC & 1) a[q] = *(const float4*)(xv + (u4 + q) * 256);
            if (DC & 2) c[q] = *(const float4*)(xm + (u4 + q) * 256);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            elem(a[q].x, c[q].x);
            elem(a[q].y, c[q].y);
            elem(a[q].z, c[q].z);
            elem(a[q].w, c[q].w);
        }
    }
    for (; u4 < lmin4; ++u4) {
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f), c = a;
        if (DC & 1) a = *(const float4*)(xv + u4 * 256);
        if (DC & 2) c = *(const float4*)(xm + u4 * 256);
        elem(a.x, c.x);
        elem(a.y, c.y);
        elem(a.z, c.z);
        elem(a.w, c.w);
    }
    for (int u = 4 * u4; u < len; ++u) {
        const int o = (u >> 2) * 256 + (u & 3);
        elem((DC & 1) ? xv[o] : 0.0f, (DC & 2) ? xm[o] : 0.0f);
    }
    s1 += a1;
    s2 += a2;
}

// Private parameters of the lane's slots, both chains.
template <int RS>
struct LrPriv {
    float q[RS][2], p[RS][2], g[RS][2];
};

// Shared parameters, distributed over the lanes: lane x < 2 Dsh holds
// parameter k = x / 2 of chain c = x % 2 (the other lanes hold inert values:
// q = 1, p = g = 0).  Uniform reads go through readlane.
struct LrShared {
    float q, p, g;
    float v;           // the value terms read: xf(q) for a transformed parameter
                       // (LrCtx::shxf, eval.h xf_apply), else q
    float is, iv, lg;  // 1/v, 1/v^2, f32 log v: the derived scale values
};

// One Normal term with a broadcast scale and compile-time operand kinds
// (value, loc, scale) = (K0, K1, K2): moment sums per lane, no per-term kind
// branches.  Same arithmetic as the generic path's moment branch.
template <int RS, int K0, int K1, int K2>
MC_DEV void lr_normal_term(const MC_CONST LrTerm* T, const float* sd, int j, LrPriv<RS>& R,
                           const LrShared& sh, float (&lpp)[2],
                           float (&gshp)[kLrMaxShared][2]) {
    constexpr int DC = (K0 == SK_DATA ? 1 : 0) | (K1 == SK_DATA ? 2 : 0);
    constexpr int PPS = (K0 == SK_PP) ? 0 : ((K1 == SK_PP) ? 1 : -1);
    const int nslot = T->nslot;
    const float w = T->weight, c0 = T->c0;
    const int j0 = T->jsh[0], j1 = T->jsh[1], j2 = T->jsh[2];
    const int32_t* lens = (const int32_t*)sd + T->len_off;
    float uv[2], um[2], is[2], iv[2], lg[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        uv[c] = (K0 == SK_SHARED) ? rl(sh.v, 2 * j0 + c) : (K0 == SK_CONST ? T->cval[0] : 0.0f);
        um[c] = (K1 == SK_SHARED) ? rl(sh.v, 2 * j1 + c) : (K1 == SK_CONST ? T->cval[1] : 0.0f);
        is[c] = (K2 == SK_SHARED) ? rl(sh.is, 2 * j2 + c) : T->cinv;
        iv[c] = (K2 == SK_SHARED) ? rl(sh.iv, 2 * j2 + c) : T->cinv2;
        lg[c] = (K2 == SK_SHARED) ? rl(sh.lg, 2 * j2 + c) : T->clogs;
    }
    float pv[2] = {0.f, 0.f}, pm[2] = {0.f, 0.f}, ps[2] = {0.f, 0.f};
#pragma unroll
    for (int r = 0; r < RS; ++r) {
        if (r >= nslot) break;
        const int len = lens[r * 64 + j];
        if (len <= 0) continue;
        const int toff = T->toff[r] + 4 * j;
        const float* x0 = sd + T->doff[0] + toff;
        const float* x1 = sd + T->doff[1] + toff;
        const f2 vv = (K0 == SK_PP) ? (f2){R.q[r][0], R.q[r][1]} : (f2){uv[0], uv[1]};
        const f2 mm = (K1 == SK_PP) ? (f2){R.q[r][0], R.q[r][1]} : (f2){um[0], um[1]};
        f2 s1 = {0.f, 0.f}, s2 = {0.f, 0.f};
        lr_moments<DC>(x0, x1, len, T->lmin4[r], vv, mm, s1, s2);
        const float cnt = (float)len;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const float lpt = cnt * (c0 - lg[c]) - (0.5f * s2[c]) * iv[c];
            lpp[c] += w * lpt;
            const float t = w * (s1[c] * iv[c]);
            if (PPS == 0) R.g[r][c] += -t;
            if (PPS == 1) R.g[r][c] += t;
            pv[c] += -t;
            pm[c] += t;
            ps[c] += w * ((s2[c] * iv[c] - cnt) * is[c]);
        }
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        if (K0 == SK_SHARED) add4(gshp, j0, c, pv[c]);
        if (K1 == SK_SHARED) add4(gshp, j1, c, pm[c]);
        if (K2 == SK_SHARED) add4(gshp, j2, c, ps[c]);
    }
}

// ---- sweep-ahead terms ------------------------------------------------------
// A "swept" term (Normal, broadcast scale, neither value nor loc a shared
// parameter: y ~ N(theta_g, sigma), theta ~ N(m, sigma) ...) needs only the
// private parameters for its moment sums; the shared scale enters only when
// they are finished.  So the sums of step l + 1 are taken while the records
// of step l travel, and finished once the shared parameters of step l + 1
// are known.  Same arithmetic as lr_normal_term.
constexpr int kLrSweep = 2;  // swept terms per slice (the planner puts them first)

template <int RS>
struct LrMoments {
    f2 s1[kLrSweep][RS], s2[kLrSweep][RS];
};

template <int RS, int K0, int K1>
MC_DEV void lr_sweep_term(const MC_CONST LrTerm* T, const float* sd, int j, const LrPriv<RS>& R,
                          f2 (&s1)[RS], f2 (&s2)[RS]) {
    constexpr int DC = (K0 == SK_DATA ? 1 : 0) | (K1 == SK_DATA ? 2 : 0);
    const int nslot = T->nslot;
    const int32_t* lens = (const int32_t*)sd + T->len_off;
    const f2 cv = {K0 == SK_CONST ? T->cval[0] : T->cval[1], K0 == SK_CONST ? T->cval[0] : T->cval[1]};
#pragma unroll
    for (int r = 0; r < RS; ++r) {
        s1[r] = (f2){0.f, 0.f};
        s2[r] = (f2){0.f, 0.f};
        if (r >= nslot) continue;
        const int len = lens[r * 64 + j];
        if (len <= 0) continue;
        const int toff = T->toff[r] + 4 * j;
        const f2 th = {R.q[r][0], R.q[r][1]};
        const f2 vv = (K0 == SK_PP) ? th : cv;
        const f2 mm = (K1 == SK_PP) ? th : cv;
        lr_moments<DC>(sd + T->doff[0] + toff, sd + T->doff[1] + toff, len, T->lmin4[r], vv, mm,
                       s1[r], s2[r]);
    }
}

template <int RS>
MC_DEV void lr_sweep(const MC_CONST LrTerm* tt, int nsweep, const float* sd, int j,
                     const LrPriv<RS>& R, LrMoments<RS>& M) {
#pragma unroll
    for (int t = 0; t < kLrSweep; ++t) {
        if (t >= nsweep) break;
        const MC_CONST LrTerm* T = tt + t;
        switch (T->sig) {
            case LS_DATA_PP_SH:
            case LS_DATA_PP_C: lr_sweep_term<RS, SK_DATA, SK_PP>(T, sd, j, R, M.s1[t], M.s2[t]); break;
            case LS_PP_DATA_SH: lr_sweep_term<RS, SK_PP, SK_DATA>(T, sd, j, R, M.s1[t], M.s2[t]); break;
            default: lr_sweep_term<RS, SK_PP, SK_CONST>(T, sd, j, R, M.s1[t], M.s2[t]); break;
        }
    }
}

// A "direct" term: theta ~ Normal(loc, scale) with value = the lane's private
// parameter, loc / scale broadcast (shared or constant), at most one element
// per parameter in this slice (hierarchical priors).  Evaluated in the finish
// from registers, with the moment branch's arithmetic at count 1.
constexpr int kLrDirect = 2;

// Per-lane element counts of the swept terms and presence of the direct
// terms, read once per launch from the slices' length tables.
template <int RS>
struct LrCounts {
    float cs[kLrSweep][RS];
    bool pd[kLrDirect][RS];
};

// Finish the swept terms from their moment sums, and evaluate the direct
// terms, at the current shared values.  Both chains at once in packed FP32
// (every lane operation rounds exactly as its scalar counterpart).
MC_DEV f2 f2s(float x) { return (f2){x, x}; }
template <int RS>
MC_DEV void lr_finish(const MC_CONST LrTerm* tt, int nsweep, int ndirect, LrPriv<RS>& R,
                      const LrShared& sh, const LrMoments<RS>& M, const LrCounts<RS>& K,
                      f2& lpp, float (&gshp)[kLrMaxShared][2]) {
#pragma unroll
    for (int t = 0; t < kLrSweep; ++t) {
        if (t >= nsweep) break;
        const MC_CONST LrTerm* T = tt + t;
        const int pp = T->pp, j2 = T->jsh[2];
        const bool shs = T->kind[2] == SK_SHARED;
        const f2 w = f2s(T->weight), c0 = f2s(T->c0);
        const f2 is = shs ? (f2){rl(sh.is, 2 * j2), rl(sh.is, 2 * j2 + 1)} : f2s(T->cinv);
        const f2 iv = shs ? (f2){rl(sh.iv, 2 * j2), rl(sh.iv, 2 * j2 + 1)} : f2s(T->cinv2);
        const f2 lg = shs ? (f2){rl(sh.lg, 2 * j2), rl(sh.lg, 2 * j2 + 1)} : f2s(T->clogs);
        f2 ps = {0.f, 0.f};
#pragma unroll
        for (int r = 0; r < RS; ++r) {
            const float cn = K.cs[t][r];
            if (cn == 0.0f) continue;
            const f2 cnt = f2s(cn), s1 = M.s1[t][r], s2 = M.s2[t][r];
            const f2 lpt = cnt * (c0 - lg) - (f2s(0.5f) * s2) * iv;
            lpp += w * lpt;
            const f2 u = w * (s1 * iv);
            if (pp == 0) {
                R.g[r][0] += -u[0];
                R.g[r][1] += -u[1];
            } else {
                R.g[r][0] += u[0];
                R.g[r][1] += u[1];
            }
            ps += w * ((s2 * iv - cnt) * is);
        }
        if (shs) {
            add4(gshp, j2, 0, ps[0]);
            add4(gshp, j2, 1, ps[1]);
        }
    }
#pragma unroll
    for (int t = 0; t < kLrDirect; ++t) {
        if (t >= ndirect) break;
        const MC_CONST LrTerm* T = tt + nsweep + t;
        const int j1 = T->jsh[1], j2 = T->jsh[2];
        const bool shm = T->kind[1] == SK_SHARED, shs = T->kind[2] == SK_SHARED;
        const f2 w = f2s(T->weight), c0 = f2s(T->c0);
        const f2 um = shm ? (f2){rl(sh.v, 2 * j1), rl(sh.v, 2 * j1 + 1)} : f2s(T->cval[1]);
        const f2 is = shs ? (f2){rl(sh.is, 2 * j2), rl(sh.is, 2 * j2 + 1)} : f2s(T->cinv);
        const f2 iv = shs ? (f2){rl(sh.iv, 2 * j2), rl(sh.iv, 2 * j2 + 1)} : f2s(T->cinv2);
        const f2 lg = shs ? (f2){rl(sh.lg, 2 * j2), rl(sh.lg, 2 * j2 + 1)} : f2s(T->clogs);
        f2 pm = {0.f, 0.f}, ps = {0.f, 0.f};
#pragma unroll
        for (int r = 0; r < RS; ++r) {
            if (!K.pd[t][r]) continue;
            const f2 d = (f2){R.q[r][0], R.q[r][1]} - um;
            const f2 s2 = pk_fma(d, d, f2s(0.0f));
            const f2 lpt = f2s(1.0f) * (c0 - lg) - (f2s(0.5f) * s2) * iv;
            lpp += w * lpt;
            const f2 u = w * (d * iv);
            R.g[r][0] += -u[0];
            R.g[r][1] += -u[1];
            pm += u;
            ps += w * ((s2 * iv - f2s(1.0f)) * is);
        }
        if (shm) {
            add4(gshp, j1, 0, pm[0]);
            add4(gshp, j1, 1, pm[1]);
        }
        if (shs) {
            add4(gshp, j2, 0, ps[0]);
            add4(gshp, j2, 1, ps[1]);
        }
    }
}

// A Normal term with a per-element data scale (LS_DSCALE): the planner
// stored 1/s^2 in the scale's tile and f32 log s in the private operand's
// tile; the other of value / loc is a constant, a shared parameter or data.
// Per element, both chains packed: d = value - loc,
// lp = (c0 - log s) - (0.5 d^2) / s^2, d lp / d value = -d / s^2.
template <int RS>
MC_DEV void lr_dscale_term(const MC_CONST LrTerm* T, const float* sd, int j, LrPriv<RS>& R,
                           const LrShared& sh, float (&lpp)[2],
                           float (&gshp)[kLrMaxShared][2]) {
    const int ppo = T->pp;  // 0: value private (loc the other), 1: loc private
    const int oth = 1 - ppo;
    const int ko = T->kind[oth], jo = T->jsh[oth];
    const int nslot = T->nslot;
    const f2 w = f2s(T->weight), c0 = f2s(T->c0), half = f2s(0.5f);
    const int32_t* lens = (const int32_t*)sd + T->len_off;
    const f2 uo = ko == SK_SHARED ? (f2){rl(sh.v, 2 * jo), rl(sh.v, 2 * jo + 1)}
                                  : f2s(T->cval[oth]);
    f2 lp = {0.f, 0.f}, po = {0.f, 0.f};
#pragma unroll
    for (int r = 0; r < RS; ++r) {
        if (r >= nslot) break;
        const int len = lens[r * 64 + j];
        if (len <= 0) continue;
        const int toff = T->toff[r] + 4 * j;
        const float* xo = sd + T->doff[oth] + toff;
        const float* xl = sd + T->doff[ppo] + toff;
        const float* xi = sd + T->doff[2] + toff;
        const f2 th = {R.q[r][0], R.q[r][1]};
        f2 gp = {0.f, 0.f};
        for (int u = 0; u < len; ++u) {
            const int o = (u >> 2) * 256 + (u & 3);
            const f2 other = ko == SK_DATA ? f2s(xo[o]) : uo;
            const f2 d = ppo == 0 ? th - other : other - th;
            const f2 iv = f2s(xi[o]);
            const f2 lpt = (c0 - f2s(xl[o])) - (half * (d * d)) * iv;
            lp += w * lpt;
            const f2 t = w * (d * iv);
            gp += ppo == 0 ? -t : t;
            po += ppo == 0 ? t : -t;
        }
        R.g[r][0] += gp[0];
        R.g[r][1] += gp[1];
    }
    lpp[0] += lp[0];
    lpp[1] += lp[1];
    if (ko == SK_SHARED) {
        add4(gshp, jo, 0, po[0]);
        add4(gshp, jo, 1, po[1]);
    }
}

// An affine-loc Normal term (LS_AFF; reference: the user's `alpha[g] + beta *
// x` or `a + b * x` as the loc of Normal(...).log_prob(y), hmc.py:53-67
// differentiated by mx.grad): per element, both chains packed,
//   m = loc + b * x (two f32 roundings, as the tape's strided_generic),
//   d = y - m, s1 += d, s2 = fma(d, d, s2), sx = fma(x, d, sx)
// (5 packed ops + 1 for m), then with the scale's 1/s, 1/s^2, log s:
//   log p += w (n (c0 - log s) - (0.5 s2) / s^2),
//   d/dloc = w s1 / s^2 (private: complete in the lane; shared: a partial),
//   d/db = w sx / s^2, d/ds = w (s2 / s^2 - n) / s.
// The loc is private (the lane's slot parameter: a grouped term tiled by
// group) or a chunk term's shared / constant value.
template <int RS, int K1>
MC_DEV void lr_affine_term(const MC_CONST LrTerm* T, const float* sd, int j, LrPriv<RS>& R,
                           const LrShared& sh, float (&lpp)[2],
                           float (&gshp)[kLrMaxShared][2]) {
    const int nslot = T->nslot;
    const f2 w = f2s(T->weight), c0 = f2s(T->c0), half = f2s(0.5f);
    const int j1 = T->jsh[1], j2 = T->jsh[2], jb = T->jb;
    const bool shs = T->kind[2] == SK_SHARED, shb = T->kb == SK_SHARED;
    const int32_t* lens = (const int32_t*)sd + T->len_off;
    const f2 um = (K1 == SK_SHARED) ? (f2){rl(sh.v, 2 * j1), rl(sh.v, 2 * j1 + 1)}
                                    : f2s(T->cval[1]);
    const f2 b = shb ? (f2){rl(sh.v, 2 * jb), rl(sh.v, 2 * jb + 1)} : f2s(T->cb);
    const f2 is = shs ? (f2){rl(sh.is, 2 * j2), rl(sh.is, 2 * j2 + 1)} : f2s(T->cinv);
    const f2 iv = shs ? (f2){rl(sh.iv, 2 * j2), rl(sh.iv, 2 * j2 + 1)} : f2s(T->cinv2);
    const f2 lg = shs ? (f2){rl(sh.lg, 2 * j2), rl(sh.lg, 2 * j2 + 1)} : f2s(T->clogs);
    f2 lp = {0.f, 0.f}, pm = {0.f, 0.f}, pb = {0.f, 0.f}, ps = {0.f, 0.f};
#pragma unroll
    for (int r = 0; r < RS; ++r) {
        if (r >= nslot) break;
        const int len = lens[r * 64 + j];
        if (len <= 0) continue;
        const int toff = T->toff[r] + 4 * j;
        const float* yv = sd + T->doff[0] + toff;
        const float* xv = sd + T->xoff + toff;
        const f2 mm = (K1 == SK_PP) ? (f2){R.q[r][0], R.q[r][1]} : um;
        f2 s1 = {0.f, 0.f}, s2 = {0.f, 0.f}, sx = {0.f, 0.f};
        auto elem = [&](float y, float x) {
            const f2 xx = f2s(x);
            const f2 m = mm + b * xx;
            const f2 d = f2s(y) - m;
            s1 += d;
            s2 = pk_fma(d, d, s2);
            sx = pk_fma(xx, d, sx);
        };
        int u = 0;
        for (; u + 4 <= len; u += 4) {
            const float4 Y = *(const float4*)(yv + (u >> 2) * 256);
            const float4 X = *(const float4*)(xv + (u >> 2) * 256);
            elem(Y.x, X.x);
            elem(Y.y, X.y);
            elem(Y.z, X.z);
            elem(Y.w, X.w);
        }
        for (; u < len; ++u) {
            const int o = (u >> 2) * 256 + (u & 3);
            elem(yv[o], xv[o]);
        }
        const f2 cnt = f2s((float)len);
        lp += w * (cnt * (c0 - lg) - (half * s2) * iv);
        const f2 t = w * (s1 * iv);
        if (K1 == SK_PP) {
            R.g[r][0] += t[0];
            R.g[r][1] += t[1];
        } else {
            pm += t;
        }
        pb += w * (sx * iv);
        ps += w * ((s2 * iv - cnt) * is);
    }
    lpp[0] += lp[0];
    lpp[1] += lp[1];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        if (K1 == SK_SHARED) add4(gshp, j1, c, pm[c]);
        if (shb) add4(gshp, jb, c, pb[c]);
        if (shs) add4(gshp, j2, c, ps[c]);
    }
}

// one affine term, by its loc's kind
template <int RS>
MC_DEV void lr_affine(const MC_CONST LrTerm* T, const float* sd, int j, LrPriv<RS>& R,
                      const LrShared& sh, float (&lpp)[2], float (&gshp)[kLrMaxShared][2]) {
    if (T->kind[1] == SK_PP) lr_affine_term<RS, SK_PP>(T, sd, j, R, sh, lpp, gshp);
    else if (T->kind[1] == SK_SHARED) lr_affine_term<RS, SK_SHARED>(T, sd, j, R, sh, lpp, gshp);
    else lr_affine_term<RS, SK_CONST>(T, sd, j, R, sh, lpp, gshp);
}

#ifdef MC_JIT_LANES
// An LS_EXPR term's lane sweep, generated per program (jit.hip
// gen_lane_term): both chains packed per element, the expression's forward
// values and reverse-mode adjoints as the tape's (eval.h ex2_fwd / ex2_bwd),
// its broadcast leaves' cotangents summed over the lane's run into gshp.
// need_lp: the step's log p is read (the trajectory's last step); otherwise
// the nodes only the log density needs are left out.
MC_DEV void mc_jit_lane_expr(const MC_CONST LrTerm* T, const float* sd, int j,
                             const LrShared& sh, float (&lpp)[2],
                             float (&gshp)[kLrMaxShared][2], bool need_lp);
// The same for one chain per wave (k_nuts_sl: lane K of sh holds shared
// ordinal K; two elements packed per instruction): log p into lpp, the
// shared cotangent partials into gsh[K].
MC_DEV void mc_jit_lane_expr1(const MC_CONST LrTerm* T, const float* sd, int j,
                              const LrShared& sh, float& lpp, float (&gsh)[kLrMaxShared]);
// Its log p alone (k_mh_sl's forward pass).
MC_DEV void mc_jit_lane_expr1v(const MC_CONST LrTerm* T, const float* sd, int j,
                               const LrShared& sh, float& lpp);
#endif

// Log p partial of this slice at the current point; private gradients
// (complete) into R.g, this lane's shared-cotangent partials into gshp.
// need_lp = false: the caller reads no log p of this point (an intermediate
// leapfrog step); terms that can skip work for it may, the others add theirs.
template <int RS>
MC_DEV void lr_eval(const MC_CONST LrTerm* tt, int t0, int nact, const float* sd, int j,
                    LrPriv<RS>& R, const LrShared& sh, float (&lpp)[2],
                    float (&gshp)[kLrMaxShared][2], bool need_lp = true) {
    (void)need_lp;
    for (int t = t0; t < nact; ++t) {
        const MC_CONST LrTerm* T = tt + t;
        switch (T->sig) {
            case LS_DATA_PP_SH:
                lr_normal_term<RS, SK_DATA, SK_PP, SK_SHARED>(T, sd, j, R, sh, lpp, gshp);
                continue;
            case LS_DATA_PP_C:
                lr_normal_term<RS, SK_DATA, SK_PP, SK_CONST>(T, sd, j, R, sh, lpp, gshp);
                continue;
            case LS_PP_SH_SH:
                lr_normal_term<RS, SK_PP, SK_SHARED, SK_SHARED>(T, sd, j, R, sh, lpp, gshp);
                continue;
            case LS_PP_C_C:
                lr_normal_term<RS, SK_PP, SK_CONST, SK_CONST>(T, sd, j, R, sh, lpp, gshp);
                continue;
            case LS_PP_DATA_SH:
                lr_normal_term<RS, SK_PP, SK_DATA, SK_SHARED>(T, sd, j, R, sh, lpp, gshp);
                continue;
            case LS_DATA_SH_SH:
                lr_normal_term<RS, SK_DATA, SK_SHARED, SK_SHARED>(T, sd, j, R, sh, lpp, gshp);
                continue;
            case LS_DSCALE:
                lr_dscale_term<RS>(T, sd, j, R, sh, lpp, gshp);
                continue;
            case LS_AFF:
                lr_affine<RS>(T, sd, j, R, sh, lpp, gshp);
                continue;
            case LS_EXPR:
#ifdef MC_JIT_LANES
                mc_jit_lane_expr(T, sd, j, sh, lpp, gshp, need_lp);
#endif
                // (the library's own instantiations never see one: a program
                // with LS_EXPR terms launches the JIT-compiled kernel or the tape)
                continue;
            default:
                break;
        }
        const int dist = T->dist, mode = T->mode, pp = T->pp, nslot = T->nslot;
        const int k0 = T->kind[0], k1 = T->kind[1], k2 = T->kind[2];
        const int j0 = T->jsh[0], j1 = T->jsh[1], j2 = T->jsh[2];
        const float w = T->weight, c0 = T->c0;
        const int32_t* lens = (const int32_t*)sd + T->len_off;
        // the chains' broadcast operand values and derived scale values
        float uv[2], um[2], us[2], is[2], iv[2], lg[2];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            uv[c] = k0 == SK_SHARED ? rl(sh.v, 2 * j0 + c) : (k0 == SK_CONST ? T->cval[0] : 0.f);
            um[c] = k1 == SK_SHARED ? rl(sh.v, 2 * j1 + c) : (k1 == SK_CONST ? T->cval[1] : 0.f);
            us[c] = k2 == SK_SHARED ? rl(sh.v, 2 * j2 + c) : (k2 == SK_CONST ? T->cval[2] : 0.f);
            is[c] = k2 == SK_SHARED ? rl(sh.is, 2 * j2 + c) : T->cinv;
            iv[c] = k2 == SK_SHARED ? rl(sh.iv, 2 * j2 + c) : T->cinv2;
            lg[c] = k2 == SK_SHARED ? rl(sh.lg, 2 * j2 + c) : T->clogs;
        }
        float pv[2] = {0.f, 0.f}, pm[2] = {0.f, 0.f}, ps[2] = {0.f, 0.f};
#pragma unroll
        for (int r = 0; r < RS; ++r) {
            if (r >= nslot) break;
            const int len = lens[r * 64 + j];
            if (len <= 0) continue;
            const int toff = T->toff[r] + 4 * j;
            const float* x0 = sd + T->doff[0] + toff;
            const float* x1 = sd + T->doff[1] + toff;
            const float* x2 = sd + T->doff[2] + toff;
            const float th[2] = {R.q[r][0], R.q[r][1]};
            float rc[2] = {0.f, 0.f};
            if (mode == 0) {
                f2 s1 = {0.f, 0.f}, s2 = {0.f, 0.f};
                float cnt[2];
                bool neg[2] = {false, false};
                if (dist == MC_DIST_NORMAL) {
                    const f2 vv = {k0 == SK_PP ? th[0] : uv[0], k0 == SK_PP ? th[1] : uv[1]};
                    const f2 mm = {k1 == SK_PP ? th[0] : um[0], k1 == SK_PP ? th[1] : um[1]};
                    const int dc = (k0 == SK_DATA ? 1 : 0) | (k1 == SK_DATA ? 2 : 0);
                    const int lmin4 = T->lmin4[r];
                    if (dc == 1) lr_moments<1>(x0, x1, len, lmin4, vv, mm, s1, s2);
                    else if (dc == 0) lr_moments<0>(x0, x1, len, lmin4, vv, mm, s1, s2);
                    else if (dc == 2) lr_moments<2>(x0, x1, len, lmin4, vv, mm, s1, s2);
                    else lr_moments<3>(x0, x1, len, lmin4, vv, mm, s1, s2);
                    cnt[0] = cnt[1] = (float)len;
                } else {
                    // HalfNormal: moments of the value over value >= 0
                    cnt[0] = cnt[1] = 0.0f;
                    float a1[2] = {0.f, 0.f}, a2[2] = {0.f, 0.f};
                    for (int u = 0; u < len; ++u) {
                        const float x = (k0 == SK_DATA) ? x0[(u >> 2) * 256 + (u & 3)] : 0.0f;
#pragma unroll
                        for (int c = 0; c < 2; ++c) {
                            const float d = (k0 == SK_DATA) ? x : (k0 == SK_PP ? th[c] : uv[c]);
                            if (d >= 0.0f) {
                                a1[c] += d;
                                a2[c] = fmaf(d, d, a2[c]);
                                cnt[c] += 1.0f;
                            } else {
                                neg[c] = true;
                            }
                        }
                    }
                    s1 = (f2){a1[0], a1[1]};
                    s2 = (f2){a2[0], a2[1]};
                }
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    const float lpt = neg[c] ? -__builtin_inff()
                                             : cnt[c] * (c0 - lg[c]) - (0.5f * s2[c]) * iv[c];
                    lpp[c] += w * lpt;
                    const float t = w * (s1[c] * iv[c]);
                    rc[c] = (pp == 0) ? -t : t;
                    pv[c] += -t;
                    pm[c] += t;
                    ps[c] += w * ((s2[c] * iv[c] - cnt[c]) * is[c]);
                }
            } else {
                // per-element formula, one chain at a time
                const bool lgv = (k1 == SK_DATA || k1 == SK_PP || k2 == SK_DATA || k2 == SK_PP);
                for (int c = 0; c < 2; ++c) {
                    const float thc = c ? th[1] : th[0];
                    const float uvc = c ? uv[1] : uv[0], umc = c ? um[1] : um[0];
                    const float usc = c ? us[1] : us[0];
                    const float lsc = (k2 == SK_PP) ? logf(thc) : (c ? lg[1] : lg[0]);
                    const float lgu = (k1 == SK_SHARED || k2 == SK_SHARED)
                                          ? lgamma_norm(dist, umc, usc) : T->clg;
                    float lpc = 0.f, rcc = 0.f, pvc = 0.f, pmc = 0.f, psc = 0.f;
                    for (int u = 0; u < len; ++u) {
                        const int o = (u >> 2) * 256 + (u & 3);
                        const float v = (k0 == SK_DATA) ? x0[o] : (k0 == SK_PP ? thc : uvc);
                        const float m = (k1 == SK_DATA) ? x1[o] : (k1 == SK_PP ? thc : umc);
                        const float sc = (k2 == SK_DATA) ? x2[o] : (k2 == SK_PP ? thc : usc);
                        const float ls = (k2 == SK_DATA) ? logf(sc) : lsc;
                        const float lgx = lgv ? lgamma_norm(dist, m, sc) : lgu;
                        const ElemOut e = elem_eval(dist, c0, v, m, sc, ls, lgx);
                        lpc += w * e.lp;
                        rcc += w * (pp == 0 ? e.dv : (pp == 1 ? e.dm : e.ds));
                        pvc += w * e.dv;
                        pmc += w * e.dm;
                        psc += w * e.ds;
                    }
                    if (c) {
                        lpp[1] += lpc; rc[1] = rcc; pv[1] += pvc; pm[1] += pmc; ps[1] += psc;
                    } else {
                        lpp[0] += lpc; rc[0] = rcc; pv[0] += pvc; pm[0] += pmc; ps[0] += psc;
                    }
                }
            }
            if (pp >= 0) {
                R.g[r][0] += rc[0];
                R.g[r][1] += rc[1];
            }
        }
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            if (k0 == SK_SHARED) add4(gshp, j0, c, pv[c]);
            if (k1 == SK_SHARED) add4(gshp, j1, c, pm[c]);
            if (k2 == SK_SHARED) add4(gshp, j2, c, ps[c]);
        }
    }
}

// The scalar terms (constants and shared parameters only).  Priors of one
// shared parameter ("own" terms) are evaluated by the lane holding that
// parameter (lane 2k + c): its cotangent stays in the lane, the log p terms
// are summed over k in order.  Any other scalar term is evaluated
// lane-parallel from the LDS copy (lane x: term x / 2, chain x % 2) and summed
// per chain with wave_sum8.  Every slice computes the same sums and adds them
// to the exchanged totals.  Results: lp[c] (uniform), g_self (this lane's
// shared parameter, lanes < 2 nsh).
// The lane's own prior (lanes < 2 Dsh; the planner keeps one per shared
// parameter), read once per launch.
struct LrOwn {
    bool on, hn;            // present; HalfNormal (else Normal)
    float m, cinv, cinv2;   // constant loc; 1/scale, 1/scale^2
    float c0l, wn;          // c0 - log(scale); weight * count
};
MC_DEV LrOwn lr_own_prior(int n_sterms, const LrSterm* st, int j, int nsh) {
    LrOwn o = {false, false, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (j >= 2 * nsh) return o;
    for (int t = 0; t < n_sterms; ++t) {
        const LrSterm& T = st[t];
        if (!T.own || (T.jsh & 15) != (j >> 1)) continue;
        o.on = true;
        o.hn = T.dist == MC_DIST_HALFNORMAL;
        o.m = ((T.kinds >> 4) & 15) == SK_CONST ? T.cval[1] : 0.0f;
        o.cinv = T.cinv;
        o.cinv2 = T.cinv * T.cinv;
        o.c0l = T.c0 - T.clogs;
        o.wn = T.wn;
        break;
    }
    return o;
}

MC_DEV void wave_sum8(const float (&v)[8], float (&out)[8]);
// g_self: the cotangent of the lane's parameter's value sh.v; g_raw: of its
// raw q (the raw-bit operands of a transformed parameter, lanes.h LrSterm).
MC_DEV void lr_scalar_terms(int n_sterms, int n_generic, const LrSterm* st, const LrOwn& own,
                            const LrShared& sh, int j, int nsh, float (&lp)[2], float& g_self,
                            float& g_raw) {
    const int xk = j >> 1;
    float lp_own = 0.0f, g_own = 0.0f;
    g_raw = 0.0f;
    if (own.on) {
        // moment form with the constant scale's reciprocals, as the sliced terms
        const float v = sh.v;
        const float d = own.hn ? v : v - own.m;
        const float d2 = d * d;
        const bool out = own.hn && !(v >= 0.0f);
        const float lpe = out ? -__builtin_inff() : own.c0l - (0.5f * d2) * own.cinv2;
        lp_own = own.wn * lpe;
        g_own = out ? 0.0f : own.wn * -(d * own.cinv2);
    }
    for (int k = 0; k < nsh; ++k) {
        lp[0] += rl(lp_own, 2 * k);
        lp[1] += rl(lp_own, 2 * k + 1);
    }
    g_self = g_own;
    if (n_generic == 0) return;
    // other scalar terms: every lane evaluates them for its chain c = j % 2 and
    // keeps the cotangent of its own shared parameter (k = j / 2); lanes 0 / 1
    // hold the chains' log p sums (term order)
    const int c = j & 1;
    float lpg = 0.0f;
    for (int t = 0; t < n_sterms; ++t) {
        const LrSterm& T = st[t];  // uniform address: LDS broadcast
        if (T.own) continue;
        const int k0 = T.kinds & 15, k1 = (T.kinds >> 4) & 15, k2 = (T.kinds >> 8) & 15;
        const int j0 = T.jsh & 15, j1 = (T.jsh >> 4) & 15, j2 = (T.jsh >> 8) & 15;
        const bool r0 = T.raw & 1, r1 = (T.raw >> 1) & 1, r2 = (T.raw >> 2) & 1;
        const float q0 = __shfl(r0 ? sh.q : sh.v, 2 * j0 + c);
        const float q1 = __shfl(r1 ? sh.q : sh.v, 2 * j1 + c);
        const float q2 = __shfl(r2 ? sh.q : sh.v, 2 * j2 + c);
        const float v = k0 == SK_SHARED ? q0 : (k0 == SK_CONST ? T.cval[0] : 0.f);
        const float m = k1 == SK_SHARED ? q1 : (k1 == SK_CONST ? T.cval[1] : 0.f);
        const float sc = k2 == SK_SHARED ? q2 : (k2 == SK_CONST ? T.cval[2] : 0.f);
        const float ls = (k2 == SK_CONST) ? T.clogs : logf(sc);
        const float lgx =
            (k1 == SK_SHARED || k2 == SK_SHARED) ? lgamma_norm(T.dist, m, sc) : T.clg;
        const ElemOut e = elem_eval(T.dist, T.c0, v, m, sc, ls, lgx);
        lpg += T.wn * e.lp;
        float y = 0.0f, yr = 0.0f;
        if (k0 == SK_SHARED && j0 == xk) (r0 ? yr : y) += T.wn * e.dv;
        if (k1 == SK_SHARED && j1 == xk) (r1 ? yr : y) += T.wn * e.dm;
        if (k2 == SK_SHARED && j2 == xk) (r2 ? yr : y) += T.wn * e.ds;
        g_self += y;
        g_raw += yr;
    }
    lp[0] += rl(lpg, 0);
    lp[1] += rl(lpg, 1);
}

// Wave totals of 8 values at once (a fixed tree, the same in every wave):
// v32/v16 swaps pair the values across lane halves / quarters, then one
// 16-lane DPP row sum per register; the total of value i is read from the row
// that holds it.
MC_DEV void wave_sum8(const float (&v)[8], float (&out)[8]) {
    float w[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {  // lanes 0-31: v[2m], lanes 32-63: v[2m+1]
        const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[2 * m]),
                                                        __float_as_uint(v[2 * m + 1]), false, false);
        w[m] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
    float x[2];
#pragma unroll
    for (int n = 0; n < 2; ++n) {  // per 32-lane half: lanes 0-15 w[2n], 16-31 w[2n+1]
        const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(w[2 * n]),
                                                        __float_as_uint(w[2 * n + 1]), false, false);
        x[n] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
#pragma unroll
    for (int n = 0; n < 2; ++n) {
        float t = x[n];
        t += dpp_row<0xB1>(t);
        t += dpp_row<0x4E>(t);
        t += dpp_row<0x141>(t);
        t += dpp_row<0x140>(t);
        // rows: 0 -> v[4n], 1 -> v[4n+2], 2 -> v[4n+1], 3 -> v[4n+3]
        out[4 * n + 0] = rl(t, 0);
        out[4 * n + 2] = rl(t, 16);
        out[4 * n + 1] = rl(t, 32);
        out[4 * n + 3] = rl(t, 48);
    }
}

// ---------------------------------------------------------------------------
// the sampler
// ---------------------------------------------------------------------------
// X1: a program of one slice (an unsliced program): no exchange — a
// compile-time flag so the sliced variants keep their code and registers.
// XL: records published with L2-resident stores (sliced.h
// granule_store_xcd: the block's slices share an XCD), the placement checked
// at the launch's first iteration.
template <int RS, int NSH, int NW, bool X1, bool XL = false>
__global__ void __launch_bounds__(64 * NW)
k_hmc_lr(LrCtx P, RunArgs A, int64_t chain_base, int64_t n_groups, mc_chain_scalars* scal,
         float* st_q, float* st_g, float* samples, TraceDev tr, unsigned long long* xch,
         int* status, uint32_t ebase) {
    constexpr int NB = 2 * NW;  // chains per block: wave w owns chains 2w, 2w + 1
    // record items: 0 lp, 1..NSH shared cotangents, NSH+1 K0, NSH+2 K1; pair
    // 2 item + c (chain c) is granule `pair` of the wave's line
    constexpr int NPAIR = 2 * (NSH + 3), NPASS = (NPAIR + 3) / 4;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const mc_run_config& cfg = A.cfg;
    if (!X1 && A.fault && blockIdx.x == gridDim.x - 1) return;  // test hook: never publishes
    const int tid = threadIdx.x;
    const int wave = tid >> 6, j = tid & 63;
    const int S = P.S, D = P.D, Dsh = P.Dsh;
    int64_t grp;
    int slice;
    {
        const int64_t w = blockIdx.x, nwg = gridDim.x;
        if (nwg % 8 == 0 && (nwg / 8) % S == 0) {  // a block's slices share an XCD (speed only)
            const int64_t x = w & 7, r = w >> 3;
            grp = x * ((nwg / 8) / S) + r / S;
            slice = (int)(r % S);
        } else {
            grp = w / S;
            slice = (int)(w % S);
        }
    }
    const int64_t C = cfg.num_chains;
    const int64_t cbase = chain_base + grp * NB;
    const int b0 = 2 * wave;
    int64_t cc[2];  // this wave's chains (clamped for reads and draws)
    bool live[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        live[c] = cbase + b0 + c < C;
        cc[c] = min(cbase + b0 + c, C - 1);
    }
    // this lane's shared parameter (lanes < 2 Dsh): k = j / 2 of chain c = j % 2
    const int xk = j >> 1, xc = j & 1;
    const bool xon = j < 2 * Dsh;
    int xg = P.shl[0];
#pragma unroll
    for (int k = 1; k < kLrMaxShared; ++k) xg = (xk == k) ? P.shl[k] : xg;
    const int64_t xch_id = xc ? cc[1] : cc[0];
    const bool xlive = xon && (xc ? live[1] : live[0]);
    const int rep = P.rep;                     // lanes per private parameter
    const bool lead = (j & (rep - 1)) == 0;    // this lane counts its parameters
    int xxf = P.shxf[0];  // the lane's parameter's transform
#pragma unroll
    for (int k = 1; k < kLrMaxShared; ++k) xxf = (xk == k) ? P.shxf[k] : xxf;
    xxf = xon ? xxf : MC_XF_NONE;

    float* sd = smem;
    const int64_t* blk = P.blocks + 4 * (int64_t)slice;
    const int64_t doff = blk[0];
    const int dlen = (int)blk[1];
    const int nact = (int)blk[2];
    const int nsweep = (int)(blk[3] & 255);          // active terms [0, nsweep): swept,
    const int ndirect = (int)((blk[3] >> 8) & 255);  // then ndirect direct terms
    const int nfast = nsweep + ndirect;
    for (int i = tid; 4 * i < dlen; i += 64 * NW)
        *(float4*)(sd + 4 * i) = *(const float4*)(P.data + doff + 4 * i);
    LrSterm* sst = (LrSterm*)(smem + P.sdata_floats);  // the scalar terms, after the block
    for (int i = tid; i < P.n_sterms * (int)(sizeof(LrSterm) / 16); i += 64 * NW)
        ((float4*)sst)[i] = ((const float4*)P.sterms)[i];

    // ---- registers: private slots and the lane's shared parameter ----------------
    LrPriv<RS> R;
    int gk[RS];
#pragma unroll
    for (int r = 0; r < RS; ++r) {
        gk[r] = P.gidx[((int64_t)slice * kLrMaxSlots + r) * 64 + j];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            R.q[r][c] = gk[r] >= 0 ? st_q[cc[c] * D + gk[r]] : 0.0f;
            R.g[r][c] = gk[r] >= 0 ? st_g[cc[c] * D + gk[r]] : 0.0f;
            R.p[r][c] = 0.0f;
        }
    }
    LrShared sh;
    sh.q = xon ? st_q[xch_id * D + xg] : 1.0f;
    sh.g = xon ? st_g[xch_id * D + xg] : 0.0f;
    sh.p = 0.0f;
    sh.v = xf_apply(xxf, sh.q);
    double eps[2];
    float lp[2];
    int nacc[2], ntot[2], wacc[2], wtot[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        eps[c] = scal[cc[c]].step_size;
        lp[c] = scal[cc[c]].logp;
        nacc[c] = scal[cc[c]].n_accept;
        ntot[c] = scal[cc[c]].n_total;
        wacc[c] = scal[cc[c]].warmup_accept;
        wtot[c] = scal[cc[c]].warmup_total;
    }
    MC_STAMP_INIT
    __syncthreads();  // the slice block is in LDS

    const MC_CONST LrTerm* tt = cptr(P.terms) + (int64_t)slice * P.n_terms;
    const LrOwn own = lr_own_prior(P.n_sterms, sst, j, Dsh);
    LrCounts<RS> KC;
#pragma unroll
    for (int t = 0; t < kLrSweep; ++t)
#pragma unroll
        for (int r = 0; r < RS; ++r) {
            KC.cs[t][r] = 0.0f;
            if (t < nsweep && r < tt[t].nslot)
                KC.cs[t][r] = (float)((const int32_t*)sd)[tt[t].len_off + r * 64 + j];
        }
#pragma unroll
    for (int t = 0; t < kLrDirect; ++t)
#pragma unroll
        for (int r = 0; r < RS; ++r) {
            KC.pd[t][r] = false;
            if (t < ndirect && r < tt[nsweep + t].nslot)
                KC.pd[t][r] = ((const int32_t*)sd)[tt[nsweep + t].len_off + r * 64 + j] > 0;
        }

    const int L = cfg.num_leapfrog_steps;
    uint32_t epoch = ebase;  // tags continue across launches (api.hip ws_reserve)
    bool ok = true;
    // granules: one 128-byte line per (wave, slice) record, written by one
    // store instruction of one wave (lane = pair), so a polled line is never
    // rewritten by another wave while it is read.  Per lane: its own line
    // (publish) and line j % 16 (poll), for both epoch parities.
    unsigned long long* gpub[2];
    unsigned long long* gpoll[2];
#pragma unroll
    for (int par = 0; par < 2; ++par) {
        unsigned long long* b = xch + (((int64_t)par * n_groups + grp) * (NB / 2) + wave) * S * 16;
        gpub[par] = b + slice * 16 + j;
        gpoll[par] = b + (j & 15) * 16 + (j >> 4);
    }
    const bool poll_lane = (j & 15) < S;
    const int64_t it_end = cfg.iter_begin + cfg.iter_count;
    // XL: the block's slices share an XCD (sliced.h xcd_announce / xcd_agree;
    // slots: granule 15 of each slice's parity-0 line of wave 0 — the record
    // pairs are granules 0 .. NPAIR - 1 < 15)
    static_assert(NPAIR <= 15, "granule 15 of a record line is the XCD check's");
    constexpr bool xchk = XL && !X1;
    unsigned long long* const xslots = xch + ((int64_t)grp * (NB / 2)) * S * 16 + 15;
    XcdPoll xpoll = {0ull};
    if (xchk && cfg.iter_count > 0)
        xpoll = xcd_announce(xslots, S, slice, ebase + 1, wave == 0 && j == 0);
    for (int64_t it = cfg.iter_begin; it < it_end && ok; ++it) {
        if (xchk && it == cfg.iter_begin) {  // (before the launch's first publish)
            const bool same = xcd_agree(xpoll, xslots, S, ebase + 1, ok);
            if (ok && slice == 0 && wave == 0 && j == 0)  // (one per block)
                __hip_atomic_fetch_add(status + (same ? 8 : 9), 1, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            if (!ok || !same) {  // nothing published: the chains keep their state
                __hip_atomic_store(status, ok ? 2 : 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = false;
                break;
            }
        }
        MC_STAMP_DECL
        const bool warm = it < cfg.num_warmup;
        float h[2], e[2];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            if (it == cfg.num_warmup) {  // hmc.py:175-180
                wacc[c] = nacc[c];
                wtot[c] = ntot[c];
                nacc[c] = 0;
                ntot[c] = 0;
            }
            h[c] = (float)(0.5 * eps[c]);
            e[c] = (float)eps[c];
        }
        const float xh = xc ? h[1] : h[0], xe = xc ? e[1] : e[0];
        // momentum: parameter g takes normal g % 4 of Philox block g / 4
        auto normal_of = [&](int g, int64_t chain) {
            const mc_u32x4 rr = mc_draw(cfg.seed, (uint32_t)(cfg.chain_offset + chain),
                                        (uint32_t)it, MC_RNG_TAG_MOMENTUM, 0, (uint32_t)(g >> 2));
            float z0, z1;
            if ((g & 3) < 2) mc_box_muller(rr.x, rr.y, &z0, &z1);
            else mc_box_muller(rr.z, rr.w, &z0, &z1);
            return (g & 1) ? z1 : z0;
        };
        float k0p[2] = {0.f, 0.f};
#pragma unroll
        for (int r = 0; r < RS; ++r) {
            if (gk[r] < 0) continue;
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const float z = normal_of(gk[r], cc[c]);
                R.p[r][c] = z;
                if (lead) k0p[c] += z * z;
            }
        }
        sh.p = xon ? normal_of(xg, xch_id) : 0.0f;
        const float K0w[2] = {wave_sum(k0p[0]), wave_sum(k0p[1])};
        float k0s[2] = {0.f, 0.f};  // the shared parameters' part, in parameter order
        {
            const float p2 = sh.p * sh.p;
            for (int k = 0; k < Dsh; ++k) {
                k0s[0] += rl(p2, 2 * k);
                k0s[1] += rl(p2, 2 * k + 1);
            }
        }
        // the start point, restored on rejection
        float q0[RS][2], g0[RS][2];
#pragma unroll
        for (int r = 0; r < RS; ++r)
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                q0[r][c] = R.q[r][c];
                g0[r][c] = R.g[r][c];
            }
        const float q0s = sh.q, g0s = sh.g;
        float lpn[2] = {lp[0], lp[1]}, K0[2] = {0.f, 0.f}, K1[2] = {0.f, 0.f};
        MC_STAMP(5);
        // kick + drift of step 0 (private and shared), then the swept terms'
        // moment sums at the new point
        auto drift_private = [&](bool second_half) {
#pragma unroll
            for (int c = 0; c < 2; ++c) {
#pragma unroll
                for (int r = 0; r < RS; ++r) {
                    float pj = R.p[r][c];
                    if (second_half) pj = pj + h[c] * R.g[r][c];  // end of the previous step
                    pj = pj + h[c] * R.g[r][c];
                    R.p[r][c] = pj;
                    R.q[r][c] = R.q[r][c] + e[c] * pj;
                }
            }
        };
        auto drift_shared = [&](bool second_half) {
            float pj = sh.p;
            if (second_half) pj = pj + xh * sh.g;
            pj = pj + xh * sh.g;
            sh.p = pj;
            sh.q = sh.q + xe * pj;
            sh.v = xf_apply(xxf, sh.q);  // (mx.exp(log_sigma) ...: the terms' value)
            sh.is = 1.0f / sh.v;
            sh.iv = 1.0f / (sh.v * sh.v);
            sh.lg = logf(sh.v);
        };
        LrMoments<RS> M;
        drift_private(false);
        drift_shared(false);
        lr_sweep<RS>(tt, nsweep, sd, j, R, M);
        for (int l = 0; l < L; ++l) {
            MC_STAMP(0);
            // step l at the point q(l+1): finish the swept terms (shared values
            // of this step are known), evaluate the others
            float gshp[kLrMaxShared][2];
#pragma unroll
            for (int k = 0; k < kLrMaxShared; ++k) gshp[k][0] = gshp[k][1] = 0.0f;
#pragma unroll
            for (int r = 0; r < RS; ++r) R.g[r][0] = R.g[r][1] = 0.0f;
            f2 lpp2 = {0.f, 0.f};
            lr_finish<RS>(tt, nsweep, ndirect, R, sh, M, KC, lpp2, gshp);
            float lpp[2] = {lpp2[0], lpp2[1]};
            lr_eval<RS>(tt, nfast, nact, sd, j, R, sh, lpp, gshp, l == L - 1);
            if (rep > 1) {  // a replicated parameter's gradient: its lanes' partials
#pragma unroll
                for (int r = 0; r < RS; ++r) grp_sum2(R.g[r][0], R.g[r][1], rep);
            }
            MC_STAMP(1);
            // the wave totals of the record, pair-indexed (2 item + chain)
            float rec[NPAIR];
            {
                float v8[8], t8[8];
                v8[0] = lpp[0];
                v8[1] = lpp[1];
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    v8[2 + 2 * k] = gshp[k][0];
                    v8[3 + 2 * k] = gshp[k][1];
                }
                wave_sum8(v8, t8);
#pragma unroll
                for (int x = 0; x < 8; ++x) rec[x] = t8[x];
                // the 4th shared parameter and the final kinetic partial
                float k1p[2] = {0.f, 0.f};
                if (l == L - 1 && lead) {
#pragma unroll
                    for (int c = 0; c < 2; ++c)
#pragma unroll
                        for (int r = 0; r < RS; ++r) {
                            const float pj = R.p[r][c] + h[c] * R.g[r][c];
                            k1p[c] += pj * pj;
                        }
                }
                if (NSH > 3 || l == L - 1) {
                    v8[0] = gshp[3][0];
                    v8[1] = gshp[3][1];
                    v8[2] = k1p[0];
                    v8[3] = k1p[1];
#pragma unroll
                    for (int x = 4; x < 8; ++x) v8[x] = 0.0f;
                    wave_sum8(v8, t8);
                }
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    if (NSH > 3) rec[8 + c] = t8[c];
                    rec[2 * (NSH + 1) + c] = (l == 0) ? K0w[c] : 0.0f;
                    rec[2 * (NSH + 2) + c] = (l == L - 1) ? t8[2 + c] : 0.0f;
                }
            }
            ++epoch;
            const int par = epoch & 1;
            // publish: lane x < NPAIR stores pair x (one slice: nothing to exchange)
            if (!X1 && j < NPAIR) {
                float v = rec[0];
#pragma unroll
                for (int x = 1; x < NPAIR; ++x) v = (j == x) ? rec[x] : v;
                granule_put(par ? gpub[1] : gpub[0], epoch, v, XL);
            }
            MC_STAMP(2);
            // the sweep at a higher wave priority than the latency-bound rest of
            // the step (k_hmc_lf: the two waves of a SIMD settle out of phase)
            __builtin_amdgcn_s_setprio(1);
            // while the records travel: the private parameters' next position
            // (their gradients are complete) and the swept terms' sums there,
            // and the scalar terms of this step
            if (l + 1 < L) {
                drift_private(true);
                lr_sweep<RS>(tt, nsweep, sd, j, R, M);
            }
            // poll: pass ps, lane x -> pair 4 ps + x / 16, slice x % 16.  The
            // first round is issued now and checked after the scalar terms
            unsigned long long* gp = par ? gpoll[1] : gpoll[0];
            unsigned long long y0[NPASS];
#pragma unroll
            for (int ps = 0; ps < NPASS; ++ps)
                y0[ps] = (!X1 && poll_lane && 4 * ps + (j >> 4) < NPAIR) ? granule_load(gp + 4 * ps) : 0ull;
            float slp[2] = {0.f, 0.f}, sg_self = 0.0f, sg_raw = 0.0f;
            lr_scalar_terms(P.n_sterms, P.n_sterms_generic, sst, own, sh, j, Dsh, slp, sg_self,
                            sg_raw);
            MC_STAMP(7);
            float vals[NPASS];
            uint32_t need = 0;
#pragma unroll
            for (int ps = 0; ps < NPASS; ++ps) {
                vals[ps] = 0.0f;
                if (!X1 && poll_lane && 4 * ps + (j >> 4) < NPAIR) {
                    if ((uint32_t)(y0[ps] >> 32) == epoch) vals[ps] = __uint_as_float((uint32_t)y0[ps]);
                    else need |= 1u << ps;
                }
            }
            uint32_t spins = 0;
            while (__ballot(need != 0)) {
                if (++spins > kSpinLimit) {
                    ok = false;
                    break;
                }
                // (no s_sleep between polls: the round trip paces them, as in
                // k_hmc_lf)
#pragma unroll
                for (int ps = 0; ps < NPASS; ++ps) {
                    if ((need >> ps) & 1u) {
                        const unsigned long long y = granule_load(gp + 4 * ps);
                        if ((uint32_t)(y >> 32) == epoch) {
                            vals[ps] = __uint_as_float((uint32_t)y);
                            need &= ~(1u << ps);
                        }
                    }
                }
            }
            if (!ok) {
                __hip_atomic_store(status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            MC_STAMP(3);
            __builtin_amdgcn_s_setprio(0);
            // slice sums: a fixed 16-lane DPP tree per pair, read from the row's lane 0
            float tot[4 * NPASS];
            if constexpr (X1) {
#pragma unroll
                for (int x = 0; x < 4 * NPASS; ++x) tot[x] = x < NPAIR ? rec[x] : 0.0f;
            } else {
#pragma unroll
                for (int ps = 0; ps < NPASS; ++ps) {
                    float t = vals[ps];
                    t += dpp_row<0xB1>(t);
                    t += dpp_row<0x4E>(t);
                    t += dpp_row<0x141>(t);
                    t += dpp_row<0x140>(t);
#pragma unroll
                    for (int row = 0; row < 4; ++row) tot[4 * ps + row] = rl(t, 16 * row);
                }
            }
            // totals: the slice sum plus the scalar terms' sum
            lpn[0] = (tot[0] + slp[0]) + P.lp_const;
            lpn[1] = (tot[1] + slp[1]) + P.lp_const;
            {
                float gx = 0.0f;
#pragma unroll
                for (int k = 0; k < NSH; ++k)
                    if (xk == k) gx = xc ? tot[2 + 2 * k + 1] : tot[2 + 2 * k];
                // the value's cotangent through the transform's VJP, then the
                // raw-parameter terms (eval.h xf_chain: the tape's arithmetic)
                sh.g = xon ? xf_chain(xxf, gx + sg_self, sh.q, sh.v) + sg_raw : 0.0f;
            }
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                if (l == 0) K0[c] = tot[2 * (NSH + 1) + c];
                if (l == L - 1) K1[c] = tot[2 * (NSH + 2) + c];
            }
            if (l + 1 < L) drift_shared(true);  // the shared parameters' next position
            MC_STAMP(4);
        }
        if (!ok) break;
        // ---- accept / adapt (identical in every slice of the block) ------------
        float k1s[2] = {0.f, 0.f};
        {
            const float p1 = sh.p + xh * sh.g;
            const float p2 = p1 * p1;
            for (int k = 0; k < Dsh; ++k) {
                k1s[0] += rl(p2, 2 * k);
                k1s[1] += rl(p2, 2 * k + 1);
            }
        }
        bool acc[2];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const float H0 = -lp[c] + 0.5f * (K0[c] + k0s[c]);
            const float H1 = -lpn[c] + 0.5f * (K1[c] + k1s[c]);
            const float ratio = -(H1 - H0);
            const mc_u32x4 ru = mc_draw(cfg.seed, (uint32_t)(cfg.chain_offset + cc[c]),
                                        (uint32_t)it, MC_RNG_TAG_ACCEPT, 0, 0);
            const float logu = mc_logf_u01(mc_u01_f32(ru.x));
            const bool accepted = logu < ratio;
            acc[c] = accepted;
            nacc[c] += accepted ? 1 : 0;
            ntot[c] += 1;
            const double eps_used = eps[c];
            if (warm && cfg.adapt_step_size && it > 10) {
                const double rate = (double)nacc[c] / (double)ntot[c];
                eps[c] = (rate < cfg.target_accept) ? eps_used * 0.95 : eps_used * 1.05;
            }
            if (accepted) {
                lp[c] = lpn[c];
            } else {
#pragma unroll
                for (int r = 0; r < RS; ++r) {
                    R.q[r][c] = q0[r][c];
                    R.g[r][c] = g0[r][c];
                }
            }
            if (slice == 0 && j == 0 && live[c]) {
                const int64_t ti = it - tr.iter_begin;
                if (ti >= 0 && ti < tr.capacity) {
                    const int64_t o = cc[c] * tr.capacity + ti;
                    if (tr.accepted) tr.accepted[o] = accepted ? 1 : 0;
                    if (tr.accept_stat) tr.accept_stat[o] = ratio;
                    if (tr.step_size) tr.step_size[o] = eps_used;
                    if (tr.energy) tr.energy[o] = H0;
                    if (tr.tree_depth) tr.tree_depth[o] = L;
                    if (tr.n_leapfrog) tr.n_leapfrog[o] = L;
                }
            }
        }
        if (!(xc ? acc[1] : acc[0])) {
            sh.q = q0s;
            sh.g = g0s;
        }
        if (!warm && samples != nullptr) {
            const int64_t s = it - cfg.num_warmup - cfg.sample_begin;
            if (s >= 0 && s < cfg.sample_capacity) {
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    if (!live[c]) continue;
                    float* out = samples + (cc[c] * cfg.sample_capacity + s) * (int64_t)D;
#pragma unroll
                    for (int r = 0; r < RS; ++r)
                        if (gk[r] >= 0 && lead) out[gk[r]] = R.q[r][c];
                }
                if (slice == 0 && xlive)
                    samples[(xch_id * cfg.sample_capacity + s) * (int64_t)D + xg] = sh.q;
            }
        }
        MC_STAMP(6);
    }

    // ---- launch epilogue: state back to HBM ---------------------------------------
    MC_STAMP_FLUSH
    if (!ok) return;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        if (!live[c]) continue;
#pragma unroll
        for (int r = 0; r < RS; ++r) {
            if (gk[r] >= 0 && lead) {
                st_q[cc[c] * D + gk[r]] = R.q[r][c];
                st_g[cc[c] * D + gk[r]] = R.g[r][c];
            }
        }
        if (slice == 0 && j == 0) {
            mc_chain_scalars& sc = scal[cc[c]];
            sc.logp = lp[c];
            sc.step_size = eps[c];
            sc.n_accept = nacc[c];
            sc.n_total = ntot[c];
            sc.warmup_accept = wacc[c];
            sc.warmup_total = wtot[c];
            sc.n_grad += cfg.iter_count * (int64_t)L;
        }
    }
    if (slice == 0 && xlive) {
        st_q[xch_id * D + xg] = sh.q;
        st_g[xch_id * D + xg] = sh.g;
    }
}

}  // namespace mc
