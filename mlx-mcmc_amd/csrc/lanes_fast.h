// lanes_fast.h — the lane-resident HMC kernel for "fast-form" programs
// (k_hmc_lf): the layout, exchange protocol and arithmetic of k_hmc_lr
// (lanes.h; reference hmc.py:7-206 per chain) with everything a fast-form
// program does not need compiled out.
//
// Fast form (host planner, api.hip plan_lanes: LanePlan::fast): every slice
// holds at most one swept term — y ~ N(theta[g], scale), value data, loc the
// lane's private parameter, scale shared or constant: moment sums over the
// private parameter's elements — and at most one direct term — theta ~
// N(loc, scale), one element per parameter — and every scalar term is the
// "own" prior of one shared parameter.  The hierarchical models of BASELINE
// configs[2]/[3] and the isotropic / diagonal Gaussians of configs[1]/[4] are
// of this form.
//
// FORM (template): -1 reads the form from the terms at run time; FORM >= 0
// fixes it at compile time (bits LF_*; the planner sets LanePlan::form when
// every slice has the same terms and the shared roles are distinct
// parameters).  A compile-time form keys the record's cotangent items by
// *role* (swept scale, direct loc, direct scale) instead of by shared
// ordinal: no selects between them, and the lane that holds a role's total
// after the exchange holds that role's parameter.
//
// What differs from k_hmc_lr:
//   * the terms' fields, the lanes holding their shared operands and the
//     runs' data pointers are read once per launch;
//   * both chains' per-step arithmetic runs packed (v_pk_*_f32: the same
//     IEEE operations per chain, two chains per instruction), the per-launch
//     uniform values pinned in VGPRs (no SGPR spills reloaded per step);
//   * the moment sweep keeps even and odd elements in separate packed
//     accumulators (two dependency chains each; a dependent v_pk_add_f32
//     advances every 10 cycles, scripts/micro/pk_probe.hip);
//   * the wave totals of the record are reduce-scattered (permlane32 /
//     permlane16 swaps + one 16-lane DPP row sum) so that pair P's total is
//     in row perm[P % 4] of register P / 4 — no readlanes, no publish select;
//     the poll uses the same pair -> row map, so after the slice sums the
//     lane that holds shared slot (k, c) finds its cotangent total in its own
//     register (lane 16 perm[P % 4] + P / 4, P = 2 (k + 1) + c);
//   * the shared parameters' own priors enter slice 0's log-p record (one
//     add in the lane that holds the parameter, instead of a per-step
//     readlane sum over the shared parameters after the exchange);
//   * the kinetic-energy items K0 / K1 travel only on the first / last step;
//   * log p is evaluated, exchanged and summed on the last step only: a
//     leapfrog step needs the gradient alone, and the Hamiltonian of the
//     proposal (hmc.py:139-153) reads log p at the end of the trajectory, so
//     the intermediate steps' log-p items (their terms' log / normaliser
//     work, the records' lp pairs and their polls) were never used.
// Results equal k_hmc_lr's up to fp32 summation order; runs are
// bit-reproducible and independent of how chains are split over launches.
#pragma once
#include <type_traits>

#include "lanes.h"

namespace mc {

// compile-time term forms (FORM bits)
constexpr int LF_SW = 1;    // a swept term
constexpr int LF_SWS = 2;   //   its scale a shared parameter (else constant)
constexpr int LF_DIR = 4;   // a direct term
constexpr int LF_DM = 8;    //   its loc a shared parameter (else constant)
constexpr int LF_DS = 16;   //   its scale a shared parameter (else constant)
// the shared slots of a compile-time form: swept scale, direct loc, direct
// scale, in that order, for the roles present
constexpr int lf_slot_sws(int F) { return (void)F, 0; }
constexpr int lf_slot_dm(int F) { return (F & LF_SWS) ? 1 : 0; }
constexpr int lf_slot_ds(int F) { return lf_slot_dm(F) + ((F & LF_DM) ? 1 : 0); }
constexpr int lf_nroles(int F) { return lf_slot_ds(F) + ((F & LF_DS) ? 1 : 0); }

// pair P -> the row (16-lane group) that holds its total after the
// reduce-scatter / the slice sums: rows hold values 4n + {0, 2, 1, 3}
MC_DEV constexpr int lf_row(int P) { return (P & 3) == 1 ? 2 : ((P & 3) == 2 ? 1 : (P & 3)); }
// the lane that holds shared slot k of chain c
MC_DEV constexpr int lf_shlane(int k, int c) {
    return 16 * lf_row(2 * (k + 1) + c) + (2 * (k + 1) + c) / 4;
}
// Uniform (per chain) value `v` of shared slot k, chain c.
MC_DEV float lf_sh(float v, int k, int c) { return rl(v, lf_shlane(k, c)); }
// Both chains' values of shared slot k.
MC_DEV f2 lf_sh2(float v, int k) { return (f2){rl(v, lf_shlane(k, 0)), rl(v, lf_shlane(k, 1))}; }

// Keep a wave-uniform value in a VGPR: the kernel holds more uniform values
// than there are SGPRs, and a spilled SGPR costs a v_readlane at every use.
MC_DEV float vpin(float x) {
    asm volatile("" : "+v"(x));
    return x;
}
MC_DEV f2 vpin(f2 x) {
    asm volatile("" : "+v"(x));
    return x;
}
MC_DEV f2 bc2(float x) { return (f2){x, x}; }

// Reduce-scatter of 8 per-lane values over the wave: returns two registers;
// row r of register n holds (in all 16 lanes) the wave total of value
// 4n + {0, 2, 1, 3}[r].  A fixed tree: the same bits in every wave / slice.
// Z01: v[0] and v[1] are zero in every lane (their totals are +0).
template <bool Z01 = false>
MC_DEV void lf_rs8(const float (&v)[8], float (&x)[2]) {
    float w[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {  // lanes 0-31: v[2m] sums, lanes 32-63: v[2m+1]
        if (Z01 && m == 0) {
            w[0] = 0.0f;
            continue;
        }
        const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[2 * m]),
                                                        __float_as_uint(v[2 * m + 1]), false, false);
        w[m] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
#pragma unroll
    for (int n = 0; n < 2; ++n) {  // per 32-lane half: lanes 0-15 w[2n], 16-31 w[2n+1]
        const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(w[2 * n]),
                                                        __float_as_uint(w[2 * n + 1]), false, false);
        float t = __uint_as_float(r[0]) + __uint_as_float(r[1]);
        t += dpp_row<0xB1>(t);
        t += dpp_row<0x4E>(t);
        t += dpp_row<0x141>(t);
        t += dpp_row<0x140>(t);
        x[n] = t;
    }
}

// (xy.y, xy.y) - th in one v_pk_add_f32: the backend copies the odd register
// of a pair to an even one before broadcasting it (one v_mov per element
// pair); op_sel on the pair reads it in place.
MC_DEV f2 lf_hi_minus(f2 xy, f2 th) {
    f2 d;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1] neg_lo:[0,1] neg_hi:[0,1]"
        : "=v"(d)
        : "v"(xy), "v"(th));
    return d;
}

// Moment sums of one lane's run (value = data x, loc = the lane's private
// parameter th) for both chains, packed FP32: d = x - th, s1 += d,
// s2 = fma(d, d, s2), with the even and odd elements in separate packed
// accumulators (two independent dependency chains each).
MC_DEV void lf_moments(const float* xv, int len, int lmin4, int lmax, f2 th, f2& s1, f2& s2) {
    f2 a1[2], a2[2];
    // a register pair's elements broadcast by swizzle (op_sel on the pair,
    // no copy of the odd register); the first pair assigns the accumulators
    // (d and d * d: what 0 + d and fma(d, d, 0) round to), so no zeros are
    // materialised per sweep
    auto pair = [&](f2 xy, auto first) {
        const f2 d0 = xy.xx - th;
        const f2 d1 = lf_hi_minus(xy, th);
        if constexpr (decltype(first)::value) {
            a1[0] = d0;
            a2[0] = d0 * d0;
            a1[1] = d1;
            a2[1] = d1 * d1;
        } else {
            a1[0] += d0;
            a2[0] = pk_fma(d0, d0, a2[0]);
            a1[1] += d1;
            a2[1] = pk_fma(d1, d1, a2[1]);
        }
    };
    const std::false_type acc;
    int u4 = 0;
    // 16 elements per round; the next round's LDS loads are issued before
    // this round's arithmetic (software pipelined over two register sets that
    // alternate, so no copies: a lone wave per SIMD — fewer slices — does not
    // wait for the load latency)
    if (lmin4 >= 4) {
        float4 A[4], B[4];
        auto load = [&](float4 (&X)[4], int g) {
#pragma unroll
            for (int q = 0; q < 4; ++q) X[q] = *(const float4*)(xv + (g + q) * 256);
        };
        auto round = [&](const float4 (&X)[4], auto first) {
            pair((f2){X[0].x, X[0].y}, first);
            pair((f2){X[0].z, X[0].w}, acc);
#pragma unroll
            for (int q = 1; q < 4; ++q) {
                pair((f2){X[q].x, X[q].y}, acc);
                pair((f2){X[q].z, X[q].w}, acc);
            }
        };
        // (the prefetch index is clamped to the last full round: the loads
        // are unconditional, so the register sets never need copies)
        const int last = lmin4 - 4;
        load(A, 0);
        const bool more = 8 <= lmin4;
        load(B, min(4, last));
        round(A, std::true_type());
        u4 = 4;
        if (more) {
            for (;;) {
                const bool more_a = u4 + 8 <= lmin4;
                load(A, min(u4 + 4, last));
                round(B, acc);
                u4 += 4;
                if (!more_a) break;
                const bool more_b = u4 + 8 <= lmin4;
                load(B, min(u4 + 4, last));
                round(A, acc);
                u4 += 4;
                if (!more_b) break;
            }
        }
    } else {
        a1[0] = a1[1] = a2[0] = a2[1] = (f2){0.f, 0.f};
    }
    // the groups every lane holds in full (uniform), then the ragged end:
    // element e of the lanes with more elements (e < lmax, uniform bounds),
    // masked per lane (the tile is padded to whole groups, so every load is
    // in bounds); no exec-masked loop, no per-lane branch
    for (; u4 < lmin4; ++u4) {
        const float4 a = *(const float4*)(xv + u4 * 256);
        pair((f2){a.x, a.y}, acc);
        pair((f2){a.z, a.w}, acc);
    }
    const f2 z = {0.f, 0.f};
    for (int e = 4 * lmin4; e < lmax; e += 4) {
        const float4 a = *(const float4*)(xv + (e >> 2) * 256);
        const float x[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (e + k >= lmax) break;  // (uniform)
            f2 d = (f2){x[k], x[k]} - th;
            d = (e + k < len) ? d : z;
            a1[k & 1] += d;
            a2[k & 1] = pk_fma(d, d, a2[k & 1]);
        }
    }
    s1 = a1[0] + a1[1];
    s2 = a2[0] + a2[1];
}

// The fast-form terms of a slice, read once per launch: at most one swept
// term (y ~ N(theta[g], scale): value data, loc private, scale shared or
// constant) and one direct term (theta ~ N(loc, scale), loc / scale shared or
// constant).  Shared operands are named by their shared ordinals.
struct LfTerms {
    bool sw, dir;
    // swept term
    float sw_w, sw_c0, sw_cinv, sw_cinv2, sw_clogs;
    bool sw_shs;
    int sw_ks;           // shared ordinal of the scale (or -1)
    // direct term
    float d_w, d_c0, d_m, d_cinv, d_cinv2, d_clogs;
    bool d_shm, d_shs;
    int d_km, d_ks;      // shared ordinals of loc / scale (or -1)
};

MC_DEV LfTerms lf_terms(const MC_CONST LrTerm* tt, int nsweep, int ndirect) {
    LfTerms F;
    F.sw = nsweep > 0;
    F.dir = ndirect > 0;
    const MC_CONST LrTerm* T = tt;
    F.sw_w = F.sw ? T->weight : 0.f;
    F.sw_c0 = F.sw ? T->c0 : 0.f;
    F.sw_cinv = F.sw ? T->cinv : 0.f;
    F.sw_cinv2 = F.sw ? T->cinv2 : 0.f;
    F.sw_clogs = F.sw ? T->clogs : 0.f;
    F.sw_shs = F.sw && T->kind[2] == SK_SHARED;
    F.sw_ks = F.sw_shs ? T->jsh[2] : -1;
    const MC_CONST LrTerm* U = tt + nsweep;
    F.d_w = F.dir ? U->weight : 0.f;
    F.d_c0 = F.dir ? U->c0 : 0.f;
    F.d_m = F.dir ? U->cval[1] : 0.f;
    F.d_cinv = F.dir ? U->cinv : 0.f;
    F.d_cinv2 = F.dir ? U->cinv2 : 0.f;
    F.d_clogs = F.dir ? U->clogs : 0.f;
    F.d_shm = F.dir && U->kind[1] == SK_SHARED;
    F.d_shs = F.dir && U->kind[2] == SK_SHARED;
    F.d_km = F.d_shm ? U->jsh[1] : -1;
    F.d_ks = F.d_shs ? U->jsh[2] : -1;
    return F;
}

// NSH: shared slots of the record (FORM >= 0: lf_nroles(FORM)).
// XL: the host found every exchange group's workgroups on one XCD
// (host.h xcd_round_robin): records are published with L2-resident stores
// (sliced.h granule_store_xcd), after an in-kernel check of the placement.
template <int RS, int NSH, int NW, bool X1, int FORM, bool XL = false>
__global__ void __launch_bounds__(64 * NW)
k_hmc_lf(LrCtx P, RunArgs A, int64_t chain_base, int64_t n_groups, mc_chain_scalars* scal,
         float* st_q, float* st_g, float* samples, TraceDev tr, unsigned long long* xch,
         int* status, uint32_t ebase) {
    static_assert(NSH <= kLrMaxShared, "shared parameters");
    constexpr bool CF = FORM >= 0;      // the form is fixed at compile time
    static_assert(!CF || lf_nroles(FORM) == NSH, "record slots of a compile-time form");
    constexpr int NB = 2 * NW;          // chains per block: wave w owns chains 2w, 2w + 1
    constexpr int NV = 2 * (NSH + 1);   // per-step pairs: lp and the shared cotangents
    constexpr int NPAIR = NV + 4;       // + K0 (first step) and K1 (last step)
    constexpr int NPASS = (NPAIR + 3) / 4, NPASS_V = (NV + 3) / 4;
    constexpr int NRS = (NV + 7) / 8;   // reduce-scatter calls per step
    if (!X1 && A.fault && blockIdx.x == gridDim.x - 1) return;  // test hook: never publishes
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const mc_run_config& cfg = A.cfg;
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
    int64_t cc[2];
    bool live[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        live[c] = cbase + b0 + c < C;
        cc[c] = min(cbase + b0 + c, C - 1);
    }

    float* sd = smem;
    const int64_t* blk = P.blocks + 4 * (int64_t)slice;
    const int64_t doff = blk[0];
    const int dlen = (int)blk[1];
    const int nsweep = (int)(blk[3] & 255);
    const int ndirect = (int)((blk[3] >> 8) & 255);
    for (int i = tid; 4 * i < dlen; i += 64 * NW)
        *(float4*)(sd + 4 * i) = *(const float4*)(P.data + doff + 4 * i);
    LrSterm* sst = (LrSterm*)(smem + P.sdata_floats);
    for (int i = tid; i < P.n_sterms * (int)(sizeof(LrSterm) / 16); i += 64 * NW)
        ((float4*)sst)[i] = ((const float4*)P.sterms)[i];

    const MC_CONST LrTerm* tt = cptr(P.terms) + (int64_t)slice * P.n_terms;
    const LfTerms F = lf_terms(tt, nsweep, ndirect);
    // the form, folded to constants when FORM >= 0
    const bool SW = CF ? (FORM & LF_SW) != 0 : F.sw;
    const bool SWS = CF ? (FORM & LF_SWS) != 0 : F.sw_shs;
    const bool DIR = CF ? (FORM & LF_DIR) != 0 : F.dir;
    const bool DM = CF ? (FORM & LF_DM) != 0 : F.d_shm;
    const bool DS = CF ? (FORM & LF_DS) != 0 : F.d_shs;
    // the shared slot of each role: its role index (compile-time form) or its
    // shared ordinal (run-time form)
    const int ksw = CF ? lf_slot_sws(FORM) : max(F.sw_ks, 0);
    const int kdm = CF ? lf_slot_dm(FORM) : max(F.d_km, 0);
    const int kds = CF ? lf_slot_ds(FORM) : max(F.d_ks, 0);
    const int nsl = CF ? NSH : Dsh;  // shared slots
    // shared ordinal of slot k
    auto ord_of = [&](int k) {
        int o = F.d_ks;  // selects, not an indexed read of F (scratch)
        o = (DM && k == kdm) ? F.d_km : o;
        o = (SWS && k == ksw) ? F.sw_ks : o;
        return CF ? o : k;
    };
    // this lane's shared slot: (xk, xc) with lf_shlane(xk, xc) == j
    int xk = -1, xc = 0;
#pragma unroll
    for (int k = 0; k < kLrMaxShared; ++k)
#pragma unroll
        for (int c = 0; c < 2; ++c)
            if (k < nsl && lf_shlane(k, c) == j) {
                xk = k;
                xc = c;
            }
    const bool xon = xk >= 0;
    const int xo = xon ? ord_of(xk) : 0;  // its shared ordinal
    int xg = P.shl[0];
#pragma unroll
    for (int k = 1; k < kLrMaxShared; ++k) xg = (xo == k) ? P.shl[k] : xg;
    const int64_t xch_id = xc ? cc[1] : cc[0];
    const bool xlive = xon && (xc ? live[1] : live[0]);
    const int rep = P.rep;                   // lanes per private parameter (lanes.h)
    const bool lead = (j & (rep - 1)) == 0;  // this lane counts its parameters
    // a transformed shared parameter (lanes.h LrCtx::shxf) and the identity
    // terms over its raw value: a uniform branch, so programs without them
    // run the same instructions as before
    const bool hxf = P.has_xf != 0;
    int xxf = P.shxf[0];
    float xid = P.shid[0];
#pragma unroll
    for (int k = 1; k < kLrMaxShared; ++k) {
        xxf = (xo == k) ? P.shxf[k] : xxf;
        xid = (xo == k) ? P.shid[k] : xid;
    }
    xxf = xon ? xxf : MC_XF_NONE;
    xid = xon ? xid : 0.0f;

    LrPriv<RS> R0;  // (loaded as in k_hmc_lr, then packed per slot)
    int gk[RS];
    f2 q[RS], p[RS], g[RS];
#pragma unroll
    for (int r = 0; r < RS; ++r) {
        gk[r] = P.gidx[((int64_t)slice * kLrMaxSlots + r) * 64 + j];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            R0.q[r][c] = gk[r] >= 0 ? st_q[cc[c] * D + gk[r]] : 0.0f;
            R0.g[r][c] = gk[r] >= 0 ? st_g[cc[c] * D + gk[r]] : 0.0f;
        }
        q[r] = (f2){R0.q[r][0], R0.q[r][1]};
        g[r] = (f2){R0.g[r][0], R0.g[r][1]};
        p[r] = (f2){0.f, 0.f};
    }
    // the lane RNG plan (api.hip plan_lane_rng), when the planner made one
    const bool rngp = P.rng != nullptr;
    int4 rw = {0, 0, 0, 0};
    if (rngp) rw = P.rng[(int64_t)slice * 64 + j];
    const int racc0 = __builtin_amdgcn_readfirstlane((rw.w >> 8) & 63);
    const int racc1 = __builtin_amdgcn_readfirstlane((rw.w >> 14) & 63);
    // the lane holding this lane's shared parameter's Philox block (chain xc)
    int sh_src = 0;
    if (rngp) {
        const int target = (xc + 1) | ((xg >> 2) << 3);
        for (int i = 0; i < 64; ++i)
            sh_src = (__builtin_amdgcn_readlane(rw.x, i) == target) ? i : sh_src;
    }
    LrShared sh;
    sh.q = xon ? st_q[xch_id * D + xg] : 1.0f;
    sh.g = xon ? st_g[xch_id * D + xg] : 0.0f;
    sh.p = 0.0f;
    sh.v = hxf ? xf_apply(xxf, sh.q) : sh.q;
    sh.is = sh.iv = 1.0f;
    sh.lg = 0.0f;
    double eps[2];
    f2 lp;
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

    // the lane's own prior (lr_own_prior keys it by ordinal); it enters
    // slice 0's log-p record through this lane
    const LrOwn own = lr_own_prior(P.n_sterms, sst, xon ? 2 * xo + xc : 64, Dsh);
    const bool own_lp0 = own.on && slice == 0 && xc == 0;
    const bool own_lp1 = own.on && slice == 0 && xc == 1;
    const float o_m = vpin(own.m), o_cinv2 = vpin(own.cinv2), o_c0l = vpin(own.c0l),
                o_wn = vpin(own.wn);
    // per slot: the swept term's run (data pointer, length, full float4
    // groups of every lane) and the direct term's presence
    const float* xv[RS];
    int len[RS], lmin4[RS], lmax[RS];
    f2 cnt[RS];
    bool pdir[RS];
#pragma unroll
    for (int r = 0; r < RS; ++r) {
        len[r] = 0;
        lmin4[r] = 0;
        lmax[r] = 0;
        xv[r] = sd;
        if (SW && r < tt[0].nslot) {
            len[r] = ((const int32_t*)sd)[tt[0].len_off + r * 64 + j];
            lmin4[r] = tt[0].lmin4[r];
            xv[r] = sd + tt[0].doff[0] + tt[0].toff[r] + 4 * j;
        }
        cnt[r] = bc2((float)len[r]);
        // the slot's longest run (uniform: a wave max, once per launch)
        {
            int m = len[r];
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) m = max(m, __shfl_xor(m, o));
            lmax[r] = __builtin_amdgcn_readfirstlane(m);
        }
        pdir[r] = DIR && r < tt[nsweep].nslot &&
                  ((const int32_t*)sd)[tt[nsweep].len_off + r * 64 + j] > 0;
    }
    // the terms' constants, pinned in VGPRs
    const f2 sw_w = vpin(bc2(F.sw_w)), sw_c0 = vpin(bc2(F.sw_c0));
    const f2 sw_cinv = vpin(bc2(F.sw_cinv)), sw_cinv2 = vpin(bc2(F.sw_cinv2)),
             sw_clogs = vpin(bc2(F.sw_clogs));
    const f2 d_w = vpin(bc2(F.d_w)), d_c0 = vpin(bc2(F.d_c0)), d_m = vpin(bc2(F.d_m));
    // (one slot: the direct term's weight per lane, zero where the lane's
    // parameter has no direct term)
    const f2 d_w1 = vpin(bc2(pdir[0] ? F.d_w : 0.0f));
    const f2 d_cinv = vpin(bc2(F.d_cinv)), d_cinv2 = vpin(bc2(F.d_cinv2)),
             d_clogs = vpin(bc2(F.d_clogs));
    const f2 half = bc2(0.5f), one = bc2(1.0f);
    const float lp_const = vpin(P.lp_const);
    // the swept terms' moment sums at the current point, both chains
    auto sweep = [&](f2 (&s1)[RS], f2 (&s2)[RS]) {
#pragma unroll
        for (int r = 0; r < RS; ++r) {
            s1[r] = (f2){0.f, 0.f};
            s2[r] = (f2){0.f, 0.f};
            if (len[r] > 0) lf_moments(xv[r], len[r], lmin4[r], lmax[r], q[r], s1[r], s2[r]);
        }
    };

    const int L = cfg.num_leapfrog_steps;
    uint32_t epoch = ebase;  // tags continue across launches (api.hip ws_reserve)
    bool ok = true;
    // one 128-byte line per (wave, slice) record; lanes publish the pairs
    // they hold after the reduce-scatter, pass ps of the poll reads pair
    // 4 ps + perm[lane / 16] of slice lane % 16
    unsigned long long* gline[2];
#pragma unroll
    for (int par = 0; par < 2; ++par)
        gline[par] = xch + (((int64_t)par * n_groups + grp) * (NB / 2) + wave) * S * 16;
    const int row = j >> 4, col = j & 15;
    const bool poll_lane = col < S;
    // the poll address of pass 0 (pass ps: + 4 ps), per epoch parity
    unsigned long long* gp[2];
#pragma unroll
    for (int par = 0; par < 2; ++par) gp[par] = gline[par] + min(col, S - 1) * 16 + lf_row(row);
    // publishing: lanes 16 r + n (n < NRS * 2) hold pair 8 (n / 2) + 4 (n % 2) + perm[r]
    const int pub_pair = (col < 2 * NRS) ? 8 * (col >> 1) + 4 * (col & 1) + lf_row(row) : -1;
    const bool pub_rec = pub_pair >= 0 && pub_pair < NV;
    // an intermediate step's store: the pairs past the log-p pair, at their
    // granule of either parity's line
    const bool pub_mid = pub_rec && pub_pair >= 2;
    const int pub_x = 2 * (col >> 1) + (col & 1);
    const int pub_off = slice * 16 + max(pub_pair, 0);
    // poll passes by kind: record pairs every step, K0 / K1 pairs on the first / last
    uint32_t need_v = 0, need_lp = 0, need_k0 = 0, need_k1 = 0;
#pragma unroll
    for (int ps = 0; ps < NPASS; ++ps) {
        const int pr = 4 * ps + lf_row(row);
        if (X1 || !poll_lane || pr >= NPAIR) continue;
        if (pr < 2) need_lp |= 1u << ps;  // the log-p pairs: last step only
        else if (pr < NV) need_v |= 1u << ps;
        else if (pr < NV + 2) need_k0 |= 1u << ps;
        else need_k1 |= 1u << ps;
    }
    // XL: check that the block's slices share an XCD (sliced.h xcd_announce /
    // xcd_agree) before the first publish.  The check's granules: granule 15
    // of each slice's parity-0 line of wave 0 (record pairs use 0 .. NPAIR - 1
    // < 15); its tag ebase + 1 is never 0, the value of a freshly cleared
    // line (the steps' tags start there too, on the record granules).  Its
    // loads are issued here and completed after the first sweep.
    constexpr bool xchk = XL && !X1;
    unsigned long long* const xslots = xch + ((int64_t)grp * (NB / 2)) * S * 16 + 15;
    XcdPoll xpoll = {0ull};
    if (xchk && cfg.iter_count > 0)
        xpoll = xcd_announce(xslots, S, slice, ebase + 1, wave == 0 && j == 0);
    static_assert(NPAIR <= 15, "granule 15 of a record line is the XCD handshake's");
    const int64_t it_end = cfg.iter_begin + cfg.iter_count;
    for (int64_t it = cfg.iter_begin; it < it_end && ok; ++it) {
        MC_STAMP_DECL
        const bool warm = it < cfg.num_warmup;
        float hs[2], es[2];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            if (it == cfg.num_warmup) {  // hmc.py:175-180
                wacc[c] = nacc[c];
                wtot[c] = ntot[c];
                nacc[c] = 0;
                ntot[c] = 0;
            }
            hs[c] = (float)(0.5 * eps[c]);
            es[c] = (float)eps[c];
        }
        const f2 h = vpin((f2){hs[0], hs[1]}), e = vpin((f2){es[0], es[1]});
        const float xh = vpin(xc ? hs[1] : hs[0]), xe = vpin(xc ? es[1] : es[0]);
        // momentum: parameter g takes normal g % 4 of Philox block g / 4
        auto normal_of = [&](int gi, int64_t chain) {
            const mc_u32x4 rr = mc_draw(cfg.seed, (uint32_t)(cfg.chain_offset + chain),
                                        (uint32_t)it, MC_RNG_TAG_MOMENTUM, 0, (uint32_t)(gi >> 2));
            float z0, z1;
            if ((gi & 3) < 2) mc_box_muller(rr.x, rr.y, &z0, &z1);
            else mc_box_muller(rr.z, rr.w, &z0, &z1);
            return (gi & 1) ? z1 : z0;
        };
        f2 k0p = {0.f, 0.f};
        float logu_acc[2] = {0.f, 0.f};  // the chains' accept logs (lane RNG plan)
        if (rngp) {
            // the lane RNG plan (api.hip plan_lane_rng): this lane's Philox
            // block — a momentum block of one chain or a chain's accept draw —
            // and both Box-Muller pairs of it; the accept lanes' first log is
            // the accept log (mc_logf_unit of the same uniform transform the
            // per-lane path uses); the normals are fetched from their lanes
            const int kind = rw.x & 7;
            const bool acl = kind >= 3;
            const int csel = (kind == 2 || kind == 4) ? 1 : 0;
            const mc_u32x4 rr =
                mc_draw(cfg.seed, (uint32_t)(cfg.chain_offset + (csel ? cc[1] : cc[0])),
                        (uint32_t)it, acl ? MC_RNG_TAG_ACCEPT : MC_RNG_TAG_MOMENTUM, 0,
                        acl ? 0u : ((uint32_t)rw.x >> 3));
            const float la = mc_logf_unit(acl ? mc_u01_f32(rr.x) : mc_u01_boxf(rr.x));
            const float lb = mc_logf_unit(mc_u01_boxf(rr.z));
            float z[4];
            mc_box_muller_log(la, rr.y, &z[0], &z[1]);
            mc_box_muller_log(lb, rr.w, &z[2], &z[3]);
            logu_acc[0] = rl(la, racc0);
            logu_acc[1] = rl(la, racc1);
            auto fetch = [&](int src, int comp) {
                float v = __shfl(z[0], src);
                const float v1 = __shfl(z[1], src), v2 = __shfl(z[2], src), v3 = __shfl(z[3], src);
                v = comp == 1 ? v1 : v;
                v = comp == 2 ? v2 : v;
                return comp == 3 ? v3 : v;
            };
#pragma unroll
            for (int r = 0; r < RS; ++r) {
                const int word = (r < 2 ? rw.y : rw.z) >> (14 * (r & 1));
                const int comp = (word >> 12) & 3;
                const f2 zz = {fetch(word & 63, comp), fetch((word >> 6) & 63, comp)};
                if (gk[r] < 0) continue;  // (an empty slot's p stays 0: its g is always 0)
                p[r] = zz;
                if (lead) k0p += zz * zz;
            }
            const float zs = fetch(sh_src, xg & 3);
            sh.p = xon ? zs : 0.0f;
        } else {
#pragma unroll
            for (int r = 0; r < RS; ++r) {
                if (gk[r] < 0) continue;  // (an empty slot's p stays 0: its g is always 0)
                const f2 z = {normal_of(gk[r], cc[0]), normal_of(gk[r], cc[1])};
                p[r] = z;
                if (lead) k0p += z * z;
            }
            sh.p = xon ? normal_of(xg, xch_id) : 0.0f;
        }
        const float K0w[2] = {wave_sum(k0p[0]), wave_sum(k0p[1])};
        float k0s[2] = {0.f, 0.f};  // the shared parameters' part, in slot order
        {
            const float p2 = sh.p * sh.p;
            for (int k = 0; k < nsl; ++k) {
                k0s[0] += lf_sh(p2, k, 0);
                k0s[1] += lf_sh(p2, k, 1);
            }
        }
        f2 q0[RS], g0[RS];
#pragma unroll
        for (int r = 0; r < RS; ++r) {
            q0[r] = q[r];
            g0[r] = g[r];
        }
        const float q0s = sh.q, g0s = sh.g;
        f2 lpn = lp;
        float K0[2] = {0.f, 0.f}, K1[2] = {0.f, 0.f};
        MC_STAMP(5);
        // (the two half kicks of consecutive steps stay separate roundings, as
        // the reference's; their common product h * g is formed once)
        auto drift_private = [&](bool second_half) {
#pragma unroll
            for (int r = 0; r < RS; ++r) {
                const f2 hg = h * g[r];
                f2 pj = p[r];
                if (second_half) pj = pj + hg;  // end of the previous step
                pj = pj + hg;
                p[r] = pj;
                q[r] = q[r] + e * pj;
            }
        };
        auto drift_shared = [&](bool second_half) {
            const float hg = xh * sh.g;
            float pj = sh.p;
            if (second_half) pj = pj + hg;
            pj = pj + hg;
            sh.p = pj;
            sh.q = sh.q + xe * pj;
            sh.v = sh.q;
            if (hxf) sh.v = xf_apply(xxf, sh.q);  // (mx.exp(log_sigma) ...: the terms' value)
            // the shared scale's reciprocals (moment form): hardware v_rcp_f32
            // (<= 1 ulp) instead of the IEEE division — one dependent chain of
            // ~40 VALU on every step's critical path becomes 2; the same bits in
            // every slice, so the replicas stay identical.  Its log (v_log_f32)
            // is taken on the last step only, where log p is formed.
            sh.is = __builtin_amdgcn_rcpf(sh.v);
            sh.iv = sh.is * sh.is;
        };
        f2 M1[RS], M2[RS];
        drift_private(false);
        drift_shared(false);
        sweep(M1, M2);
        if (xchk && it == cfg.iter_begin) {  // (before the launch's first publish)
            const bool same = xcd_agree(xpoll, xslots, S, ebase + 1, ok);
            // (diagnostic: blocks found on one XCD / not, counted by slice 0,
            // in the status area's words 8 / 9; mc_debug_workspace_xcd)
            if (ok && slice == 0 && wave == 0 && j == 0)  // (one per block)
                __hip_atomic_fetch_add(status + (same ? 8 : 9), 1, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            if (!ok || !same) {
                // a timeout (1), or a placement the L2-resident stores would
                // not reach (2): nothing published, the block's chains keep
                // their state, the launch reports it (mc_workspace_status)
                __hip_atomic_store(status, ok ? 2 : 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = false;
                break;
            }
        }
        // one leapfrog step at the point q(l + 1), compiled per kind so that the
        // intermediate steps carry none of the first / last steps' work (K0 /
        // K1 items, log p) nor its uniform branches and their live masks:
        // 0 first (l = 0 < L - 1), 1 intermediate, 2 last (l = L - 1 > 0),
        // 3 the only step (L = 1).  Returns false on an exchange timeout.
        // PAR: the record lines' parity when the caller knows it (an
        // intermediate step, compiled once per parity: the publish and poll
        // addresses are then fixed registers, no per-step selects), else -1
        auto step = [&](int l, auto kind, auto parc) -> bool {
            constexpr int KIND = decltype(kind)::value;
            constexpr int PAR = decltype(parc)::value;
            constexpr bool FIRST = KIND == 0 || KIND == 3, LAST = KIND == 2 || KIND == 3;
            (void)l;
            // no vector-memory operation is in flight here (the last poll was
            // waited for): saying so explicitly keeps the compiler's wait-count
            // state clean at the step's entry, where the kinds' paths merge —
            // else it guards the sweep's first register writes with a
            // vmcnt(0) that also waits for this step's own publish store
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) expcnt(7) lgkmcnt(15)
            if constexpr (LAST)  // the shared scales' logs, for log p (log2 v * ln 2)
                sh.lg = __builtin_amdgcn_logf(sh.v) * 0.693147180559945f;
            MC_STAMP(0);
            constexpr bool lst = LAST;  // log p: the last step only
            // finish the swept term from its moment sums, evaluate the direct
            // term (k_hmc_lr's lr_finish; same arithmetic, both chains packed):
            // log p partial (last step), complete private gradients, cotangent
            // partials of the swept scale (cs), the direct loc (cm) and scale (cd)
            // (the first contribution to each sum is assigned, not added to
            // zero: x + 0 is not folded under IEEE signed zeros)
            f2 lpp = {0.f, 0.f}, cs = {0.f, 0.f}, cm = {0.f, 0.f}, cd = {0.f, 0.f};
            bool lpp0 = true, cs0 = true, cm0 = true, cd0 = true;
            bool g0r[RS];
#pragma unroll
            for (int r = 0; r < RS; ++r) {
                g[r] = (f2){0.f, 0.f};
                g0r[r] = true;
            }
            auto acc = [](f2& s, bool& first, f2 v) {
                s = first ? v : s + v;
                first = false;
            };
            // (a shared scale's 1/s^2 is squared here from its 1/s: the
            // holding lane's sh.iv = sh.is * sh.is, the same rounding)
            if (SW) {
                const f2 is = SWS ? lf_sh2(sh.is, ksw) : sw_cinv;
                const f2 iv = SWS ? is * is : sw_cinv2;
#pragma unroll
                for (int r = 0; r < RS; ++r) {
                    const bool on = len[r] != 0;
                    const f2 z = {0.f, 0.f};
                    if (RS == 1) {
                        // one slot: an empty lane's moment sums and count are
                        // zeros (the sweep skips it), so are its gradient and
                        // cotangent; its log p is selected away
                        g[r] = sw_w * (M1[r] * iv);
                        cs = sw_w * ((M2[r] * iv - cnt[r]) * is);
                        cs0 = g0r[r] = false;
                    } else if (on) {
                        acc(g[r], g0r[r], sw_w * (M1[r] * iv));
                        acc(cs, cs0, sw_w * ((M2[r] * iv - cnt[r]) * is));
                    }
                    if (lst) {
                        const f2 lg = SWS ? lf_sh2(sh.lg, ksw) : sw_clogs;
                        const f2 lpt = cnt[r] * (sw_c0 - lg) - (half * M2[r]) * iv;
                        if (RS == 1) {
                            lpp = on ? sw_w * lpt : z;
                            lpp0 = false;
                        } else if (on) {
                            acc(lpp, lpp0, sw_w * lpt);
                        }
                    }
                }
            }
            if (DIR) {
                const f2 um = DM ? lf_sh2(sh.v, kdm) : d_m;
                const f2 is = DS ? lf_sh2(sh.is, kds) : d_cinv;
                const f2 iv = DS ? is * is : d_cinv2;
#pragma unroll
                for (int r = 0; r < RS; ++r) {
                    // one slot: a lane without the term weighs it by zero (its
                    // cotangent items 0 * finite, its gradient g - 0) instead
                    // of branching around it under an exec mask
                    if (RS > 1 && !pdir[r]) continue;
                    const f2 dw = RS == 1 ? d_w1 : d_w;
                    const f2 d = q[r] - um;
                    const f2 s2 = d * d;
                    const f2 u = dw * (d * iv);
                    acc(g[r], g0r[r], -u);
                    acc(cm, cm0, u);
                    acc(cd, cd0, dw * ((s2 * iv - one) * is));
                    if (lst) {
                        const f2 lg = DS ? lf_sh2(sh.lg, kds) : d_clogs;
                        const f2 lpt = one * (d_c0 - lg) - (half * s2) * iv;
                        acc(lpp, lpp0, dw * lpt);
                    }
                }
            }
            // a replicated parameter's gradient: the sum of its lanes' partials
            if (rep > 1) {
#pragma unroll
                for (int r = 0; r < RS; ++r) {
                    float a = g[r][0], b = g[r][1];
                    grp_sum2(a, b, rep);
                    g[r] = (f2){a, b};
                }
            }
            // the own prior of this lane's shared parameter (moment form with
            // the constant scale's reciprocals, as the sliced terms); its log p
            // enters slice 0's record
            float g_own = 0.0f;
            {
                const float v = sh.v;
                const float d = own.hn ? v : v - o_m;
                const bool out = own.hn && !(v >= 0.0f);
                g_own = (out || !own.on) ? 0.0f : o_wn * -(d * o_cinv2);
                if (lst) {
                    const float d2 = d * d;
                    const float lpe = out ? -__builtin_inff() : o_c0l - (0.5f * d2) * o_cinv2;
                    const float lp_own = o_wn * lpe;
                    if (own_lp0) lpp[0] += lp_own;
                    if (own_lp1) lpp[1] += lp_own;
                    // the identity terms over the raw parameter (log-Jacobians)
                    if (hxf && slice == 0 && xon) {
                        if (xc == 0) lpp[0] += xid * sh.q;
                        else lpp[1] += xid * sh.q;
                    }
                }
            }
            MC_STAMP(1);
            // wave totals, reduce-scattered: pair P = 2 slot + chain
            float xr[2 * NRS];
            {
                float v[8 * NRS];
#pragma unroll
                for (int x = 0; x < 8 * NRS; ++x) v[x] = 0.0f;
                v[0] = lpp[0];
                v[1] = lpp[1];
                if constexpr (CF) {
                    if (FORM & LF_SWS) {
                        v[2 + 2 * lf_slot_sws(FORM)] = cs[0];
                        v[3 + 2 * lf_slot_sws(FORM)] = cs[1];
                    }
                    if (FORM & LF_DM) {
                        v[2 + 2 * lf_slot_dm(FORM)] = cm[0];
                        v[3 + 2 * lf_slot_dm(FORM)] = cm[1];
                    }
                    if (FORM & LF_DS) {
                        v[2 + 2 * lf_slot_ds(FORM)] = cd[0];
                        v[3 + 2 * lf_slot_ds(FORM)] = cd[1];
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < NSH; ++k)
#pragma unroll
                        for (int c = 0; c < 2; ++c)
                            v[2 + 2 * k + c] = ((F.sw_ks == k ? cs[c] : 0.0f) +
                                                (F.d_km == k ? cm[c] : 0.0f)) +
                                               (F.d_ks == k ? cd[c] : 0.0f);
                }
#pragma unroll
                for (int qq = 0; qq < NRS; ++qq) {
                    float vv[8], xx[2];
#pragma unroll
                    for (int x = 0; x < 8; ++x) vv[x] = v[8 * qq + x];
                    if (qq == 0 && !lst) lf_rs8<true>(vv, xx);  // (no log-p pairs)
                    else lf_rs8(vv, xx);
                    xr[2 * qq] = xx[0];
                    xr[2 * qq + 1] = xx[1];
                }
            }
            // the kinetic partials of the last step (uniform)
            float k1w[2] = {0.f, 0.f};
            if constexpr (LAST) {
                f2 k1p = {0.f, 0.f};
#pragma unroll
                for (int r = 0; r < RS; ++r) {
                    const f2 pj = p[r] + h * g[r];
                    if (lead) k1p += pj * pj;
                }
                k1w[0] = wave_sum(k1p[0]);
                k1w[1] = wave_sum(k1p[1]);
            }
            ++epoch;
            const int par = PAR >= 0 ? PAR : (int)(epoch & 1);
            if constexpr (!X1 && !FIRST && !LAST) {
                // an intermediate step: the record pairs only (addresses and
                // the lane's pair fixed per launch)
                float pv = xr[0];
#pragma unroll
                for (int x = 1; x < 2 * NRS; ++x) pv = (x == pub_x) ? xr[x] : pv;
                if (pub_mid) granule_put(gline[par] + pub_off, epoch, pv, XL);
            } else if (!X1) {
                // one store instruction: the record pairs, and the K items on the
                // first / last step (lanes 2, 3 of rows 0 / 1)
                int pp = -1;
                float pv = 0.0f;
                if (pub_rec && (lst || pub_pair >= 2)) {  // (log-p pairs: last step)
                    pp = pub_pair;
                    pv = xr[0];
#pragma unroll
                    for (int x = 1; x < 2 * NRS; ++x)
                        if (x == 2 * (col >> 1) + (col & 1)) pv = xr[x];
                }
                if (col == 2 * NRS || col == 2 * NRS + 1) {
                    const int c = col - 2 * NRS;
                    if (FIRST && row == 0) {
                        pp = NV + c;
                        pv = c ? K0w[1] : K0w[0];
                    }
                    if (LAST && row == 1) {
                        pp = NV + 2 + c;
                        pv = c ? k1w[1] : k1w[0];
                    }
                }
                if (pp >= 0) granule_put(gline[par] + slice * 16 + pp, epoch, pv, XL);
            }
            MC_STAMP(2);
            // the sweep issues at a higher wave priority than the latency-bound
            // rest of the step (slice sums, shared drift, finish, reduce-scatter,
            // publish): the two waves of a SIMD settle out of phase, one
            // sweeping while the other's dependent chains fill its gaps (with
            // equal priorities the SQ's oldest-first choice kept them in step;
            // A/B on one box 92.0 -> 100.0 M steps/s, the same with priority 1, 2
            // or 3, and with the poll at either level, profiles/r3/ab/ab34)
            __builtin_amdgcn_s_setprio(1);
            // poll: pass ps reads pair 4 ps + perm[row] of slice col
            constexpr bool kstep = FIRST || LAST;
            const uint32_t need =
                need_v | (FIRST ? need_k0 : 0u) | (LAST ? (need_k1 | need_lp) : 0u);
            float vals[NPASS];
#pragma unroll
            for (int ps = 0; ps < NPASS; ++ps) vals[ps] = 0.0f;
            // every pass's granules loaded at once (one round trip; lanes that
            // need none read an in-bounds line and ignore it); ready when every
            // needed tag is this step's.  A granule of this step is never
            // rewritten before this wave publishes the next one (the line
            // parity alternates per step), so the values of the last load
            // are the record's.
            unsigned long long y[NPASS];
            auto poll_issue = [&]() {
#pragma unroll
                for (int ps = 0; ps < NPASS; ++ps)
                    y[ps] = (ps < NPASS_V || kstep) ? granule_load(gp[par] + 4 * ps) : 0ull;
            };
            // while the records travel: the private parameters' next position
            // and the swept terms' sums there (a poll issued inside the sweep
            // costs a second round trip when the records have not landed yet:
            // A/B 83.2 vs 94.7 M steps/s, profiles/r4/ab)
            if constexpr (!LAST) {
                drift_private(true);
                sweep(M1, M2);
            }
            MC_STAMP(8);
            if (!X1) poll_issue();
            auto poll_eval = [&]() {
                bool ready = true;  // (bitwise: lane masks, no branches)
#pragma unroll
                for (int ps = 0; ps < NPASS; ++ps) {
                    const bool nd = ((need >> ps) & 1u) != 0u;
                    // a pass this lane does not need stays 0: the 16-lane slice
                    // sums run over every column (S < 16 leaves columns idle)
                    vals[ps] = nd ? __uint_as_float((uint32_t)y[ps]) : 0.0f;
                    ready = ready & (!nd | ((uint32_t)(y[ps] >> 32) == epoch));
                }
                return ready;
            };
            bool ready = X1 ? true : poll_eval();
            MC_STAMP(7);
            uint32_t spins = 0;
            while (__ballot(!ready)) {
                if (++spins > kSpinLimit) {
                    ok = false;
                    break;
                }
                // (no s_sleep between polls: the round trip paces them; A/B
                // medium 186.0 -> 188.8 M steps/s, large +0.3 %, profiles/r4/ab)
                poll_issue();
                ready = poll_eval();
            }
            if (!ok) {
                __hip_atomic_store(status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return false;
            }
            MC_STAMP(3);
            __builtin_amdgcn_s_setprio(0);
            // slice sums: a fixed 16-lane DPP tree per pass; pair 4 ps + perm[r]
            // in row r of tot[ps]
            float tot[NPASS];
            if constexpr (X1) {
#pragma unroll
                for (int ps = 0; ps < NPASS; ++ps) tot[ps] = ps < 2 * NRS ? xr[ps] : 0.0f;
            } else {
#pragma unroll
                for (int ps = 0; ps < NPASS; ++ps) {
                    float t = vals[ps];
                    if (ps < NPASS_V || kstep) {
                        t += dpp_row<0xB1>(t);
                        t += dpp_row<0x4E>(t);
                        t += dpp_row<0x141>(t);
                        t += dpp_row<0x140>(t);
                    }
                    tot[ps] = t;
                }
            }
            // totals: the slice sum (the own priors are in slice 0's record)
            if constexpr (LAST) {
                lpn[0] = rl(tot[0], 0) + lp_const;
                lpn[1] = rl(tot[0], 16 * lf_row(1)) + lp_const;
            }
            {
                float gx = 0.0f;
#pragma unroll
                for (int ps = 0; ps < NPASS_V; ++ps)
                    if (col == ps) gx = tot[ps];  // lane 16 row + P / 4 holds pair P
                float gt = gx + g_own;
                // the value's cotangent through the transform's VJP, plus the
                // raw identity terms (eval.h xf_chain: the tape's arithmetic)
                if (hxf) gt = xf_chain(xxf, gt, sh.q, sh.v) + xid;
                sh.g = xon ? gt : 0.0f;
            }
            if constexpr (FIRST) {
                constexpr int p0 = NV, p1 = NV + 1;
                if constexpr (X1) {
                    K0[0] = K0w[0];
                    K0[1] = K0w[1];
                } else {
                    K0[0] = rl(tot[p0 / 4], 16 * lf_row(p0));
                    K0[1] = rl(tot[p1 / 4], 16 * lf_row(p1));
                }
            }
            if constexpr (LAST) {
                constexpr int p0 = NV + 2, p1 = NV + 3;
                if constexpr (X1) {
                    K1[0] = k1w[0];
                    K1[1] = k1w[1];
                } else {
                    K1[0] = rl(tot[p0 / 4], 16 * lf_row(p0));
                    K1[1] = rl(tot[p1 / 4], 16 * lf_row(p1));
                }
            }
            if constexpr (!LAST) drift_shared(true);  // the shared parameters' next position
            MC_STAMP(4);
            return true;
        };
        const std::integral_constant<int, -1> rtpar;
        if (L == 1) {
            ok = step(0, std::integral_constant<int, 3>(), rtpar);
        } else {
            ok = step(0, std::integral_constant<int, 0>(), rtpar);
            for (int l = 1; ok && l < L - 1; ++l) {
                if (X1) ok = step(l, std::integral_constant<int, 1>(), rtpar);
                else if (epoch & 1) ok = step(l, std::integral_constant<int, 1>(), std::integral_constant<int, 0>());
                else ok = step(l, std::integral_constant<int, 1>(), std::integral_constant<int, 1>());
            }
            if (ok) ok = step(L - 1, std::integral_constant<int, 2>(), rtpar);
        }
        if (!ok) break;
        // ---- accept / adapt (identical in every slice of the block) ------------
        float k1s[2] = {0.f, 0.f};
        {
            const float p1 = sh.p + xh * sh.g;
            const float p2 = p1 * p1;
            for (int k = 0; k < nsl; ++k) {
                k1s[0] += lf_sh(p2, k, 0);
                k1s[1] += lf_sh(p2, k, 1);
            }
        }
        bool acc[2];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const float H0 = -lp[c] + 0.5f * (K0[c] + k0s[c]);
            const float H1 = -lpn[c] + 0.5f * (K1[c] + k1s[c]);
            const float ratio = -(H1 - H0);
            float logu = logu_acc[c];
            if (!rngp) {
                const mc_u32x4 ru = mc_draw(cfg.seed, (uint32_t)(cfg.chain_offset + cc[c]),
                                            (uint32_t)it, MC_RNG_TAG_ACCEPT, 0, 0);
                logu = mc_logf_u01(mc_u01_f32(ru.x));
            }
            const bool accepted = logu < ratio;
            acc[c] = accepted;
            nacc[c] += accepted ? 1 : 0;
            ntot[c] += 1;
            const double eps_used = eps[c];
            if (warm && cfg.adapt_step_size && it > 10) {
                const double rate = (double)nacc[c] / (double)ntot[c];
                eps[c] = (rate < cfg.target_accept) ? eps_used * 0.95 : eps_used * 1.05;
            }
            if (accepted) lp[c] = lpn[c];
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
#pragma unroll
        for (int r = 0; r < RS; ++r) {
            q[r] = (f2){acc[0] ? q[r][0] : q0[r][0], acc[1] ? q[r][1] : q0[r][1]};
            g[r] = (f2){acc[0] ? g[r][0] : g0[r][0], acc[1] ? g[r][1] : g0[r][1]};
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
                        if (gk[r] >= 0 && lead) out[gk[r]] = q[r][c];
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
                st_q[cc[c] * D + gk[r]] = q[r][c];
                st_g[cc[c] * D + gk[r]] = g[r][c];
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
