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
// What differs from k_hmc_lr:
//   * the terms' fields, the lanes holding their shared operands and the
//     runs' data pointers are read once per launch (k_hmc_lr re-reads them
//     from constant memory at every step and indexes its cotangent partials
//     by a runtime ordinal, which the compiler keeps in scratch);
//   * the moment sweep keeps even and odd elements in separate packed
//     accumulators (two dependency chains each; a dependent v_pk_add_f32
//     advances every 10 cycles, scripts/micro/pk_probe.hip);
//   * the wave totals of the record are reduce-scattered (permlane32 /
//     permlane16 swaps + one 16-lane DPP row sum) so that pair P's total is
//     in row perm[P % 4] of register P / 4 — no readlanes, no publish select;
//     the poll uses the same pair -> row map, so after the slice sums the
//     lane that holds shared parameter (k, c) finds its cotangent total in
//     its own register (lane 16 perm[P % 4] + P / 4, P = 2 (k + 1) + c);
//   * the kinetic-energy items K0 / K1 travel only on the first / last step.
// Results equal k_hmc_lr's up to fp32 summation order; runs are
// bit-reproducible and independent of how chains are split over launches.
#pragma once
#include "lanes.h"

namespace mc {

// pair P -> the row (16-lane group) that holds its total after the
// reduce-scatter / the slice sums: rows hold values 4n + {0, 2, 1, 3}
MC_DEV constexpr int lf_row(int P) { return (P & 3) == 1 ? 2 : ((P & 3) == 2 ? 1 : (P & 3)); }
// the lane that holds shared parameter k of chain c
MC_DEV constexpr int lf_shlane(int k, int c) {
    return 16 * lf_row(2 * (k + 1) + c) + (2 * (k + 1) + c) / 4;
}
// Uniform (per chain) value `v` of shared parameter k, chain c.
MC_DEV float lf_sh(float v, int k, int c) { return rl(v, lf_shlane(k, c)); }

// Reduce-scatter of 8 per-lane values over the wave: returns two registers;
// row r of register n holds (in all 16 lanes) the wave total of value
// 4n + {0, 2, 1, 3}[r].  A fixed tree: the same bits in every wave / slice.
MC_DEV void lf_rs8(const float (&v)[8], float (&x)[2]) {
    float w[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {  // lanes 0-31: v[2m] sums, lanes 32-63: v[2m+1]
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

// Moment sums of one lane's run (value = data x, loc = the lane's private
// parameter th) for both chains, packed FP32: d = x - th, s1 += d,
// s2 = fma(d, d, s2), with the even and odd elements in separate packed
// accumulators (two independent dependency chains each).
MC_DEV void lf_moments(const float* xv, int len, int lmin4, f2 th, f2& s1, f2& s2) {
    f2 a1[2] = {{0.f, 0.f}, {0.f, 0.f}}, a2[2] = {{0.f, 0.f}, {0.f, 0.f}};
    auto elem = [&](float x, int hh) {
        const f2 d = (f2){x, x} - th;
        a1[hh] += d;
        a2[hh] = pk_fma(d, d, a2[hh]);
    };
    int u4 = 0;
    for (; u4 + 4 <= lmin4; u4 += 4) {
        float4 a[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) a[q] = *(const float4*)(xv + (u4 + q) * 256);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            elem(a[q].x, 0);
            elem(a[q].y, 1);
            elem(a[q].z, 0);
            elem(a[q].w, 1);
        }
    }
    for (; u4 < lmin4; ++u4) {
        const float4 a = *(const float4*)(xv + u4 * 256);
        elem(a.x, 0);
        elem(a.y, 1);
        elem(a.z, 0);
        elem(a.w, 1);
    }
    for (int u = 4 * u4; u < len; ++u) elem(xv[(u >> 2) * 256 + (u & 3)], u & 1);
    s1 = a1[0] + a1[1];
    s2 = a2[0] + a2[1];
}

// The fast-form terms of a slice, read once per launch: at most one swept
// term (y ~ N(theta[g], scale): value data, loc private, scale shared or
// constant) and one direct term (theta ~ N(loc, scale), loc / scale shared or
// constant).  Shared operands are addressed by the lanes that hold them.
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

template <int RS, int NSH, int NW, bool X1>
__global__ void __launch_bounds__(64 * NW)
k_hmc_lf(LrCtx P, RunArgs A, int64_t chain_base, int64_t n_groups, mc_chain_scalars* scal,
         float* st_q, float* st_g, float* samples, TraceDev tr, unsigned long long* xch,
         int* status, uint32_t ebase) {
    static_assert(NSH <= kLrMaxShared, "shared parameters");
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
    // this lane's shared parameter: (xk, xc) with lf_shlane(xk, xc) == j
    int xk = -1, xc = 0;
#pragma unroll
    for (int k = 0; k < kLrMaxShared; ++k)
#pragma unroll
        for (int c = 0; c < 2; ++c)
            if (k < Dsh && lf_shlane(k, c) == j) {
                xk = k;
                xc = c;
            }
    const bool xon = xk >= 0;
    int xg = P.shl[0];
#pragma unroll
    for (int k = 1; k < kLrMaxShared; ++k) xg = (xk == k) ? P.shl[k] : xg;
    const int64_t xch_id = xc ? cc[1] : cc[0];
    const bool xlive = xon && (xc ? live[1] : live[0]);

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
    sh.is = sh.iv = 1.0f;
    sh.lg = 0.0f;
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
    // the lane's own prior: lr_own_prior keys it by ordinal k = lane / 2
    const LrOwn own = lr_own_prior(P.n_sterms, sst, xon ? 2 * xk + xc : 64, Dsh);
    const LfTerms F = lf_terms(tt, nsweep, ndirect);
    // per slot: the swept term's run (data pointer, length, full float4
    // groups of every lane) and the direct term's presence
    const float* xv[RS];
    int len[RS], lmin4[RS];
    float cnt[RS];
    bool pdir[RS];
#pragma unroll
    for (int r = 0; r < RS; ++r) {
        len[r] = 0;
        lmin4[r] = 0;
        xv[r] = sd;
        if (F.sw && r < tt[0].nslot) {
            len[r] = ((const int32_t*)sd)[tt[0].len_off + r * 64 + j];
            lmin4[r] = tt[0].lmin4[r];
            xv[r] = sd + tt[0].doff[0] + tt[0].toff[r] + 4 * j;
        }
        cnt[r] = (float)len[r];
        pdir[r] = F.dir && r < tt[nsweep].nslot &&
                  ((const int32_t*)sd)[tt[nsweep].len_off + r * 64 + j] > 0;
    }
    // the lanes that hold the shared operands, per chain
    const int sw_l0 = lf_shlane(max(F.sw_ks, 0), 0), sw_l1 = lf_shlane(max(F.sw_ks, 0), 1);
    const int dm_l0 = lf_shlane(max(F.d_km, 0), 0), dm_l1 = lf_shlane(max(F.d_km, 0), 1);
    const int ds_l0 = lf_shlane(max(F.d_ks, 0), 0), ds_l1 = lf_shlane(max(F.d_ks, 0), 1);
    // the swept terms' moment sums at the current point, both chains
    auto sweep = [&](f2 (&s1)[RS], f2 (&s2)[RS]) {
#pragma unroll
        for (int r = 0; r < RS; ++r) {
            s1[r] = (f2){0.f, 0.f};
            s2[r] = (f2){0.f, 0.f};
            if (len[r] > 0) lf_moments(xv[r], len[r], lmin4[r], (f2){R.q[r][0], R.q[r][1]}, s1[r], s2[r]);
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
    // publishing: lanes 16 r + n (n < NRS * 2) hold pair 8 (n / 2) + 4 (n % 2) + perm[r]
    const int pub_pair = (col < 2 * NRS) ? 8 * (col >> 1) + 4 * (col & 1) + lf_row(row) : -1;
    const int64_t it_end = cfg.iter_begin + cfg.iter_count;
    for (int64_t it = cfg.iter_begin; it < it_end && ok; ++it) {
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
                k0p[c] += z * z;
            }
        }
        sh.p = xon ? normal_of(xg, xch_id) : 0.0f;
        const float K0w[2] = {wave_sum(k0p[0]), wave_sum(k0p[1])};
        float k0s[2] = {0.f, 0.f};  // the shared parameters' part, in parameter order
        {
            const float p2 = sh.p * sh.p;
            for (int k = 0; k < Dsh; ++k) {
                k0s[0] += lf_sh(p2, k, 0);
                k0s[1] += lf_sh(p2, k, 1);
            }
        }
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
            sh.is = 1.0f / sh.q;
            sh.iv = 1.0f / (sh.q * sh.q);
            sh.lg = logf(sh.q);
        };
        f2 M1[RS], M2[RS];
        drift_private(false);
        drift_shared(false);
        sweep(M1, M2);
        for (int l = 0; l < L; ++l) {
            MC_STAMP(0);
            // finish the swept term from its moment sums, evaluate the direct
            // term (k_hmc_lr's lr_finish; same arithmetic, scalar per chain):
            // log p partial, complete private gradients, cotangent partials of
            // the swept scale (cs), the direct loc (cm) and scale (cd)
            float lpp[2] = {0.f, 0.f}, cs[2] = {0.f, 0.f}, cm[2] = {0.f, 0.f}, cd[2] = {0.f, 0.f};
#pragma unroll
            for (int r = 0; r < RS; ++r) R.g[r][0] = R.g[r][1] = 0.0f;
            if (F.sw) {
                float is[2], iv[2], lg[2];
                is[0] = F.sw_shs ? rl(sh.is, sw_l0) : F.sw_cinv;
                is[1] = F.sw_shs ? rl(sh.is, sw_l1) : F.sw_cinv;
                iv[0] = F.sw_shs ? rl(sh.iv, sw_l0) : F.sw_cinv2;
                iv[1] = F.sw_shs ? rl(sh.iv, sw_l1) : F.sw_cinv2;
                lg[0] = F.sw_shs ? rl(sh.lg, sw_l0) : F.sw_clogs;
                lg[1] = F.sw_shs ? rl(sh.lg, sw_l1) : F.sw_clogs;
#pragma unroll
                for (int r = 0; r < RS; ++r) {
                    if (cnt[r] == 0.0f) continue;
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        const float s1 = M1[r][c], s2 = M2[r][c];
                        const float lpt = cnt[r] * (F.sw_c0 - lg[c]) - (0.5f * s2) * iv[c];
                        lpp[c] += F.sw_w * lpt;
                        R.g[r][c] += F.sw_w * (s1 * iv[c]);
                        cs[c] += F.sw_w * ((s2 * iv[c] - cnt[r]) * is[c]);
                    }
                }
            }
            if (F.dir) {
                float um[2], is[2], iv[2], lg[2];
                um[0] = F.d_shm ? rl(sh.q, dm_l0) : F.d_m;
                um[1] = F.d_shm ? rl(sh.q, dm_l1) : F.d_m;
                is[0] = F.d_shs ? rl(sh.is, ds_l0) : F.d_cinv;
                is[1] = F.d_shs ? rl(sh.is, ds_l1) : F.d_cinv;
                iv[0] = F.d_shs ? rl(sh.iv, ds_l0) : F.d_cinv2;
                iv[1] = F.d_shs ? rl(sh.iv, ds_l1) : F.d_cinv2;
                lg[0] = F.d_shs ? rl(sh.lg, ds_l0) : F.d_clogs;
                lg[1] = F.d_shs ? rl(sh.lg, ds_l1) : F.d_clogs;
#pragma unroll
                for (int r = 0; r < RS; ++r) {
                    if (!pdir[r]) continue;
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        const float d = R.q[r][c] - um[c];
                        const float s2 = d * d;
                        const float lpt = 1.0f * (F.d_c0 - lg[c]) - (0.5f * s2) * iv[c];
                        lpp[c] += F.d_w * lpt;
                        const float u = F.d_w * (d * iv[c]);
                        R.g[r][c] += -u;
                        cm[c] += u;
                        cd[c] += F.d_w * ((s2 * iv[c] - 1.0f) * is[c]);
                    }
                }
            }
            MC_STAMP(1);
            // wave totals, reduce-scattered: pair P = 2 item + chain
            float xr[2 * NRS];
            {
                float v[8 * NRS];
#pragma unroll
                for (int x = 0; x < 8 * NRS; ++x) v[x] = 0.0f;
                v[0] = lpp[0];
                v[1] = lpp[1];
#pragma unroll
                for (int k = 0; k < NSH; ++k)
#pragma unroll
                    for (int c = 0; c < 2; ++c)
                        v[2 + 2 * k + c] = ((F.sw_ks == k ? cs[c] : 0.0f) +
                                            (F.d_km == k ? cm[c] : 0.0f)) +
                                           (F.d_ks == k ? cd[c] : 0.0f);
#pragma unroll
                for (int q = 0; q < NRS; ++q) {
                    float vv[8], xx[2];
#pragma unroll
                    for (int x = 0; x < 8; ++x) vv[x] = v[8 * q + x];
                    lf_rs8(vv, xx);
                    xr[2 * q] = xx[0];
                    xr[2 * q + 1] = xx[1];
                }
            }
            // the kinetic partials of the first / last step (uniform)
            float k1w[2] = {0.f, 0.f};
            if (l == L - 1) {
                float k1p[2] = {0.f, 0.f};
#pragma unroll
                for (int c = 0; c < 2; ++c)
#pragma unroll
                    for (int r = 0; r < RS; ++r) {
                        const float pj = R.p[r][c] + h[c] * R.g[r][c];
                        k1p[c] += pj * pj;
                    }
                k1w[0] = wave_sum(k1p[0]);
                k1w[1] = wave_sum(k1p[1]);
            }
            ++epoch;
            const int par = epoch & 1;
            if (!X1) {
                // one store instruction: the record pairs, and the K items on the
                // first / last step (lanes 2, 3 of rows 0 / 1)
                int pp = -1;
                float pv = 0.0f;
                if (pub_pair >= 0 && pub_pair < NV) {
                    pp = pub_pair;
                    pv = xr[0];
#pragma unroll
                    for (int x = 1; x < 2 * NRS; ++x)
                        if (x == 2 * (col >> 1) + (col & 1)) pv = xr[x];
                }
                if (col == 2 * NRS || col == 2 * NRS + 1) {
                    const int c = col - 2 * NRS;
                    if (row == 0 && l == 0) {
                        pp = NV + c;
                        pv = c ? K0w[1] : K0w[0];
                    }
                    if (row == 1 && l == L - 1) {
                        pp = NV + 2 + c;
                        pv = c ? k1w[1] : k1w[0];
                    }
                }
                if (pp >= 0) granule_store(gline[par] + slice * 16 + pp, epoch, pv);
            }
            MC_STAMP(2);
            // while the records travel: the private parameters' next position
            // and the swept terms' sums there
            if (l + 1 < L) {
                drift_private(true);
                sweep(M1, M2);
            }
            // poll: pass ps reads pair 4 ps + perm[row] of slice col
            float vals[NPASS];
            uint32_t need = 0;
            unsigned long long y0[NPASS];
            const bool kstep = (l == 0) || (l == L - 1);
#pragma unroll
            for (int ps = 0; ps < NPASS; ++ps) {
                const int pr = 4 * ps + lf_row(row);
                const bool want = !X1 && poll_lane && pr < NPAIR && (pr < NV || kstep) &&
                                  (pr < NV || (pr < NV + 2 ? l == 0 : l == L - 1));
                y0[ps] = want ? granule_load(gline[par] + col * 16 + pr) : 0ull;
                vals[ps] = 0.0f;
                if (want) need |= 1u << ps;
            }
            // the own priors of the shared parameters (lanes holding one)
            float lp_own = 0.0f, g_own = 0.0f;
            if (own.on) {
                const float v = sh.q;
                const float d = own.hn ? v : v - own.m;
                const float d2 = d * d;
                const bool out = own.hn && !(v >= 0.0f);
                const float lpe = out ? -__builtin_inff() : own.c0l - (0.5f * d2) * own.cinv2;
                lp_own = own.wn * lpe;
                g_own = out ? 0.0f : own.wn * -(d * own.cinv2);
            }
            float slp[2] = {0.f, 0.f};
            for (int k = 0; k < Dsh; ++k) {
                slp[0] += lf_sh(lp_own, k, 0);
                slp[1] += lf_sh(lp_own, k, 1);
            }
            MC_STAMP(7);
#pragma unroll
            for (int ps = 0; ps < NPASS; ++ps) {
                if ((need >> ps) & 1u) {
                    if ((uint32_t)(y0[ps] >> 32) == epoch) {
                        vals[ps] = __uint_as_float((uint32_t)y0[ps]);
                        need &= ~(1u << ps);
                    }
                }
            }
            uint32_t spins = 0;
            while (__ballot(need != 0)) {
                if (++spins > kSpinLimit) {
                    ok = false;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
#pragma unroll
                for (int ps = 0; ps < NPASS; ++ps) {
                    if ((need >> ps) & 1u) {
                        const int pr = 4 * ps + lf_row(row);
                        const unsigned long long y = granule_load(gline[par] + col * 16 + pr);
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
            // totals: the slice sum plus the own priors' sum
            lpn[0] = (rl(tot[0], 0) + slp[0]) + P.lp_const;
            lpn[1] = (rl(tot[0], 16 * lf_row(1)) + slp[1]) + P.lp_const;
            {
                float gx = 0.0f;
#pragma unroll
                for (int ps = 0; ps < NPASS_V; ++ps)
                    if (j % 16 == ps) gx = tot[ps];  // lane 16 row + P / 4 holds pair P
                sh.g = xon ? gx + g_own : 0.0f;
            }
            if (l == 0) {
                const int p0 = NV, p1 = NV + 1;
                if constexpr (X1) {
                    K0[0] = K0w[0];
                    K0[1] = K0w[1];
                } else {
                    K0[0] = rl(tot[p0 / 4], 16 * lf_row(p0));
                    K0[1] = rl(tot[p1 / 4], 16 * lf_row(p1));
                }
            }
            if (l == L - 1) {
                const int p0 = NV + 2, p1 = NV + 3;
                if constexpr (X1) {
                    K1[0] = k1w[0];
                    K1[1] = k1w[1];
                } else {
                    K1[0] = rl(tot[p0 / 4], 16 * lf_row(p0));
                    K1[1] = rl(tot[p1 / 4], 16 * lf_row(p1));
                }
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
            const mc_u32x4 ru = mc_draw(cfg.seed, (uint32_t)(cfg.chain_offset + cc[c]),
                                        (uint32_t)it, MC_RNG_TAG_ACCEPT, 0, 0);
            const float logu = mc_logf_ref(mc_u01_f32(ru.x));
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
                        if (gk[r] >= 0) out[gk[r]] = R.q[r][c];
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
            if (gk[r] >= 0) {
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
