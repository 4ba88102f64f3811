// mh_sliced.h — sliced random-walk Metropolis-Hastings (k_mh_sl): k_mh's
// sampler (mh.h; reference metropolis.py:6-101, the MCMC.run default,
// mcmc.py:135-189) on the data slices and record exchange of the fast-form
// lane layout (lanes_fast.h, nuts_sliced.h), for models too large for one
// chain-per-workgroup tape pass (VERDICT r4 "Next round" 6).
//
// One chain per wave and slice, NW chains per workgroup (k_nuts_sl's
// geometry).  Per iteration:
//   proposal  q' = q + f32(z * f32(scale)), z ~ N(0, I): parameter g takes
//             normal g % 4 of Philox block g / 4 (TAG_PROPOSAL), k_mh's draws;
//             the shared parameters (lane k holds slot k) in every slice
//   log p     forward only: the swept term's sum of squares at q' (d = x - th,
//             s2 = fma(d, d, s2), element pairs packed), the direct term and
//             the shared parameters' own priors (slice 0) — one wave total per
//             slice, one granule per (wave, slice), a fixed column-sum tree
//   accept    f32 log U < f32(lp' - lp) (NaN rejects), the current point stored
//             after every iteration, the proposal's log p carried on acceptance
// Every slice sums the same granules in the same order, so all take the same
// decision and keep the shared parameters' replicas identical.
#pragma once
#include "nuts_sliced.h"

namespace mc {

constexpr int kMslLine = 16;  // granules per (wave, slice) line (one used: 128-byte lines)

// Sum of squares of (x - th) over one lane's run, element pairs packed.
MC_DEV float msl_sumsq(const float* xv, int len, int lmin4, int lmax, float th) {
    f2 a[2] = {{0.f, 0.f}, {0.f, 0.f}};
    const f2 t2 = {th, th};
    int u4 = 0;
    for (; u4 + 2 <= lmin4; u4 += 2) {
        const float4 X = *(const float4*)(xv + u4 * 256), Y = *(const float4*)(xv + (u4 + 1) * 256);
        const f2 d0 = (f2){X.x, X.y} - t2, d1 = (f2){X.z, X.w} - t2;
        const f2 d2 = (f2){Y.x, Y.y} - t2, d3 = (f2){Y.z, Y.w} - t2;
        a[0] = pk_fma(d0, d0, a[0]);
        a[1] = pk_fma(d1, d1, a[1]);
        a[0] = pk_fma(d2, d2, a[0]);
        a[1] = pk_fma(d3, d3, a[1]);
    }
    for (; u4 < lmin4; ++u4) {
        const float4 X = *(const float4*)(xv + u4 * 256);
        const f2 d0 = (f2){X.x, X.y} - t2, d1 = (f2){X.z, X.w} - t2;
        a[0] = pk_fma(d0, d0, a[0]);
        a[1] = pk_fma(d1, d1, a[1]);
    }
    for (int e = 4 * lmin4; e < lmax; e += 4) {  // the ragged end, masked per lane
        const float4 X = *(const float4*)(xv + (e >> 2) * 256);
        f2 d0 = (f2){X.x, X.y} - t2, d1 = (f2){X.z, X.w} - t2;
        d0[0] = (e + 0 < len) ? d0[0] : 0.0f;
        d0[1] = (e + 1 < len) ? d0[1] : 0.0f;
        d1[0] = (e + 2 < len) ? d1[0] : 0.0f;
        d1[1] = (e + 3 < len) ? d1[1] : 0.0f;
        a[0] = pk_fma(d0, d0, a[0]);
        a[1] = pk_fma(d1, d1, a[1]);
    }
    const f2 b = a[0] + a[1];
    return b[0] + b[1];
}

// XL: records published with L2-resident stores (the same-XCD exchange of
// k_hmc_lf, sliced.h granule_store_xcd), the placement checked first.
template <int RS, int NSH, int NW, int OCC, int FORM, bool XL = false>
__global__ void __launch_bounds__(64 * NW, OCC)
k_mh_sl(LrCtx P, RunArgs A, float scale, int64_t chain_base, int64_t n_groups,
        mc_chain_scalars* scal, float* st_q, float* samples, TraceDev tr, unsigned long long* xch,
        int* status, uint32_t ebase) {
    static_assert(NSH <= kLrMaxShared, "shared parameters");
    constexpr bool CF = FORM >= 0;
    static_assert(!CF || lf_nroles(FORM) == NSH, "record slots of a compile-time form");
    if (A.fault && blockIdx.x == gridDim.x - 1) return;  // test hook: never publishes
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const mc_run_config& cfg = A.cfg;
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), j = tid & 63;
    const int S = P.S, D = P.D, Dsh = P.Dsh;
    int64_t grp;
    int slice;
    {
        const int64_t w = blockIdx.x, nwg = gridDim.x;
        if (nwg % 8 == 0 && (nwg / 8) % S == 0) {  // a chain block's slices share an XCD
            const int64_t x = w & 7, r = w >> 3;
            grp = x * ((nwg / 8) / S) + r / S;
            slice = (int)(r % S);
        } else {
            grp = w / S;
            slice = (int)(w % S);
        }
    }
    const int64_t C = cfg.num_chains;
    const int64_t c_raw = chain_base + grp * NW + wave;
    const bool live = c_raw < C;
    const int64_t c = min(c_raw, C - 1);

    float* sd = smem;
    const int64_t* blk = P.blocks + 4 * (int64_t)slice;
    const int64_t doff = blk[0];
    const int dlen = (int)blk[1];
    const int nact = (int)blk[2];
    const int nsweep = (int)(blk[3] & 255);
    const int ndirect = (int)((blk[3] >> 8) & 255);
    (void)nact;
    for (int i = tid; 4 * i < dlen; i += 64 * NW)
        *(float4*)(sd + 4 * i) = *(const float4*)(P.data + doff + 4 * i);
    LrSterm* sst = (LrSterm*)(smem + P.sdata_floats);
    const int sterm_floats = P.n_sterms * (int)(sizeof(LrSterm) / 4);
    for (int i = tid; i < sterm_floats / 4; i += 64 * NW)
        ((float4*)sst)[i] = ((const float4*)P.sterms)[i];
    __syncthreads();  // (the only workgroup barrier)
    if (!live) return;

    const MC_CONST LrTerm* tt = cptr(P.terms) + (int64_t)slice * P.n_terms;
    const LfTerms F = lf_terms(tt, nsweep, ndirect);
    const bool SW = CF ? (FORM & LF_SW) != 0 : F.sw;
    const bool SWS = CF ? (FORM & LF_SWS) != 0 : F.sw_shs;
    const bool DIR = CF ? (FORM & LF_DIR) != 0 : F.dir;
    const bool DM = CF ? (FORM & LF_DM) != 0 : F.d_shm;
    const bool DS = CF ? (FORM & LF_DS) != 0 : F.d_shs;
    const int ksw = CF ? lf_slot_sws(FORM) : max(F.sw_ks, 0);
    const int kdm = CF ? lf_slot_dm(FORM) : max(F.d_km, 0);
    const int kds = CF ? lf_slot_ds(FORM) : max(F.d_ks, 0);
    const int nsl = CF ? NSH : Dsh;
    auto ord_of = [&](int k) {
        int o = F.d_ks;
        o = (DM && k == kdm) ? F.d_km : o;
        o = (SWS && k == ksw) ? F.sw_ks : o;
        return CF ? o : k;
    };
    const bool xon = j < nsl;
    const int xk = xon ? j : 0;
    const int xo = xon ? ord_of(xk) : 0;
    int xg = P.shl[0];
#pragma unroll
    for (int k = 1; k < kLrMaxShared; ++k) xg = (xo == k) ? P.shl[k] : xg;
    const int rep = P.rep;
    const bool lead = (j & (rep - 1)) == 0;
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
    const LrOwn own = lr_own_prior(P.n_sterms, sst, xon ? 2 * xo : 64, Dsh);
    const bool own_lp = own.on && slice == 0;

    int gk[RS];
    const float* xv[RS];
    int len[RS], lmin4[RS], lmax[RS];
    float cnt[RS];
    bool pdir[RS];
    float q[RS];
#pragma unroll
    for (int r = 0; r < RS; ++r) {
        gk[r] = P.gidx[((int64_t)slice * kLrMaxSlots + r) * 64 + j];
        len[r] = 0;
        lmin4[r] = 0;
        xv[r] = sd;
        if (SW && r < tt[0].nslot) {
            len[r] = ((const int32_t*)sd)[tt[0].len_off + r * 64 + j];
            lmin4[r] = tt[0].lmin4[r];
            xv[r] = sd + tt[0].doff[0] + tt[0].toff[r] + 4 * j;
        }
        cnt[r] = (float)len[r];
        int mx = len[r];
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) mx = max(mx, __shfl_xor(mx, o));
        lmax[r] = __builtin_amdgcn_readfirstlane(mx);
        pdir[r] = DIR && r < tt[nsweep].nslot &&
                  ((const int32_t*)sd)[tt[nsweep].len_off + r * 64 + j] > 0;
        q[r] = gk[r] >= 0 ? st_q[c * D + gk[r]] : 0.0f;
    }
    float qs = xon ? st_q[c * D + xg] : 1.0f;  // the lane's shared parameter (raw)

    // exchange: granule 0 of one 128-byte line per (wave, slice, parity);
    // lanes (row, col) with col < S poll slice col's granule (row 0 sums)
    unsigned long long* const gline0 = xch + ((int64_t)grp * NW + wave) * S * kMslLine;
    const int64_t pstride = (int64_t)n_groups * NW * S * kMslLine;
    const int CW = S > 8 ? 16 : 8;
    const int pcol = j % CW;
    const bool poll_lane = j < CW && pcol < S;
    unsigned long long* const gp0 = gline0 + min(pcol, S - 1) * kMslLine;

    float lp = scal[c].logp;
    int n_acc = scal[c].n_accept, n_tot = scal[c].n_total;
    const uint32_t chain_id = (uint32_t)(cfg.chain_offset + c);
    const float fscale = scale;
    uint32_t epoch = ebase;
    bool ok = true;
    const int64_t it_end = cfg.iter_begin + cfg.iter_count;
    // XL: the block's slices share an XCD (sliced.h xcd_announce / xcd_agree;
    // slots: granule 15 of each slice's parity-0 line of wave 0 — the record
    // is granule 0)
    unsigned long long* const xslots = xch + ((int64_t)grp * NW) * S * kMslLine + 15;
    XcdPoll xpoll = {0ull};
    if (XL && cfg.iter_count > 0)
        xpoll = xcd_announce(xslots, S, slice, ebase + 1, wave == 0 && j == 0);
    for (int64_t it = cfg.iter_begin; it < it_end; ++it) {
        if (XL && it == cfg.iter_begin) {  // (before the launch's first publish)
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
        // Gaussian random walk (metropolis.py:66-74): parameter g takes normal
        // g % 4 of Philox block g / 4 (k_mh's mapping)
        auto normal_of = [&](int gi) {
            const mc_u32x4 rr = mc_draw(cfg.seed, chain_id, (uint32_t)it, MC_RNG_TAG_PROPOSAL, 0,
                                        (uint32_t)(gi >> 2));
            float z0, z1;
            if ((gi & 3) < 2) mc_box_muller(rr.x, rr.y, &z0, &z1);
            else mc_box_muller(rr.z, rr.w, &z0, &z1);
            return (gi & 1) ? z1 : z0;
        };
        float qn[RS];
#pragma unroll
        for (int r = 0; r < RS; ++r) qn[r] = gk[r] >= 0 ? q[r] + normal_of(gk[r]) * fscale : 0.0f;
        const float qsn = xon ? qs + normal_of(xg) * fscale : 1.0f;
        // the proposal's shared values and derived scales (every lane reads
        // the holder lanes'; rcp / log as the other lane kernels)
        const float v = hxf ? xf_apply(xxf, qsn) : qsn;
        const float is = __builtin_amdgcn_rcpf(v);
        const float lgv = __builtin_amdgcn_logf(v) * 0.693147180559945f;
        // log p partial of this slice at the proposal (forward only)
        float lpp = 0.0f;
        if (SW) {
            const float sis = SWS ? rl(is, ksw) : F.sw_cinv;
            const float iv = SWS ? sis * sis : F.sw_cinv2;
            const float lg = SWS ? rl(lgv, ksw) : F.sw_clogs;
#pragma unroll
            for (int r = 0; r < RS; ++r) {
                if (len[r] == 0) continue;
                const float s2 = msl_sumsq(xv[r], len[r], lmin4[r], lmax[r], qn[r]);
                lpp += F.sw_w * (cnt[r] * (F.sw_c0 - lg) - (0.5f * s2) * iv);
            }
        }
        if (DIR) {
            const float um = DM ? rl(v, kdm) : F.d_m;
            const float dis = DS ? rl(is, kds) : F.d_cinv;
            const float iv = DS ? dis * dis : F.d_cinv2;
            const float lg = DS ? rl(lgv, kds) : F.d_clogs;
#pragma unroll
            for (int r = 0; r < RS; ++r) {
                if (!pdir[r]) continue;
                const float d = qn[r] - um;
                lpp += F.d_w * (1.0f * (F.d_c0 - lg) - (0.5f * (d * d)) * iv);
            }
        }
#ifdef MC_JIT_LANES
        // the expression terms (LS_EXPR beside a fast form: LanePlan::nuts_expr),
        // their element code generated per program, value only (jit.hip)
        if constexpr (!CF) {
            LrShared shp;
            shp.q = qsn;
            shp.v = v;
            shp.p = shp.g = 0.0f;
            shp.is = is;
            shp.iv = is * is;
            shp.lg = lgv;
            for (int t = nsweep + ndirect; t < nact; ++t)
                if (tt[t].sig == LS_EXPR) mc_jit_lane_expr1v(tt + t, sd, j, shp, lpp);
        }
#endif
        {  // the own prior of the lane's shared parameter, identity terms (slice 0)
            const float d = own.hn ? v : v - own.m;
            const bool out = own.hn && !(v >= 0.0f);
            const float lpe = out ? -__builtin_inff() : own.c0l - (0.5f * (d * d)) * own.cinv2;
            if (own_lp) lpp += own.wn * lpe;
            if (hxf && slice == 0 && xon) lpp += xid * qsn;
        }
        // the slice's total, published; every slice's, summed in a fixed tree
        const float wt = wave_sum(lpp);
        ++epoch;
        const int par = epoch & 1;
        if (j == 0) granule_put(gline0 + par * pstride + slice * kMslLine, epoch, wt, XL);
        unsigned long long* const gpp = gp0 + par * pstride;
        unsigned long long y = poll_lane ? granule_load(gpp) : 0ull;
        // the accept draw while the records travel (metropolis.py:81-88)
        const mc_u32x4 ru = mc_draw(cfg.seed, chain_id, (uint32_t)it, MC_RNG_TAG_ACCEPT, 0, 0);
        const float logu = mc_logf_u01(mc_u01_f32(ru.x));
        uint32_t spins = 0;
        while (__ballot(poll_lane && (uint32_t)(y >> 32) != epoch)) {
            if (++spins > kSpinLimit) {
                ok = false;
                break;
            }
            y = poll_lane ? granule_load(gpp) : 0ull;
        }
        if (!ok) {
            __hip_atomic_store(status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
        const float tot = nsl_colsum(poll_lane ? __uint_as_float((uint32_t)y) : 0.0f, CW);
        const float lpn = rl(tot, 0) + P.lp_const;
        const float ratio = lpn - lp;
        const bool accepted = logu < ratio;
        if (accepted) {
#pragma unroll
            for (int r = 0; r < RS; ++r) q[r] = qn[r];
            qs = qsn;
            lp = lpn;
        }
        n_acc += accepted ? 1 : 0;
        n_tot += 1;
        if (samples != nullptr) {
            const int64_t s = it - cfg.num_warmup - cfg.sample_begin;
            if (s >= 0 && s < cfg.sample_capacity) {
                float* out = samples + (c * cfg.sample_capacity + s) * (int64_t)D;
#pragma unroll
                for (int r = 0; r < RS; ++r)
                    if (gk[r] >= 0 && lead) out[gk[r]] = q[r];
                if (slice == 0 && xon) out[xg] = qs;
            }
        }
        if (slice == 0 && j == 0) {
            const int64_t ti = it - tr.iter_begin;
            if (ti >= 0 && ti < tr.capacity) {
                const int64_t o = c * tr.capacity + ti;
                if (tr.accepted) tr.accepted[o] = accepted ? 1 : 0;
                if (tr.accept_stat) tr.accept_stat[o] = ratio;
                if (tr.step_size) tr.step_size[o] = (double)scale;
                if (tr.energy) tr.energy[o] = lp;
                if (tr.tree_depth) tr.tree_depth[o] = 0;
                if (tr.n_leapfrog) tr.n_leapfrog[o] = 0;
            }
        }
    }
    if (!ok) return;  // a timed-out chain keeps its state (mc_workspace_status reports it)
#pragma unroll
    for (int r = 0; r < RS; ++r)
        if (gk[r] >= 0 && lead) st_q[c * D + gk[r]] = q[r];
    if (slice == 0 && xon) st_q[c * D + xg] = qs;
    if (slice == 0 && j == 0) {
        mc_chain_scalars& sc = scal[c];
        sc.logp = lp;
        sc.n_accept = n_acc;
        sc.n_total = n_tot;
    }
}

}  // namespace mc
