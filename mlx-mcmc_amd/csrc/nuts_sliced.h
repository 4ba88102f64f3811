// nuts_sliced.h — sliced lane-resident NUTS (k_nuts_sl): the iterative
// slice-NUTS of k_nuts / k_nuts_lr (nuts.h, nuts_lanes.h; reference
// nuts.py:16-358, the same draws and decision rules) on the data slices and
// L2 record exchange of the fast-form HMC kernel k_hmc_lf (lanes_fast.h), for
// models too large for one lane-resident slice (the README "Large" row:
// 1000 parameters, 100 K observations).
//
// Work split.  A workgroup holds one data slice (LDS) and NW chains, one
// chain per wave.  The S waves of a chain (one per slice, S <= 16) walk the
// same tree in lock step: every leaf is one leapfrog step and one gradient,
// each slice evaluates its share, and the slices exchange one record per
// leaf (tagged 8-byte granules, as k_hmc_lf) and sum it in a fixed DPP tree,
// so every slice holds the same totals bit for bit and takes the same tree
// decisions.  The broadcast ("shared") parameters (mu, tau, sigma) are
// replicated in every slice (lane k holds shared slot k), the private ones
// (theta_g with its observations) live in the slice that holds their data
// (lane, register slot) exactly as in k_hmc_lf.
//
// A leaf's record: log p, the private kinetic energy, the shared cotangents
// (by role: swept scale, direct loc, direct scale), the U-turn dot partials
// of every merge the leaf closes (2 per level: the subtree's first leaf
// against this end, nuts.py:119-135 / 214) and of the top-level test when
// the leaf completes its subtree (nuts.py:276), and on an iteration's first
// leaf the kinetic energy of the drawn momentum (H0, nuts.py:231).  All
// merge levels' dots travel in the same record (they depend on no decision
// of the leaf): the merges then run in order from the exchanged totals,
// stopping at the first U-turn, as the reference's recursion does.
//
// Trajectory storage: the two ends and the current sample in registers, the
// subtrees' first leaves (q, r) in an LDS arena per wave (read at the merges),
// the candidate pool (q, g) in global memory (written every leaf, read only
// by the top-level accept), the shared parameters' share of both in a small
// LDS arena (lane k, slot k).
//
// Sweep-ahead: the next leaf's private position depends only on this leaf's
// private gradients, complete inside the lanes before the exchange — the
// next leaf continues from this end, or from the other end in the next
// subtree's drawn direction — so its moment sums are taken while this leaf's
// records travel (k_hmc_lf's pattern); when the walk stops instead, the sums
// are discarded.
#pragma once
#include "lanes_fast.h"
#include "nuts.h"

namespace mc {

constexpr int kNslLine = 32;      // granules per (wave, slice) record line
constexpr int kNslMaxDepth = 12;  // max_tree_depth the record layout holds (3 dot groups)

// LDS floats per wave of the first-leaf arena: (q, r) of the subtrees' first
// leaves, MAXJ slots x 2 components x RS register slots x 64 lanes
__host__ __device__ constexpr int64_t nuts_sl_first_floats(int rs, int maxj) {
    return (int64_t)maxj * 2 * rs * 64;
}
// the shared parameters' arena rows per wave: 2 MAXJ first-leaf rows, then
// 2 (MAXJ + 2) pool rows; 4 floats each (shared slot k at float k)
__host__ __device__ constexpr int64_t nuts_sl_shared_rows(int maxj) {
    return 2 * (int64_t)maxj + 2 * ((int64_t)maxj + 2);
}
// global candidate pool per (chain, slice): (MAXJ + 2) slots x (q, g) x RS rows x 64
__host__ __device__ constexpr int64_t nuts_sl_pool_floats(int rs, int maxj) {
    return ((int64_t)maxj + 2) * 2 * rs * 64;
}

// Moment sums of one lane's run for one chain: element pairs packed
// (d = (x0, x1) - (th, th), s1 += d, s2 = fma(d, d, s2)), two register pairs
// per float4 (four independent dependency chains), the LDS loads of the next
// 16 elements issued before this round's arithmetic (lf_moments' pipeline).
template <int PIPE = 4>
MC_DEV void nsl_moments(const float* xv, int len, int lmin4, int lmax, float th, float& s1,
                        float& s2) {
    f2 a1[2] = {{0.f, 0.f}, {0.f, 0.f}}, a2[2] = {{0.f, 0.f}, {0.f, 0.f}};
    const f2 t2 = {th, th};
    auto quad = [&](float4 X) {
        const f2 d0 = (f2){X.x, X.y} - t2;
        a1[0] += d0;
        a2[0] = pk_fma(d0, d0, a2[0]);
        const f2 d1 = (f2){X.z, X.w} - t2;
        a1[1] += d1;
        a2[1] = pk_fma(d1, d1, a2[1]);
    };
    int u4 = 0;
    // (PIPE float4 groups per round: 4 with two waves per SIMD, 2 with four,
    // where the other waves hide more of the load latency and the registers
    // are half as many)
    if (lmin4 >= PIPE) {
        float4 A[PIPE], B[PIPE];
        auto load = [&](float4 (&X)[PIPE], int g) {
#pragma unroll
            for (int q = 0; q < PIPE; ++q) X[q] = *(const float4*)(xv + (g + q) * 256);
        };
        auto round = [&](const float4 (&X)[PIPE]) {
#pragma unroll
            for (int q = 0; q < PIPE; ++q) quad(X[q]);
        };
        const int last = lmin4 - PIPE;
        load(A, 0);
        for (;;) {
            const bool more_b = u4 + 2 * PIPE <= lmin4;
            load(B, min(u4 + PIPE, last));
            round(A);
            u4 += PIPE;
            if (!more_b) break;
            const bool more_a = u4 + 2 * PIPE <= lmin4;
            load(A, min(u4 + PIPE, last));
            round(B);
            u4 += PIPE;
            if (!more_a) break;
        }
    }
    for (; u4 < lmin4; ++u4) quad(*(const float4*)(xv + u4 * 256));
    // the ragged end (uniform bounds, masked per lane; tiles are padded to
    // whole groups, so every load is in bounds)
    for (int e = 4 * lmin4; e < lmax; e += 4) {
        const float4 X = *(const float4*)(xv + (e >> 2) * 256);
        f2 d0 = (f2){X.x, X.y} - t2, d1 = (f2){X.z, X.w} - t2;
        d0[0] = (e + 0 < len) ? d0[0] : 0.0f;
        d0[1] = (e + 1 < len) ? d0[1] : 0.0f;
        d1[0] = (e + 2 < len) ? d1[0] : 0.0f;
        d1[1] = (e + 3 < len) ? d1[1] : 0.0f;
        a1[0] += d0;
        a2[0] = pk_fma(d0, d0, a2[0]);
        a1[1] += d1;
        a2[1] = pk_fma(d1, d1, a2[1]);
    }
    const f2 b1 = a1[0] + a1[1], b2 = a2[0] + a2[1];
    s1 = b1[0] + b1[1];
    s2 = b2[0] + b2[1];
}

// The fixed tree that sums a CW-lane column group (CW = 16 or 8 lanes):
// every lane of the group ends with the same bits.
MC_DEV float nsl_colsum(float t, int cw) {
    t += dpp_row<0xB1>(t);   // quad_perm [1,0,3,2]
    t += dpp_row<0x4E>(t);   // quad_perm [2,3,0,1]
    t += dpp_row<0x141>(t);  // row_half_mirror
    if (cw == 16) t += dpp_row<0x140>(t);  // row_mirror
    return t;
}

// NSH: shared slots of the record (FORM >= 0: lf_nroles(FORM)); NW chains
// (waves) per workgroup; OCC the waves per SIMD the register budget allows.
// XL: records published with L2-resident stores (the same-XCD exchange of
// k_hmc_lf, sliced.h granule_store_xcd), the placement checked at the
// launch's first iteration.
template <int RS, int NSH, int NW, int OCC, int FORM, bool XL = false>
__global__ void __launch_bounds__(64 * NW, OCC)
k_nuts_sl(LrCtx P, RunArgs A, int64_t chain_base, int64_t n_groups, mc_chain_scalars* scal,
          float* st_q, float* st_g, float* samples, TraceDev tr, unsigned long long* xch,
          float* pool, int* status, uint32_t ebase) {
    static_assert(NSH <= kLrMaxShared, "shared parameters");
    constexpr bool CF = FORM >= 0;
    static_assert(!CF || lf_nroles(FORM) == NSH, "record slots of a compile-time form");
    // record positions: group 0 = lp, K, the NSH cotangents, dot slot 0 (a,
    // b); K0 in group 0's last pair when NSH <= 3, else group 1's first; group
    // g >= 1: dot slots 4 (g - 1) + 1 .. + 4 (the dots lambda below)
    constexpr int IT_TOPA = 2 + NSH, IT_TOPB = 3 + NSH;
    constexpr int IT_K0 = NSH <= 3 ? 7 : 8;
    if (A.fault && blockIdx.x == gridDim.x - 1) return;  // test hook: never publishes
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const mc_run_config& cfg = A.cfg;
    const int tid = threadIdx.x;
    // (the wave index is uniform: saying so keeps the chain's scalars, its
    // draws and the whole tree walk in SGPRs and scalar branches)
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), j = tid & 63;
    const int S = P.S, D = P.D, Dsh = P.Dsh;
    const int MAXJ = cfg.max_tree_depth;
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

    // ---- the slice block, scalar terms and arenas in LDS ------------------------
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
    __syncthreads();  // (the only workgroup barrier: waves are independent chains)
    if (!live) return;  // every slice of a dead chain slot returns here
    float* fa = smem + P.sdata_floats + sterm_floats + (int64_t)wave * nuts_sl_first_floats(RS, MAXJ);
    float* sa = smem + P.sdata_floats + sterm_floats + (int64_t)NW * nuts_sl_first_floats(RS, MAXJ) +
                (int64_t)wave * nuts_sl_shared_rows(MAXJ) * 4;
    // first-leaf arena: slot s, component comp (0 q, 1 r), register slot r
    auto first_at = [&](int s, int comp, int r) -> float* {
        return fa + ((s * 2 + comp) * RS + r) * 64 + j;
    };
    // the global candidate pool of this (chain, slice): slot f, comp (0 q, 1 g)
    float* pl = pool + (((grp * NW + wave) * (int64_t)S + slice) * nuts_sl_pool_floats(RS, MAXJ));
    auto pool_at = [&](int f, int comp, int r) -> float* {
        return pl + ((f * 2 + comp) * RS + r) * 64 + j;
    };

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
    const int nsl = CF ? NSH : Dsh;  // shared slots
    auto ord_of = [&](int k) {
        int o = F.d_ks;
        o = (DM && k == kdm) ? F.d_km : o;
        o = (SWS && k == ksw) ? F.sw_ks : o;
        return CF ? o : k;
    };
    // lane k < nsl holds shared slot k of the chain
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
    // (uniform constants pinned in VGPRs with two waves per SIMD — a spilled
    // SGPR costs a readlane per use; with four the VGPRs are the scarcer)
    auto pin = [](float x) { return OCC <= 2 ? vpin(x) : x; };
    const float o_m = pin(own.m), o_cinv2 = pin(own.cinv2), o_c0l = pin(own.c0l),
                o_wn = pin(own.wn);

    int gk[RS];
    const float* xv[RS];
    int len[RS], lmin4[RS], lmax[RS];
    float cnt[RS];
    bool pdir[RS];
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
        int m = len[r];
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) m = max(m, __shfl_xor(m, o));
        lmax[r] = __builtin_amdgcn_readfirstlane(m);
        pdir[r] = DIR && r < tt[nsweep].nslot &&
                  ((const int32_t*)sd)[tt[nsweep].len_off + r * 64 + j] > 0;
    }
    const float sw_w = pin(F.sw_w), sw_c0 = pin(F.sw_c0), sw_cinv = pin(F.sw_cinv),
                sw_cinv2 = pin(F.sw_cinv2), sw_clogs = pin(F.sw_clogs);
    const float d_w = pin(F.d_w), d_c0 = pin(F.d_c0), d_m = pin(F.d_m), d_cinv = pin(F.d_cinv),
                d_cinv2 = pin(F.d_cinv2), d_clogs = pin(F.d_clogs);
    const float lp_const = P.lp_const;

    // the current sample (theta0 of the next iteration): its private part
    // stays in the chain state (st_q / st_g: only this lane reads or writes
    // these entries — the top-level accept copies the candidate there), the
    // shared part in the holder lanes (every slice needs it)
    float Cqs = xon ? st_q[c * D + xg] : 1.0f, Cgs = xon ? st_g[c * D + xg] : 0.0f;

    // exchange lines: one record of kNslLine granules per (wave, slice, parity)
    // (line of parity par: + par * pstride granules; an array of the two
    // pointers indexed by the parity went to scratch)
    unsigned long long* const gline0 = xch + ((int64_t)grp * NW + wave) * S * kNslLine;
    const int64_t pstride = (int64_t)n_groups * NW * S * kNslLine;
    // poll lanes: CW-lane column groups, lane (row, col) reads pair
    // (64 / CW) pass + row of slice col
    const int CW = S > 8 ? 16 : 8;
    const int IP = 64 / CW;
    const int prow = j / CW, pcol = j % CW;
    const bool poll_lane = pcol < S;
    unsigned long long* const gp0 = gline0 + min(pcol, S - 1) * kNslLine + prow;
    // publishing (lf_rs8's reduce-scatter): lane 16 r + x (x < 2 NG) holds
    // pair 8 (x / 2) + 4 (x % 2) + perm[r] in xr[x]
    const int row16 = j >> 4, col16 = j & 15;
    const int pub_pair = 8 * (col16 >> 1) + 4 * (col16 & 1) + lf_row(row16);
    // a record item's total after the slice sums (P uniform)
    auto item_lane = [&](int Pi) { return (Pi % IP) * CW; };

    mc_chain_scalars sc = scal[c];
    float lp = sc.logp;
    double eps = sc.step_size;
    const uint32_t chain_id = (uint32_t)(cfg.chain_offset + c);
    const int64_t it_end = cfg.iter_begin + cfg.iter_count;
    int64_t n_grad = 0;
    uint32_t epoch = ebase;  // tags continue across launches (api.hip ws_reserve)
    bool ok = true;
    MC_STAMP_INIT
    // XL: the block's slices share an XCD (sliced.h xcd_announce / xcd_agree;
    // slots: the check area after both parities' lines, 16 granules apart)
    unsigned long long* const xslots = xch + 2 * pstride + (int64_t)grp * S * 16;
    XcdPoll xpoll = {0ull};
    if (XL && cfg.iter_count > 0)
        xpoll = xcd_announce(xslots, S, slice, ebase + 1, wave == 0 && j == 0);

    for (int64_t it = cfg.iter_begin; it < it_end && ok; ++it) {
        MC_STAMP_DECL
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
        if (it == cfg.num_warmup) {  // nuts.py:318-319, 328-330
            if (cfg.adapt_step_size) eps = sc.step_size_bar;
            sc.warmup_accept = sc.n_accept;
            sc.warmup_total = sc.n_total;
            sc.warmup_depth_sum = sc.depth_sum;
            sc.n_accept = 0;
            sc.n_total = 0;
            sc.depth_sum = 0;
        }
        const bool warm = it < cfg.num_warmup;
        const double eps_used = eps;
        // momentum (nuts.py:223-231): parameter g takes normal g % 4 of Philox
        // block g / 4 (k_nuts' mapping)
        auto normal_of = [&](int gi) {
            const mc_u32x4 rr = mc_draw(cfg.seed, chain_id, (uint32_t)it, MC_RNG_TAG_MOMENTUM, 0,
                                        (uint32_t)(gi >> 2));
            float z0, z1;
            if ((gi & 3) < 2) mc_box_muller(rr.x, rr.y, &z0, &z1);
            else mc_box_muller(rr.z, rr.w, &z0, &z1);
            return (gi & 1) ? z1 : z0;
        };
        // the trajectory ends (private: registers; shared: lane k)
        float Mq[RS], Mp[RS], Mg[RS], Pq[RS], Pp[RS], Pg[RS];
        float k0p = 0.0f;
#pragma unroll
        for (int r = 0; r < RS; ++r) {
            const float z = gk[r] >= 0 ? normal_of(gk[r]) : 0.0f;
            const float cq = gk[r] >= 0 ? st_q[c * D + gk[r]] : 0.0f;
            const float cg = gk[r] >= 0 ? st_g[c * D + gk[r]] : 0.0f;
            Mq[r] = Pq[r] = cq;
            Mg[r] = Pg[r] = cg;
            Mp[r] = Pp[r] = z;
            if (lead) k0p += z * z;
        }
        float Mqs = Cqs, Mgs = Cgs, Pqs = Cqs, Pgs = Cgs, Mps, Pps;
        {
            const float z = xon ? normal_of(xg) : 0.0f;
            Mps = Pps = z;
        }
        float k0s = 0.0f;  // the shared parameters' part, in slot order
        {
            const float p2 = Mps * Mps;
            for (int k = 0; k < nsl; ++k) k0s += rl(p2, k);
        }
        const mc_u32x4 rsl = mc_draw(cfg.seed, chain_id, (uint32_t)it, MC_RNG_TAG_SLICE, 0, 0);
        float H0 = 0.0f;
        double logu = 0.0;
        bool first_leaf = true;  // H0 and the slice variable come with its record

        int n = 1;
        bool s = true;
        int jd = 0;
        double alpha_sum = 0.0;
        int n_alpha = 0, leaves = 0, divergent = 0;
        // the working end (the end the current subtree extends)
        float q[RS], p[RS], g[RS];
        LrShared sh;
        sh.is = sh.iv = 1.0f;
        sh.lg = 0.0f;
        sh.v = 1.0f;
        // the next leaf's speculated private half-step momentum / position and
        // moment sums (valid when spec)
        bool spec = false;
        float sq_[RS], sp_[RS], M1[RS], M2[RS];
#pragma unroll
        for (int r = 0; r < RS; ++r) sq_[r] = sp_[r] = M1[r] = M2[r] = 0.0f;
        MC_STAMP(14);

        while (s && jd < MAXJ && ok) {
            const mc_u32x4 rd = mc_draw(cfg.seed, chain_id, (uint32_t)it, MC_RNG_TAG_DEPTH,
                                        (uint32_t)jd, 0);
            const int v = (mc_u01_f32(rd.x) < 0.5f) ? 1 : -1;
            const double ve = (double)v * eps;
            const float h = (float)(0.5 * ve), e = (float)ve;
            const float xh = pin(h), xe = pin(e);
#pragma unroll
            for (int r = 0; r < RS; ++r) {
                q[r] = v > 0 ? Pq[r] : Mq[r];
                p[r] = v > 0 ? Pp[r] : Mp[r];
                g[r] = v > 0 ? Pg[r] : Mg[r];
            }
            sh.q = v > 0 ? Pqs : Mqs;
            sh.p = v > 0 ? Pps : Mps;
            sh.g = v > 0 ? Pgs : Mgs;

            // ---- build_tree(jd) iteratively (nuts.h) ------------------------
            uint32_t freemask = (1u << (MAXJ + 2)) - 1u;
            bool s_sub = true;
            int cand = -1, cn = 0;
            float pool_lp = 0.0f;          // lane f: log p of pool slot f
            int pend_idx = 0, pend_n = 0;  // lane l: the parked first half of level l
            bool top_ok = false;
            const int nleaf = 1 << jd;
            for (int k = 0; k < nleaf; ++k) {
                MC_STAMP_DECL
                // an odd leaf's level-0 dots read leaf k - 1's (q, r), parked
                // one leaf ago: read ahead here, the LDS latency off the path
                // to the publish (k_nuts_lr's read-ahead)
                float aq0[RS], ar0[RS];
                if (k & 1) {
                    const int s0 = (k == 1) ? jd : ctz_u32((uint32_t)(k - 1));
#pragma unroll
                    for (int r = 0; r < RS; ++r) {
                        aq0[r] = *first_at(s0, 0, r);
                        ar0[r] = *first_at(s0, 1, r);
                    }
                }
                // leaf: leapfrog_step(theta, r, v * eps) (nuts.py:160-161)
                if (spec) {
#pragma unroll
                    for (int r = 0; r < RS; ++r) {
                        p[r] = sp_[r];
                        q[r] = sq_[r];
                    }
                } else {
#pragma unroll
                    for (int r = 0; r < RS; ++r) {
                        p[r] = p[r] + xh * g[r];
                        q[r] = q[r] + xe * p[r];
                    }
                }
                // the shared parameters' step (their gradient came with the
                // last record) and derived scale values
                if (xon) {
                    sh.p = sh.p + xh * sh.g;
                    sh.q = sh.q + xe * sh.p;
                }
                // the shared scales' reciprocals and logs from the hardware
                // v_rcp_f32 / v_log_f32 (<= 1 ulp; the same bits in every
                // slice), as k_hmc_lf: the IEEE division and ocml logf were a
                // dependent chain of ~40 instructions on the leaf's critical path
                sh.v = hxf ? xf_apply(xxf, sh.q) : sh.q;
                sh.is = __builtin_amdgcn_rcpf(sh.v);
                sh.iv = sh.is * sh.is;
                sh.lg = __builtin_amdgcn_logf(sh.v) * 0.693147180559945f;
                if (!spec) {
#pragma unroll
                    for (int r = 0; r < RS; ++r) {
                        M1[r] = M2[r] = 0.0f;
                        if (len[r] > 0) nsl_moments<OCC >= 4 ? 2 : 4>(xv[r], len[r], lmin4[r], lmax[r], q[r], M1[r], M2[r]);
                    }
                }
                MC_STAMP(0);
                // finish the swept term, evaluate the direct term (k_hmc_lf's
                // arithmetic for one chain): log p partial, private gradients,
                // shared cotangent partials by role
                float lpp = 0.0f, cs = 0.0f, cm = 0.0f, cd = 0.0f;
#pragma unroll
                for (int r = 0; r < RS; ++r) g[r] = 0.0f;
                if (SW) {
                    const float is = SWS ? rl(sh.is, ksw) : sw_cinv;
                    const float iv = SWS ? is * is : sw_cinv2;
                    const float lg = SWS ? rl(sh.lg, ksw) : sw_clogs;
#pragma unroll
                    for (int r = 0; r < RS; ++r) {
                        if (len[r] == 0) continue;
                        g[r] = sw_w * (M1[r] * iv);
                        cs += sw_w * ((M2[r] * iv - cnt[r]) * is);
                        lpp += sw_w * (cnt[r] * (sw_c0 - lg) - (0.5f * M2[r]) * iv);
                    }
                }
                if (DIR) {
                    const float um = DM ? rl(sh.v, kdm) : d_m;
                    const float is = DS ? rl(sh.is, kds) : d_cinv;
                    const float iv = DS ? is * is : d_cinv2;
                    const float lg = DS ? rl(sh.lg, kds) : d_clogs;
#pragma unroll
                    for (int r = 0; r < RS; ++r) {
                        if (!pdir[r]) continue;
                        const float d = q[r] - um;
                        const float s2 = d * d;
                        const float u = d_w * (d * iv);
                        g[r] += -u;
                        cm += u;
                        cd += d_w * ((s2 * iv - 1.0f) * is);
                        lpp += d_w * (1.0f * (d_c0 - lg) - (0.5f * s2) * iv);
                    }
                }
                // the expression terms (LS_EXPR, after the swept / direct
                // terms: a program planned with LanePlan::nuts_expr), their
                // element code generated per program (jit.hip gen_lane_term,
                // one chain, element pairs packed): log p and the shared
                // cotangent partials by ordinal (the run-time form's slots)
#ifdef MC_JIT_LANES
                float gxe[kLrMaxShared] = {0.0f, 0.0f, 0.0f, 0.0f};
                if constexpr (!CF)
                    for (int t = nsweep + ndirect; t < nact; ++t)
                        if (tt[t].sig == LS_EXPR) mc_jit_lane_expr1(tt + t, sd, j, sh, lpp, gxe);
#endif
                if (rep > 1) {
#pragma unroll
                    for (int r = 0; r < RS; ++r) {
                        float a = g[r], b = 0.0f;
                        grp_sum2(a, b, rep);
                        g[r] = a;
                    }
                }
                // the own prior of the lane's shared parameter: its log p
                // enters slice 0's record, its gradient stays in the lane
                float g_own = 0.0f;
                {
                    const float vv = sh.v;
                    const float d = own.hn ? vv : vv - o_m;
                    const bool out = own.hn && !(vv >= 0.0f);
                    g_own = (out || !own.on) ? 0.0f : o_wn * -(d * o_cinv2);
                    const float lpe = out ? -__builtin_inff() : o_c0l - (0.5f * (d * d)) * o_cinv2;
                    if (own_lp) lpp += o_wn * lpe;
                    if (hxf && slice == 0 && xon) lpp += xid * sh.q;
                }
                // second half kick of the private momenta, their kinetic energy
                float kp = 0.0f;
#pragma unroll
                for (int r = 0; r < RS; ++r) {
                    p[r] = p[r] + xh * g[r];
                    if (lead) kp += p[r] * p[r];
                }
                // this leaf's slot in the candidate pool, the subtree it opens
                const int f = __builtin_ctz(freemask);
                const bool opens = (jd >= 1) && ((k & 1) == 0);
                const int fslot = (k == 0) ? jd : ctz_u32((uint32_t)k);
                // merges the leaf closes (k + 1's trailing zeros, up to jd) and
                // whether it completes the subtree
                const bool last = k == nleaf - 1;
                const int m = last ? jd : ctz_u32((uint32_t)(k + 1));
                // ---- the record: wave totals, reduce-scattered ----------------
                // dot slots: the top-level pair first when the leaf completes
                // its subtree, then one pair per merge level; slot 0 sits in
                // group 0 (IT_TOPA / IT_TOPB), slot d >= 1 in group 1 + (d-1)/4
                // — three leaves in four then need one group
                const int nd = m + (last ? 1 : 0);
                const int NG = max(1 + (nd + 2) / 4, (NSH > 3 && first_leaf) ? 2 : 1);
                // U-turn dot partials of dot slot d (private parameters): the
                // top level (nuts.py:276, d = q+ - q- against r- and r+) or
                // merge level l (nuts.py:214, the level-(l+1) subtree's first
                // leaf against this end)
                auto dots = [&](int d, float& a, float& b) {
                    a = b = 0.0f;
                    if (d >= nd) return;
                    const int l = d - (last ? 1 : 0);
                    if (l < 0) {
#pragma unroll
                        for (int r = 0; r < RS; ++r) {
                            if (!lead) continue;
                            const float oq = v > 0 ? Mq[r] : Pq[r], op = v > 0 ? Mp[r] : Pp[r];
                            const float dd = v > 0 ? q[r] - oq : oq - q[r];
                            a += dd * (v > 0 ? op : p[r]);
                            b += dd * (v > 0 ? p[r] : op);
                        }
                        return;
                    }
                    const int k0 = k + 1 - (2 << l);
                    const int slot = (k0 == 0) ? jd : ctz_u32((uint32_t)k0);
#pragma unroll
                    for (int r = 0; r < RS; ++r) {
                        const float bq = l == 0 ? aq0[r] : *first_at(slot, 0, r);
                        const float br = l == 0 ? ar0[r] : *first_at(slot, 1, r);
                        if (!lead) continue;
                        const float dd = v > 0 ? q[r] - bq : bq - q[r];
                        a += dd * (v > 0 ? br : p[r]);
                        b += dd * (v > 0 ? p[r] : br);
                    }
                };
                float xr[8];
#pragma unroll
                for (int x = 0; x < 8; ++x) xr[x] = 0.0f;
                {
                    float vv[8], xx[2];
                    vv[0] = lpp;
                    vv[1] = kp;
#pragma unroll
                    for (int x = 2; x < 8; ++x) vv[x] = 0.0f;
                    if constexpr (CF) {
                        if (FORM & LF_SWS) vv[2 + lf_slot_sws(FORM)] = cs;
                        if (FORM & LF_DM) vv[2 + lf_slot_dm(FORM)] = cm;
                        if (FORM & LF_DS) vv[2 + lf_slot_ds(FORM)] = cd;
                    } else {
#pragma unroll
                        for (int kk = 0; kk < NSH; ++kk)
                        {
                            vv[2 + kk] = ((F.sw_ks == kk ? cs : 0.0f) + (F.d_km == kk ? cm : 0.0f)) +
                                         (F.d_ks == kk ? cd : 0.0f);
#ifdef MC_JIT_LANES
                            vv[2 + kk] += gxe[kk];
#endif
                        }
                    }
                    dots(0, vv[IT_TOPA], vv[IT_TOPB]);
                    if (IT_K0 < 8 && first_leaf) vv[IT_K0 & 7] = k0p;
                    lf_rs8(vv, xx);
                    xr[0] = xx[0];
                    xr[1] = xx[1];
                }
#pragma unroll
                for (int gd = 1; gd < 4; ++gd) {
                    if (gd >= NG) break;
                    float vv[8], xx[2];
#pragma unroll
                    for (int i = 0; i < 4; ++i) dots(4 * (gd - 1) + i + 1, vv[2 * i], vv[2 * i + 1]);
                    if (IT_K0 >= 8 && gd == 1 && first_leaf) vv[0] = k0p;
                    lf_rs8(vv, xx);
                    xr[2 * gd] = xx[0];
                    xr[2 * gd + 1] = xx[1];
                }
                MC_STAMP(1);
                // publish: one store instruction
                ++epoch;
                const int par = epoch & 1;
                if (col16 < 2 * NG) {
                    float pv = xr[0];
#pragma unroll
                    for (int x = 1; x < 8; ++x) pv = (x == col16) ? xr[x] : pv;
                    granule_put(gline0 + par * pstride + slice * kNslLine + pub_pair, epoch, pv, XL);
                }
                // park the leaf's private part: candidate pool (q, g) and, when
                // it opens a subtree, that subtree's first leaf (q, r)
#pragma unroll
                for (int r = 0; r < RS; ++r) {
                    *pool_at(f, 0, r) = q[r];
                    *pool_at(f, 1, r) = g[r];
                    if (opens) {
                        *first_at(fslot, 0, r) = q[r];
                        *first_at(fslot, 1, r) = p[r];
                    }
                }
                MC_STAMP(2);
                // ---- sweep-ahead: the next leaf, if the walk goes on ----------
                __builtin_amdgcn_s_setprio(1);
                spec = false;
                {
                    int nv = v;  // the next leaf's direction
                    bool go = true;
                    if (last) {
                        go = jd + 1 < MAXJ;
                        if (go) {
                            const mc_u32x4 rn = mc_draw(cfg.seed, chain_id, (uint32_t)it,
                                                        MC_RNG_TAG_DEPTH, (uint32_t)(jd + 1), 0);
                            nv = (mc_u01_f32(rn.x) < 0.5f) ? 1 : -1;
                        }
                    }
                    if (go) {
#pragma unroll
                        for (int r = 0; r < RS; ++r) {
                            // from this end, or (a new subtree the other way)
                            // from the other end with -h, -e
                            const bool same = nv == v;
                            const float bq = same ? q[r] : (v > 0 ? Mq[r] : Pq[r]);
                            const float bp = same ? p[r] : (v > 0 ? Mp[r] : Pp[r]);
                            const float bg = same ? g[r] : (v > 0 ? Mg[r] : Pg[r]);
                            const float hh = same ? xh : -xh, ee = same ? xe : -xe;
                            sp_[r] = bp + hh * bg;
                            sq_[r] = bq + ee * sp_[r];
                            M1[r] = M2[r] = 0.0f;
                            // (4 float4 groups in flight at every occupancy: the
                            // sweep-ahead is the lone chain's critical path at the
                            // launch's tail, where its wave is alone on its SIMD)
                            if (len[r] > 0)
                                nsl_moments<4>(xv[r], len[r], lmin4[r], lmax[r], sq_[r], M1[r],
                                               M2[r]);
                        }
                        spec = true;
                    }
                }
                MC_STAMP(8);
                // ---- poll: every slice's record of this leaf --------------------
                // (in chunks of 4 passes, one round trip each: 2 groups with
                // 16 slices, 4 with 8 — the records of leaves with up to 4
                // merges; the registers of 8 passes spilled at 4 waves per SIMD)
                const int npass = (8 * NG) / IP;
                unsigned long long* const gpp = gp0 + par * pstride;
                float mdraw = 0.0f;
                float tot[8];
#pragma unroll
                for (int ch = 0; ch < 2; ++ch) {
                    if (4 * ch >= npass) {
#pragma unroll
                        for (int ps = 0; ps < 4; ++ps) tot[4 * ch + ps] = 0.0f;
                        continue;
                    }
                    unsigned long long y[4];
                    auto poll_issue = [&]() {
#pragma unroll
                        for (int ps = 0; ps < 4; ++ps)
                            y[ps] = 4 * ch + ps < npass ? granule_load(gpp + IP * (4 * ch + ps)) : 0ull;
                    };
                    auto poll_eval = [&]() {
                        bool ready = true;
#pragma unroll
                        for (int ps = 0; ps < 4; ++ps) {
                            const bool nd = poll_lane && 4 * ch + ps < npass;
                            tot[4 * ch + ps] = nd ? __uint_as_float((uint32_t)y[ps]) : 0.0f;
                            ready = ready & (!nd | ((uint32_t)(y[ps] >> 32) == epoch));
                        }
                        return ready;
                    };
                    poll_issue();
                    if (ch == 0) {
                        // while the records travel: the uniforms of this leaf's
                        // merges (TAG_MERGE / jd, level << 20 | k; lane l holds
                        // level l's), scalar Philox off the critical path
                        for (int l = 0; l < m; ++l) {
                            const mc_u32x4 rm = mc_draw(cfg.seed, chain_id, (uint32_t)it,
                                                        MC_RNG_TAG_MERGE, (uint32_t)jd,
                                                        ((uint32_t)l << 20) | (uint32_t)k);
                            const float u = mc_u01_f32(rm.x);
                            mdraw = (j == l) ? u : mdraw;
                        }
                    }
                    bool ready = poll_eval();
                    uint32_t spins = 0;
                    while (__ballot(!ready)) {
                        if (++spins > kSpinLimit) {
                            ok = false;
                            break;
                        }
                        poll_issue();
                        ready = poll_eval();
                    }
                    if (!ok) break;
                }
                __builtin_amdgcn_s_setprio(0);
                if (!ok) {
                    __hip_atomic_store(status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
                MC_STAMP(3);
                // slice sums: a fixed CW-lane DPP tree per pass
#pragma unroll
                for (int ps = 0; ps < 8; ++ps) tot[ps] = ps < npass ? nsl_colsum(tot[ps], CW) : 0.0f;
                // the record's totals into one register, lane P holding item P
                // (an item read by a run-time index then is one readlane; a
                // select over the pass registers became a scratch array)
                float rec = 0.0f;
#pragma unroll
                for (int ps = 0; ps < 8; ++ps) {
                    if (ps >= npass) break;
                    const float v = __shfl(tot[ps], item_lane(j));
                    rec = (j / IP == ps) ? v : rec;
                }
                auto item = [&](int Pi) { return rl(rec, Pi); };
                const float lpl = item(0) + lp_const;
                // the shared parameters' gradient (cotangent total + own prior,
                // through the transform's VJP) and second half kick
                {
                    float gx = 0.0f;
#pragma unroll
                    for (int kk = 0; kk < NSH; ++kk) {
                        const float t = item(2 + kk);
                        gx = (xk == kk) ? t : gx;
                    }
                    float gt = gx + g_own;
                    if (hxf) gt = xf_chain(xxf, gt, sh.q, sh.v) + xid;
                    sh.g = xon ? gt : 0.0f;
                    if (xon) sh.p = sh.p + xh * sh.g;
                }
                float Ksh = 0.0f;
                {
                    const float p2 = sh.p * sh.p;
                    for (int kk = 0; kk < nsl; ++kk) Ksh += rl(p2, kk);
                }
                const float Kl = item(1) + Ksh;
                if (first_leaf) {
                    // H0 and the slice variable (nuts.py:231-237)
                    const float K0 = item(IT_K0) + k0s;
                    H0 = -lp + 0.5f * K0;
                    const double log_u = (double)(-H0) + (double)mc_logf_u01(mc_u01_f32(rsl.x));
                    if (cfg.slice_mode == 0) {
                        const float x = (float)log_u;
                        const double ed = exp((double)x);
                        float uf;
                        if (ed < 1.1754943508222875e-38) {  // f32 gradual underflow
                            uf = (float)(rint(ed * 7.1362384635297994e+44) * 1.4012984643248171e-45);
                        } else {
                            uf = (float)ed;
                        }
                        logu = (uf == 0.0f) ? -__builtin_inf() : (double)mc_logf_ref(uf);
                    } else {
                        logu = log_u;
                    }
                    first_leaf = false;
                }
                const float Hl = -lpl + 0.5f * Kl;
                ++leaves;
                const int n_leaf = (logu <= (double)(-Hl)) ? 1 : 0;
                const bool s_leaf = logu < (double)(1000.0f - Hl);
                {
                    // alpha = min(1, f32 exp(H0 - H')) (nuts.py:173; NaN -> 1, Q8) with
                    // ocml's f32 exp (<= 1 ulp from the correctly rounded value
                    // mc_expf_ref gives; the oracle replay's alpha bar is the
                    // tie bound's relative error, >> 1 ulp) — a double exp per
                    // leaf held ~20 VGPRs of f64 coefficients and spilled them
                    const float a = expf(-Hl + H0);
                    alpha_sum += (double)((a < 1.0f) ? a : 1.0f);
                }
                n_alpha += 1;
                if (!s_leaf) divergent += 1;
                // the shared part of the parked leaf
                if (xon) {
                    const int pr = 2 * MAXJ + 2 * f;
                    sa[pr * 4 + xk] = sh.q;
                    sa[(pr + 1) * 4 + xk] = sh.g;
                    if (opens) {
                        sa[(2 * fslot) * 4 + xk] = sh.q;
                        sa[(2 * fslot + 1) * 4 + xk] = sh.p;
                    }
                }
                freemask &= ~(1u << f);
                pool_lp = (j == f) ? lpl : pool_lp;
                MC_STAMP(10);
                if (!s_leaf) {
                    s_sub = false;
                    break;
                }
                cand = f;
                cn = n_leaf;
                // merge completed subtrees upward (nuts.py:200-216)
                for (int l = 0; l < m; ++l) {
                    const int pidx = __builtin_amdgcn_readlane(pend_idx, l);
                    const int pn = __builtin_amdgcn_readlane(pend_n, l);
                    const double den = (double)(pn + cn) > 1.0 ? (double)(pn + cn) : 1.0;
                    // U < cn / den as U * den < cn (exact, nuts.h)
                    const bool take_second = (double)rl(mdraw, l) * den < (double)cn;
                    if (take_second) {
                        freemask |= (1u << pidx);
                    } else {
                        freemask |= (1u << cand);
                        cand = pidx;
                    }
                    cn = pn + cn;
                    // U-turn over the merged level-(l+1) subtree: the exchanged
                    // private dots plus the shared parameters' part
                    const int k0 = k + 1 - (2 << l);
                    const int slot = (k0 == 0) ? jd : ctz_u32((uint32_t)k0);
                    float as = 0.0f, bs = 0.0f;
                    if (xon) {
                        const float bq = sa[(2 * slot) * 4 + xk], br = sa[(2 * slot + 1) * 4 + xk];
                        const float d = v > 0 ? sh.q - bq : bq - sh.q;
                        as = d * (v > 0 ? br : sh.p);
                        bs = d * (v > 0 ? sh.p : br);
                    }
                    float ash = 0.0f, bsh = 0.0f;
                    for (int kk = 0; kk < nsl; ++kk) {
                        ash += rl(as, kk);
                        bsh += rl(bs, kk);
                    }
                    const int dsl = l + (last ? 1 : 0);  // its dot slot
                    const int ia = dsl == 0 ? IT_TOPA : 8 + 2 * (dsl - 1);
                    const int ib = dsl == 0 ? IT_TOPB : ia + 1;
                    const float da = item(ia) + ash, db = item(ib) + bsh;
                    if (!(da >= 0.0f && db >= 0.0f)) {
                        s_sub = false;
                        break;
                    }
                }
                MC_STAMP(12);
                if (!s_sub) break;
                if (m < jd) {  // park the completed level-m subtree as a first half
                    pend_idx = (j == m) ? cand : pend_idx;
                    pend_n = (j == m) ? cn : pend_n;
                } else if (last) {
                    // the depth-jd subtree is complete: the top-level test's dots
                    float as = 0.0f, bs = 0.0f;
                    if (xon) {
                        const float oq = v > 0 ? Mqs : Pqs, op = v > 0 ? Mps : Pps;
                        const float d = v > 0 ? sh.q - oq : oq - sh.q;
                        as = d * (v > 0 ? op : sh.p);
                        bs = d * (v > 0 ? sh.p : op);
                    }
                    float ash = 0.0f, bsh = 0.0f;
                    for (int kk = 0; kk < nsl; ++kk) {
                        ash += rl(as, kk);
                        bsh += rl(bs, kk);
                    }
                    const float da = item(IT_TOPA) + ash, db = item(IT_TOPB) + bsh;
                    top_ok = da >= 0.0f && db >= 0.0f;
                }
            }
            if (!ok) break;
            // the extended end back from the working registers
#pragma unroll
            for (int r = 0; r < RS; ++r) {
                if (v > 0) {
                    Pq[r] = q[r];
                    Pp[r] = p[r];
                    Pg[r] = g[r];
                } else {
                    Mq[r] = q[r];
                    Mp[r] = p[r];
                    Mg[r] = g[r];
                }
            }
            if (v > 0) {
                Pqs = sh.q;
                Pps = sh.p;
                Pgs = sh.g;
            } else {
                Mqs = sh.q;
                Mps = sh.p;
                Mgs = sh.g;
            }
            // ---- top level (nuts.py:262-284) ----------------------------------
            if (s_sub) {
                const double den = (double)n > 1.0 ? (double)n : 1.0;
                if ((double)mc_u01_f32(rd.y) * den < (double)cn) {
#pragma unroll
                    for (int r = 0; r < RS; ++r) {
                        const float cq = *pool_at(cand, 0, r), cg = *pool_at(cand, 1, r);
                        if (gk[r] >= 0 && lead) {
                            st_q[c * D + gk[r]] = cq;
                            st_g[c * D + gk[r]] = cg;
                        }
                    }
                    if (xon) {
                        const int pr = 2 * MAXJ + 2 * cand;
                        Cqs = sa[pr * 4 + xk];
                        Cgs = sa[(pr + 1) * 4 + xk];
                    }
                    lp = rl(pool_lp, cand);
                }
            }
            n += cn;
            s = s_sub && top_ok;
            if (!s) spec = false;  // (the speculated leaf belongs to a walk that stopped)
            jd += 1;
            MC_STAMP(13);
        }
        if (!ok) break;

        const double alpha = alpha_sum / (n_alpha > 1 ? (double)n_alpha : 1.0);
        n_grad += leaves;
        sc.n_divergent += divergent;
        sc.alpha_sum += alpha;
        sc.n_accept += (alpha > 0.5) ? 1 : 0;
        sc.n_total += 1;
        sc.depth_sum += jd;
        if (warm && cfg.adapt_step_size) {  // dual averaging, nuts.py:299-310
            const double mm = (double)it;
            const double eta = 1.0 / (mm + 10.0);
            sc.h_bar = (1.0 - eta) * sc.h_bar + eta * (cfg.target_accept - alpha);
            const float lf = sc.mu - (float)(sqrt(mm + 1.0) / 0.05 * sc.h_bar);
            double le = (double)lf;
            if (10.0 < le) le = 10.0;
            if (-10.0 > le) le = -10.0;
            eps = (double)mc_expf_ref((float)le);
            const double m_eta = pow(mm + 1.0, -0.75);
            const double lb = m_eta * log(eps) + (1.0 - m_eta) * log(sc.step_size_bar);
            sc.step_size_bar = (double)mc_expf_ref((float)lb);
        }
        if (!warm && samples != nullptr) {
            const int64_t si = it - cfg.num_warmup - cfg.sample_begin;
            if (si >= 0 && si < cfg.sample_capacity) {
                float* out = samples + (c * cfg.sample_capacity + si) * (int64_t)D;
#pragma unroll
                for (int r = 0; r < RS; ++r)
                    if (gk[r] >= 0 && lead) out[gk[r]] = st_q[c * D + gk[r]];
                if (slice == 0 && xon) out[xg] = Cqs;
            }
        }
        if (slice == 0 && j == 0) {
            const int64_t ti = it - tr.iter_begin;
            if (ti >= 0 && ti < tr.capacity) {
                const int64_t o = c * tr.capacity + ti;
                if (tr.accepted) tr.accepted[o] = (alpha > 0.5) ? 1 : 0;
                if (tr.accept_stat) tr.accept_stat[o] = (float)alpha;
                if (tr.step_size) tr.step_size[o] = eps_used;
                if (tr.energy) tr.energy[o] = H0;
                if (tr.tree_depth) tr.tree_depth[o] = jd;
                if (tr.n_leapfrog) tr.n_leapfrog[o] = leaves;
            }
        }
        MC_STAMP(15);
    }
    MC_STAMP_FLUSH
    // a timed-out chain's state is undefined: its scalars, lp and shared
    // parameters stay as the launch found them, while an accept at a completed
    // level has already written its private parameters (st_q / st_g), so they
    // may belong to a later draw.  mc_workspace_status reports the timeout and
    // the caller re-initialises the chains (include/mcmc355.h).
    if (!ok) return;

    if (slice == 0 && xon) {
        st_q[c * D + xg] = Cqs;
        st_g[c * D + xg] = Cgs;
    }
    if (slice == 0 && j == 0) {
        sc.logp = lp;
        sc.step_size = eps;
        sc.n_grad += n_grad;
        scal[c] = sc;
    }
}

}  // namespace mc
