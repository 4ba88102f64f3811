// nuts_lanes.h — lane-resident NUTS (k_nuts_lr): the iterative slice-NUTS of
// k_nuts (nuts.h; reference nuts.py:16-358, same draws, same decisions rule
// by rule) on the one-slice lane-resident layout of k_hmc_lr (lanes.h, X1).
//
// One chain per wave.  Each private parameter of the program is dealt to one
// (lane, slot) and its elements are streamed by that lane from LDS (the
// planner's one-slice layout); the broadcast parameters sit in lanes 2k, 2k+1
// (lanes.h LrShared).  The lane evaluators of lanes.h advance two chains in
// packed FP32; here both halves carry the same chain (a packed instruction
// costs what a scalar one does), so every evaluator is reused unchanged.
//
//   * The trajectory ends (q, r, grad of both ends) and the current sample
//     (q, grad) are registers; a leaf is a leapfrog step from one end, one
//     lane-resident gradient evaluation (moment sweeps, per-element terms,
//     scalar terms, one wave_sum8) and a wave sum of the kinetic energy.
//   * The subtrees' first leaves (q, r) and the candidate pool (q, grad) —
//     slots picked by run-time indices — are in an LDS arena, one float per
//     (slot, component, register slot, lane): conflict-free, no global
//     memory in the tree walk.
//   * The small per-level arrays of the walk (pending candidate / count per
//     level, the pool's log p) live one entry per lane and are read with
//     readlane.
//   * U-turn tests are two dot products over the parameters (lane partials +
//     one DPP wave sum each); summation order differs from k_nuts (j-strided
//     group sums), every decision rule is the reference's.
#pragma once
#include "lanes.h"
#include "nuts.h"

namespace mc {

// LDS arena of one wave: first-leaf slots (q, r) [MAXJ + 1] and the candidate
// pool (q, g) [MAXJ + 2], each RS private values + the lane's shared value.
__host__ __device__ constexpr int64_t nuts_lr_arena_floats(int rs, int max_depth) {
    return (2 * (int64_t)(max_depth + 1) + 2 * (int64_t)(max_depth + 2)) * (rs + 1) * 64;
}
// k_nuts_lr's draw wave (PW): two buffers of 2^max_depth merge draws and 33
// flag words after the arena
__host__ __device__ constexpr int64_t nuts_lr_draw_words(int max_depth) {
    return 2 * ((int64_t)1 << max_depth) + 36;
}

// SPEC 1: every slice term has a specialised form (no LS_GENERIC term) and
// every scalar term is an own prior (the planner checks it): the generic
// per-element and scalar-term paths are compiled out, and with them their
// register demand (inlined, it spills the tree walk's state).
// SPEC 2 (register-only programs, api.hip lanes_register_only): no broadcast
// parameter, no scalar term and one slice term with at most one element per
// (lane, slot) — a data-scale term (config 5's theta_i ~ N(0, s_i)) or a
// direct term with constant loc and scale (theta_i ~ N(m, s)): the gradient
// is that term's arithmetic on per-slot registers, nothing else is compiled.
// PW (draw wave): the workgroup's second wave computes the tree merges'
// Philox draws ahead into LDS (nuts_lr_draw_words: two iteration buffers of
// 2^MAXJ words and the flags), the chain's wave reads each with one LDS
// load instead of a scalar Philox (~100 SALU) in its leaf's issue stream.
// The same draws, so the same trees.
template <int RS, int NSH, int SPEC, bool PW = false>
__global__ void __launch_bounds__(PW ? 128 : 64)
k_nuts_lr(LrCtx P, RunArgs A, mc_chain_scalars* scal, float* st_q, float* st_g, float* samples,
          TraceDev tr) {
    static_assert(NSH <= kLrMaxShared, "shared parameters");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const mc_run_config& cfg = A.cfg;
    const int j = threadIdx.x & 63;  // lane
    // (PW: wave 1 is the draw wave)
    const int wv = PW ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0;
    const int64_t c = blockIdx.x;
    if (c >= cfg.num_chains) return;
    constexpr bool REG = SPEC == 2;
    const int D = P.D, Dsh = REG ? 0 : P.Dsh;
    const int MAXJ = cfg.max_tree_depth;

    // ---- the one slice's block and the scalar terms into LDS --------------------
    float* sd = smem;
    const int64_t* blk = P.blocks;
    const int64_t doff = blk[0];
    const int dlen = (int)blk[1];
    const int nact = (int)blk[2];
    const int nsweep = (int)(blk[3] & 255);
    const int ndirect = (int)((blk[3] >> 8) & 255);
    const int nfast = nsweep + ndirect;
    if (wv == 0)
        for (int i = j; 4 * i < dlen; i += 64)
            *(float4*)(sd + 4 * i) = *(const float4*)(P.data + doff + 4 * i);
    LrSterm* sst = (LrSterm*)(smem + P.sdata_floats);
    const int sterm_floats = P.n_sterms * (int)(sizeof(LrSterm) / 4);
    if (wv == 0)
        for (int i = j; i < sterm_floats / 4; i += 64)
            ((float4*)sst)[i] = ((const float4*)P.sterms)[i];
    float* ar = smem + P.sdata_floats + sterm_floats;  // the arena (16-byte aligned)
    // PW: the draw buffers and flags after the arena (flags: ready[2][16]
    // (iteration + 1 whose depth-jd draws are in buffer b), then the number
    // of iterations the chain's wave has completed)
    uint32_t* dbufs = (uint32_t*)(ar + nuts_lr_arena_floats(RS, MAXJ));
    int* dflags = (int*)(dbufs + 2 * (1 << MAXJ));
    if (PW && wv == 1 && j < 33) dflags[j] = 0;
    __syncthreads();
    if constexpr (PW) {
        if (wv == 1) {  // ---- the draw wave --------------------------------------
            const uint32_t cid = (uint32_t)(cfg.chain_offset + c);
            const int64_t it0 = cfg.iter_begin, it1 = cfg.iter_begin + cfg.iter_count;
            for (int64_t it = it0; it < it1; ++it) {
                const int rel = (int)(it - it0), b = rel & 1;
                // buffer b was iteration rel - 2's: wait until the chain's wave
                // has completed it
                while (__hip_atomic_load(dflags + 32, __ATOMIC_ACQUIRE,
                                         __HIP_MEMORY_SCOPE_WORKGROUP) < rel - 1)
                    __builtin_amdgcn_s_sleep(2);
                uint32_t* buf = dbufs + b * (1 << MAXJ);
                for (int jd = 1; jd < MAXJ; ++jd) {
                    // the level-l merge at leaf k, (k + 1) a multiple of
                    // 2^(l+1), is word (2^jd - 1) + (2^jd - 2^(jd-l)) + m,
                    // m = (k + 1) / 2^(l+1) - 1 (the chain's wave reads it so)
                    const int cnt = (1 << jd) - 1;
                    for (int i0 = 0; i0 < cnt; i0 += 64) {
                        const int idx = i0 + j;
                        if (idx < cnt) {
                            int l = 0;
                            while (idx >= (1 << jd) - (1 << (jd - l - 1))) ++l;
                            const int m = idx - ((1 << jd) - (1 << (jd - l)));
                            const uint32_t k = (uint32_t)(((m + 1) << (l + 1)) - 1);
                            buf[cnt + idx] = mc_draw(cfg.seed, cid, (uint32_t)it, MC_RNG_TAG_MERGE,
                                                     (uint32_t)jd, ((uint32_t)l << 20) | k).x;
                        }
                    }
                    __hip_atomic_store(dflags + b * 16 + jd, rel + 1, __ATOMIC_RELEASE,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
            return;
        }
    }

    // arena addressing: slot s of kind 0 (first: q, r) or 1 (pool: q, g),
    // component comp, register slot r (RS: the shared value)
    const int nfirst = MAXJ + 1;
    auto at = [&](int kind, int s, int comp, int r) -> float* {
        const int row = kind == 0 ? 2 * s + comp : 2 * nfirst + 2 * s + comp;
        return ar + ((int64_t)row * (RS + 1) + r) * 64 + j;
    };

    const MC_CONST LrTerm* tt = cptr(P.terms);
    const LrOwn own = lr_own_prior(P.n_sterms, sst, j, Dsh);
    LrCounts<RS> KC;
#pragma unroll
    for (int t = 0; t < kLrSweep; ++t)
        if (!REG)
#pragma unroll
        for (int r = 0; r < RS; ++r) {
            KC.cs[t][r] = 0.0f;
            if (t < nsweep && r < tt[t].nslot)
                KC.cs[t][r] = (float)((const int32_t*)sd)[tt[t].len_off + r * 64 + j];
        }
#pragma unroll
    for (int t = 0; t < kLrDirect; ++t)
        if (!REG)
#pragma unroll
        for (int r = 0; r < RS; ++r) {
            KC.pd[t][r] = false;
            if (t < ndirect && r < tt[nsweep + t].nslot)
                KC.pd[t][r] = ((const int32_t*)sd)[tt[nsweep + t].len_off + r * 64 + j] > 0;
        }

    // a data-scale term with at most one element per (lane, slot) (theta_i ~
    // N(m, s_i), config 5): its per-slot constants in registers, read once per
    // launch (lr_dscale_term's arithmetic, no LDS or constant loads per leaf)
    int ddt = -1;
    float dd_iv[RS], dd_ls[RS], dd_o[RS], dd_c0l[RS];
    bool dd_on[RS];
    int dd_ppo = 0, dd_ko = SK_CONST, dd_jo = 0;
    float dd_w = 0.f, dd_c0 = 0.f, dd_cv = 0.f;
#pragma unroll
    for (int r = 0; r < RS; ++r) {
        dd_iv[r] = dd_ls[r] = dd_o[r] = dd_c0l[r] = 0.0f;
        dd_on[r] = false;
    }
    if constexpr (REG) {
        // the one term: a data-scale term (1/s^2 and log s tiles) or a direct
        // term with constant loc and scale (its reciprocals per slot)
        const MC_CONST LrTerm* T = tt;
        const int32_t* lens = (const int32_t*)sd + T->len_off;
        const bool ds = T->sig == LS_DSCALE;
        ddt = 0;
        dd_ppo = ds ? T->pp : 0;
        const int oth = 1 - dd_ppo;
        dd_ko = T->kind[oth];
        dd_w = T->weight;
        dd_c0 = T->c0;
        dd_cv = T->cval[oth];
#pragma unroll
        for (int r = 0; r < RS; ++r) {
            dd_on[r] = r < T->nslot && lens[r * 64 + j] == 1;
            if (!dd_on[r]) continue;
            const int toff = T->toff[r] + 4 * j;
            dd_ls[r] = ds ? sd[T->doff[dd_ppo] + toff] : T->clogs;
            dd_iv[r] = ds ? sd[T->doff[2] + toff] : T->cinv2;
            dd_o[r] = dd_ko == SK_DATA ? sd[T->doff[oth] + toff] : 0.0f;
            dd_c0l[r] = dd_c0 - dd_ls[r];  // (the f32 difference every leaf formed)
        }
    } else if constexpr (SPEC == 1) {
        for (int t = nfast; t < nact; ++t)
            if (tt[t].sig == LS_DSCALE) ddt = (ddt == -1) ? t : -2;
        if (ddt >= 0) {
            const MC_CONST LrTerm* T = tt + ddt;
            const int32_t* lens = (const int32_t*)sd + T->len_off;
            bool one = true;
#pragma unroll
            for (int r = 0; r < RS; ++r) {
                const int len = r < T->nslot ? lens[r * 64 + j] : 0;
                one = one && len <= 1;
                dd_on[r] = len == 1;
            }
            if (__ballot(!one) != 0) {
                ddt = -1;
            } else {
                dd_ppo = T->pp;
                const int oth = 1 - dd_ppo;
                dd_ko = T->kind[oth];
                dd_jo = T->jsh[oth];
                dd_w = T->weight;
                dd_c0 = T->c0;
                dd_cv = T->cval[oth];
#pragma unroll
                for (int r = 0; r < RS; ++r) {
                    if (!dd_on[r]) continue;
                    const int toff = T->toff[r] + 4 * j;
                    dd_ls[r] = sd[T->doff[dd_ppo] + toff];
                    dd_iv[r] = sd[T->doff[2] + toff];
                    dd_o[r] = dd_ko == SK_DATA ? sd[T->doff[oth] + toff] : 0.0f;
                }
            }
        }
    }

    // this lane's parameters: private slots gk[r]; shared k = j / 2 (both
    // lanes 2k, 2k + 1 hold it: the two packed halves are the same chain)
    int gk[RS];
#pragma unroll
    for (int r = 0; r < RS; ++r) gk[r] = P.gidx[(int64_t)r * 64 + j];
    const int xk = j >> 1;
    const bool xon = j < 2 * Dsh;
    const int rep = P.rep;                   // lanes per private parameter (lanes.h)
    const bool lead = (j & (rep - 1)) == 0;  // this lane counts its parameters
    const bool xone = xon && (j & 1) == 0;  // counts the shared parameter once in sums
    int xg = P.shl[0];
#pragma unroll
    for (int k = 1; k < kLrMaxShared; ++k) xg = (xk == k) ? P.shl[k] : xg;

    // current sample (q, grad): one chain, no packed duplicate (registers)
    float Cq[RS], Cg[RS];
#pragma unroll
    for (int r = 0; r < RS; ++r) {
        Cq[r] = gk[r] >= 0 ? st_q[c * D + gk[r]] : 0.0f;
        Cg[r] = gk[r] >= 0 ? st_g[c * D + gk[r]] : 0.0f;
    }
    float Cqs = xon ? st_q[c * D + xg] : 1.0f, Cgs = xon ? st_g[c * D + xg] : 0.0f;

    // the log density and gradient at (R.q, sh.q): R.g, sh.g; returns log p
    LrPriv<RS> R;
    LrShared sh;
    // an end (one chain) into / from the working registers (both packed halves)
    auto load_end = [&](const auto& E) {
#pragma unroll
        for (int r = 0; r < RS; ++r)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                R.q[r][h] = E.q[r];
                R.p[r][h] = E.p[r];
                R.g[r][h] = E.g[r];
            }
    };
    auto store_end = [&](auto& E) {
#pragma unroll
        for (int r = 0; r < RS; ++r) {
            E.q[r] = R.q[r][0];
            E.p[r] = R.p[r][0];
            E.g[r] = R.g[r][0];
        }
    };
    auto derive = [&]() {
        sh.v = sh.q;  // (NUTS programs carry no transformed parameter: api.hip use_nuts_lanes)
        sh.is = 1.0f / sh.q;
        sh.iv = 1.0f / (sh.q * sh.q);
        sh.lg = logf(sh.q);
    };
    // lane_lp != nullptr and no shared parameter: the log p is left as this
    // lane's partial in *lane_lp (the caller reduces it together with the
    // kinetic energy); the return value is then the part added after the sum
    auto evaluate = [&](float* lane_lp) -> float {
        MC_STAMP_DECL
        float gshp[kLrMaxShared][2];
#pragma unroll
        for (int k = 0; k < kLrMaxShared; ++k) gshp[k][0] = gshp[k][1] = 0.0f;
#pragma unroll
        for (int r = 0; r < RS; ++r) R.g[r][0] = R.g[r][1] = 0.0f;
        f2 lpp2 = {0.f, 0.f};
        if constexpr (!REG) {
            LrMoments<RS> M;
            lr_sweep<RS>(tt, nsweep, sd, j, R, M);
            lr_finish<RS>(tt, nsweep, ndirect, R, sh, M, KC, lpp2, gshp);
        }
        float lpp[2] = {lpp2[0], lpp2[1]};
        MC_STAMP(2);
        if constexpr (SPEC >= 1) {
            // (REG: the one term, whichever list the planner put it in)
            for (int t = REG ? 0 : nfast; t < (REG ? 1 : nact); ++t) {
                if (REG) {
                    // the one term, register-resident.  With one chain per
                    // wave the loc / value role of the parameter drops out:
                    // d(theta) of -(theta - o)^2 / 2s^2 and of -(o - theta)^2 /
                    // 2s^2 is the same -(theta - o) / s^2, the squares are equal
                    // bitwise, and the cotangent 0 + -(w (d iv)) never keeps the
                    // sign of a zero d — the same bits as the general form below
                    // (selects, not a branch per slot: one basic block, so the
                    // scheduler can interleave it with the leaf's other work)
                    const f2 w = f2s(dd_w), half = f2s(0.5f);
                    f2 lpd = {0.f, 0.f};
#pragma unroll
                    for (int r = 0; r < RS; ++r) {
                        const f2 th = {R.q[r][0], R.q[r][1]};
                        const f2 other = dd_ko == SK_DATA ? f2s(dd_o[r]) : f2s(dd_cv);
                        const f2 d = th - other;
                        const f2 iv = f2s(dd_iv[r]);
                        const f2 lpt = f2s(dd_c0l[r]) - (half * (d * d)) * iv;
                        const f2 lpn = lpd + w * lpt;
                        const f2 gp = (f2){0.f, 0.f} + -(w * (d * iv));
                        lpd[0] = dd_on[r] ? lpn[0] : lpd[0];
                        lpd[1] = dd_on[r] ? lpn[1] : lpd[1];
                        R.g[r][0] = dd_on[r] ? gp[0] : 0.0f;
                        R.g[r][1] = dd_on[r] ? gp[1] : 0.0f;
                    }
                    lpp[0] += lpd[0];
                    lpp[1] += lpd[1];
                    continue;
                }
                if (t == ddt) {  // the register-resident data-scale term
                    const f2 w = f2s(dd_w), c0 = f2s(dd_c0), half = f2s(0.5f);
                    const bool ko_sh = !REG && dd_ko == SK_SHARED;  // (REG: no shared)
                    const f2 uo = ko_sh
                                      ? (f2){rl(sh.q, 2 * dd_jo), rl(sh.q, 2 * dd_jo + 1)}
                                      : f2s(dd_cv);
                    f2 lpd = {0.f, 0.f}, po = {0.f, 0.f};
#pragma unroll
                    for (int r = 0; r < RS; ++r) {
                        if (!dd_on[r]) continue;
                        const f2 th = {R.q[r][0], R.q[r][1]};
                        const f2 other = dd_ko == SK_DATA ? f2s(dd_o[r]) : uo;
                        const f2 d = dd_ppo == 0 ? th - other : other - th;
                        const f2 iv = f2s(dd_iv[r]);
                        const f2 lpt = (c0 - f2s(dd_ls[r])) - (half * (d * d)) * iv;
                        lpd += w * lpt;
                        const f2 tt2 = w * (d * iv);
                        const f2 gp = (f2){0.f, 0.f} + (dd_ppo == 0 ? -tt2 : tt2);
                        po += dd_ppo == 0 ? tt2 : -tt2;
                        R.g[r][0] += gp[0];
                        R.g[r][1] += gp[1];
                    }
                    lpp[0] += lpd[0];
                    lpp[1] += lpd[1];
                    if (ko_sh) {
                        add4(gshp, dd_jo, 0, po[0]);
                        add4(gshp, dd_jo, 1, po[1]);
                    }
                    continue;
                }
                if constexpr (REG) continue;
                const MC_CONST LrTerm* T = tt + t;
                switch (T->sig) {
                    case LS_DSCALE: lr_dscale_term<RS>(T, sd, j, R, sh, lpp, gshp); break;
                    case LS_AFF: lr_affine<RS>(T, sd, j, R, sh, lpp, gshp); break;
                    case LS_DATA_PP_SH:
                        lr_normal_term<RS, SK_DATA, SK_PP, SK_SHARED>(T, sd, j, R, sh, lpp, gshp);
                        break;
                    case LS_DATA_PP_C:
                        lr_normal_term<RS, SK_DATA, SK_PP, SK_CONST>(T, sd, j, R, sh, lpp, gshp);
                        break;
                    case LS_PP_SH_SH:
                        lr_normal_term<RS, SK_PP, SK_SHARED, SK_SHARED>(T, sd, j, R, sh, lpp, gshp);
                        break;
                    case LS_PP_C_C:
                        lr_normal_term<RS, SK_PP, SK_CONST, SK_CONST>(T, sd, j, R, sh, lpp, gshp);
                        break;
                    case LS_PP_DATA_SH:
                        lr_normal_term<RS, SK_PP, SK_DATA, SK_SHARED>(T, sd, j, R, sh, lpp, gshp);
                        break;
                    default:
                        lr_normal_term<RS, SK_DATA, SK_SHARED, SK_SHARED>(T, sd, j, R, sh, lpp, gshp);
                        break;
                }
            }
        } else {
            lr_eval<RS>(tt, nfast, nact, sd, j, R, sh, lpp, gshp);
        }
        if (__builtin_expect(rep > 1, 0)) {  // a replicated parameter's gradient: its lanes' partials
#pragma unroll
            for (int r = 0; r < RS; ++r) grp_sum2(R.g[r][0], R.g[r][1], rep);
        }
        MC_STAMP(3);
        float slp[2] = {0.f, 0.f}, sg_self = 0.0f, sg_raw = 0.0f;
        if constexpr (!REG)
            lr_scalar_terms(P.n_sterms, SPEC ? 0 : P.n_sterms_generic, sst, own, sh, j, Dsh, slp,
                            sg_self, sg_raw);
        MC_STAMP(18);
        if (Dsh == 0) {  // no shared cotangents: one reduction
            sh.g = 0.0f;
            if (lane_lp != nullptr) {
                *lane_lp = lpp[0];
                return slp[0];
            }
            const float r = (wave_sum(lpp[0]) + slp[0]) + P.lp_const;
            MC_STAMP(19);
            return r;
        }
        float v8[8], t8[8];
        v8[0] = lpp[0];
        v8[1] = lpp[1];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            v8[2 + 2 * k] = gshp[k][0];
            v8[3 + 2 * k] = gshp[k][1];
        }
        wave_sum8(v8, t8);
        float g3[2] = {0.f, 0.f};
        if (NSH > 3) {
            g3[0] = wave_sum(gshp[3][0]);
            g3[1] = wave_sum(gshp[3][1]);
        }
        float gx = 0.0f;
#pragma unroll
        for (int k = 0; k < NSH; ++k) {
            const float tk = k < 3 ? ((j & 1) ? t8[3 + 2 * k] : t8[2 + 2 * k])
                                   : ((j & 1) ? g3[1] : g3[0]);
            if (xk == k) gx = tk;
        }
        sh.g = xon ? gx + sg_self : 0.0f;
        return (t8[0] + slp[0]) + P.lp_const;
    };
    // the kinetic energy of (R.p, sh.p)
    auto kinetic = [&]() {
        float k = 0.0f;
#pragma unroll
        for (int r = 0; r < RS; ++r)
            if (lead) k += R.p[r][0] * R.p[r][0];
        if (xone) k += sh.p * sh.p;
        return wave_sum(k);
    };

    MC_STAMP_INIT
    mc_chain_scalars sc = scal[c];
    float lp = sc.logp;
    double eps = sc.step_size;
    const uint32_t chain_id = (uint32_t)(cfg.chain_offset + c);
    const int64_t it_end = cfg.iter_begin + cfg.iter_count;
    int64_t n_grad = 0;
    const float lp_const = P.lp_const;

    for (int64_t it = cfg.iter_begin; it < it_end; ++it) {
        MC_STAMP_DECL
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

        // momentum, kinetic energy, H0 (nuts.py:223-231); parameter g takes
        // normal g % 4 of Philox block g / 4 (k_nuts' mapping)
        auto normal_of = [&](int gi) {
            const mc_u32x4 rr = mc_draw(cfg.seed, chain_id, (uint32_t)it, MC_RNG_TAG_MOMENTUM, 0,
                                        (uint32_t)(gi >> 2));
            float z0, z1;
            if ((gi & 3) < 2) mc_box_muller(rr.x, rr.y, &z0, &z1);
            else mc_box_muller(rr.z, rr.w, &z0, &z1);
            return (gi & 1) ? z1 : z0;
        };
        // both ends start at the current sample with the drawn momentum
        // the trajectory ends, one chain each (the working registers R carry
        // the packed duplicate)
        struct End {
            float q[RS], p[RS], g[RS];
        } EM, EP;
        float Mqs, Mrs, Mgs, Pqs, Prs, Pgs;
#pragma unroll
        for (int r = 0; r < RS; ++r) {
            const float z = gk[r] >= 0 ? normal_of(gk[r]) : 0.0f;
            EM.q[r] = EP.q[r] = Cq[r];
            EM.g[r] = EP.g[r] = Cg[r];
            EM.p[r] = EP.p[r] = z;
        }
        {
            const float z = xon ? normal_of(xg) : 0.0f;
            Mqs = Pqs = Cqs;
            Mgs = Pgs = Cgs;
            Mrs = Prs = z;
        }
        float K0;
        {
            float k = 0.0f;
#pragma unroll
            for (int r = 0; r < RS; ++r)
                if (lead) k += EM.p[r] * EM.p[r];
            if (xone) k += Mrs * Mrs;
            K0 = wave_sum(k);
        }
        const float H0 = -lp + 0.5f * K0;

        // slice variable (nuts.py:234-237)
        const mc_u32x4 rs = mc_draw(cfg.seed, chain_id, (uint32_t)it, MC_RNG_TAG_SLICE, 0, 0);
        const double log_u = (double)(-H0) + (double)mc_logf_u01(mc_u01_f32(rs.x));
        double logu;
        if (cfg.slice_mode == 0) {
            const float x = (float)log_u;
            double ed = exp((double)x);
            float uf;
            if (ed < 1.1754943508222875e-38) {  // f32 gradual underflow, round-half-even
                uf = (float)(rint(ed * 7.1362384635297994e+44) * 1.4012984643248171e-45);
            } else {
                uf = (float)ed;
            }
            logu = (uf == 0.0f) ? -__builtin_inf() : (double)mc_logf_ref(uf);
        } else {
            logu = log_u;
        }

        int n = 1;
        bool s = true;
        int jd = 0;
        MC_STAMP(14);
        double alpha_sum = 0.0;
        int n_alpha = 0;
        int leaves = 0;
        int divergent = 0;

        // dot products of the U-turn test over every parameter
        auto no_u_turn_lanes = [&](const float (&qm)[RS + 1], const float (&qp)[RS + 1],
                                   const float (&rm)[RS + 1], const float (&rp)[RS + 1]) {
            float a = 0.0f, b = 0.0f;
#pragma unroll
            for (int r = 0; r <= RS; ++r) {
                if (r == RS && !xone) break;
                if (r < RS && !lead) continue;
                const float d = qp[r] - qm[r];
                a += d * rm[r];
                b += d * rp[r];
            }
            float ab[2] = {a, b};
            wave_sum2(ab);
            return ab[0] >= 0.0f && ab[1] >= 0.0f;
        };

        while (s && jd < MAXJ) {
            const mc_u32x4 rd = mc_draw(cfg.seed, chain_id, (uint32_t)it, MC_RNG_TAG_DEPTH,
                                        (uint32_t)jd, 0);
            // PW: this depth's merge draws (the draw wave's buffer for this
            // iteration; it runs ahead, so this rarely waits)
            const uint32_t* dbuf = dbufs + ((int)(it - cfg.iter_begin) & 1) * (1 << MAXJ) +
                                   ((1 << jd) - 1);
            if constexpr (PW) {
                if (jd >= 1) {
                    const int want = (int)(it - cfg.iter_begin) + 1;
                    const int* fl = dflags + ((int)(it - cfg.iter_begin) & 1) * 16 + jd;
                    while (__hip_atomic_load(fl, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) !=
                           want)
                        __builtin_amdgcn_s_sleep(1);
                }
            }
            const int v = (mc_u01_f32(rd.x) < 0.5f) ? 1 : -1;
            const double ve = (double)v * eps;
            const float h = (float)(0.5 * ve);
            const float e = (float)ve;
            // the end this subtree extends: into the working registers
            if (v > 0) {
                load_end(EP);
                sh.q = Pqs;
                sh.p = Prs;
                sh.g = Pgs;
            } else {
                load_end(EM);
                sh.q = Mqs;
                sh.p = Mrs;
                sh.g = Mgs;
            }

            // ---- build_tree(jd) iteratively ---------------------------------
            uint32_t freemask = (1u << (MAXJ + 2)) - 1u;
            bool s_sub = true;
            int cand = -1, cn = 0;
            float pool_lp = 0.0f;  // lane f: log p of pool slot f
            int pend_idx = 0, pend_n = 0;  // lane l: the parked first half of level l
            const int nleaf = 1 << jd;
            for (int k = 0; k < nleaf; ++k) {
                // an odd leaf closes the pair (k - 1, k): the level-0 merge's
                // U-turn test reads leaf k - 1's (q, r), parked one leaf ago —
                // read ahead here, its LDS latency hidden under the leaf
                float aq0[RS + 1], ar0[RS + 1];
                if (k & 1) {
                    const int s0 = (k == 1) ? jd : ctz_u32((uint32_t)(k - 1));
#pragma unroll
                    for (int r = 0; r <= RS; ++r) {
                        const bool in = r < RS || Dsh > 0;
                        aq0[r] = in ? *at(0, s0, 0, r) : 0.0f;
                        ar0[r] = in ? *at(0, s0, 1, r) : 0.0f;
                    }
                }
                // and that merge's draw (scalar Philox: its instructions fill
                // the leaf's dependency stalls; in the merge it was on the
                // critical path)
                uint32_t u0 = 0;
                if (k & 1)
                    u0 = PW ? __builtin_amdgcn_readfirstlane(dbuf[((k + 1) >> 1) - 1])
                            : mc_draw(cfg.seed, chain_id, (uint32_t)it, MC_RNG_TAG_MERGE,
                                      (uint32_t)jd, (uint32_t)k).x;
                // leaf: leapfrog_step(theta, r, v*eps) + hamiltonian (nuts.py:160-164)
                // (both packed halves in one instruction each: the same IEEE
                // operations as the per-half form)
#pragma unroll
                for (int r = 0; r < RS; ++r) {
                    const f2 pj = (f2){R.p[r][0], R.p[r][1]} + f2s(h) * (f2){R.g[r][0], R.g[r][1]};
                    const f2 qj = (f2){R.q[r][0], R.q[r][1]} + f2s(e) * pj;
                    R.p[r][0] = pj[0];
                    R.p[r][1] = pj[1];
                    R.q[r][0] = qj[0];
                    R.q[r][1] = qj[1];
                }
                {
                    const float pj = sh.p + h * sh.g;
                    sh.p = pj;
                    sh.q = sh.q + e * pj;
                }
                if (Dsh > 0) derive();
                MC_STAMP(8);
                float lpl, Kl;
                if (Dsh == 0) {
                    // the private gradients are complete in their lanes: the
                    // half kick and the kinetic partial need no reduction, so
                    // log p and the kinetic energy are reduced side by side
                    // (two independent DPP chains, the same trees as apart)
                    float lane_lp;
                    const float post = evaluate(&lane_lp);
                    MC_STAMP(9);
                    float k = 0.0f;
#pragma unroll
                    for (int r = 0; r < RS; ++r) {
                        const f2 pj =
                            (f2){R.p[r][0], R.p[r][1]} + f2s(h) * (f2){R.g[r][0], R.g[r][1]};
                        R.p[r][0] = pj[0];
                        R.p[r][1] = pj[1];
                        if (lead) k += R.p[r][0] * R.p[r][0];
                    }
                    float ws[2] = {lane_lp, k};
                    wave_sum2(ws);
                    lpl = (ws[0] + post) + lp_const;
                    Kl = ws[1];
                } else {
                    lpl = evaluate(nullptr);
                    MC_STAMP(9);
#pragma unroll
                    for (int r = 0; r < RS; ++r)
#pragma unroll
                        for (int hh = 0; hh < 2; ++hh) R.p[r][hh] = R.p[r][hh] + h * R.g[r][hh];
                    sh.p = sh.p + h * sh.g;
                    Kl = kinetic();
                }
                const float Hl = -lpl + 0.5f * Kl;
                ++leaves;
                const int n_leaf = (logu <= (double)(-Hl)) ? 1 : 0;
                const bool s_leaf = logu < (double)(1000.0f - Hl);
                const double a = (double)mc_expf_ref(-Hl + H0);
                alpha_sum += (a < 1.0) ? a : 1.0;
                n_alpha += 1;
                if (!s_leaf) divergent += 1;
                MC_STAMP(10);

                // park the leaf as a candidate and, if it opens a subtree of
                // level >= 1, as that subtree's first leaf
                const int f = __builtin_ctz(freemask);
                freemask &= ~(1u << f);
#pragma unroll
                for (int r = 0; r < RS; ++r) {
                    *at(1, f, 0, r) = R.q[r][0];
                    *at(1, f, 1, r) = R.g[r][0];
                }
                if (Dsh > 0) {  // (no broadcast parameter: the shared slot is unused)
                    *at(1, f, 0, RS) = sh.q;
                    *at(1, f, 1, RS) = sh.g;
                }
                pool_lp = (j == f) ? lpl : pool_lp;
                const bool opens = (jd >= 1) && ((k & 1) == 0);
                if (opens) {
                    const int fslot = (k == 0) ? jd : ctz_u32((uint32_t)k);
#pragma unroll
                    for (int r = 0; r < RS; ++r) {
                        *at(0, fslot, 0, r) = R.q[r][0];
                        *at(0, fslot, 1, r) = R.p[r][0];
                    }
                    if (Dsh > 0) {
                        *at(0, fslot, 0, RS) = sh.q;
                        *at(0, fslot, 1, RS) = sh.p;
                    }
                }
                MC_STAMP(11);
                if (!s_leaf) {
                    s_sub = false;
                    break;
                }
                cand = f;
                cn = n_leaf;

                // merge completed subtrees upward
                bool parked = false;
                for (int l = 0; l < jd; ++l) {
                    if (((k + 1) >> l) & 1) {
                        pend_idx = (j == l) ? cand : pend_idx;
                        pend_n = (j == l) ? cn : pend_n;
                        parked = true;
                        break;
                    }
                    const int pidx = __builtin_amdgcn_readlane(pend_idx, l);
                    const int pn = __builtin_amdgcn_readlane(pend_n, l);
                    const uint32_t ux =
                        l == 0 ? u0
                        : PW   ? __builtin_amdgcn_readfirstlane(
                                   dbuf[((1 << jd) - (1 << (jd - l))) + ((k + 1) >> (l + 1)) - 1])
                               : mc_draw(cfg.seed, chain_id, (uint32_t)it, MC_RNG_TAG_MERGE,
                                         (uint32_t)jd, ((uint32_t)l << 20) | (uint32_t)k).x;
                    const double den = (double)(pn + cn) > 1.0 ? (double)(pn + cn) : 1.0;
                    // U < cn / den (nuts.py:205) as U * den < cn: exact in f64 (U a
                    // multiple of 2^-24, den < 2^24), the same decision as the
                    // rounded quotient (no representable U lies between the two)
                    const bool take_second = (double)mc_u01_f32(ux) * den < (double)cn;
                    if (take_second) {
                        freemask |= (1u << pidx);
                    } else {
                        freemask |= (1u << cand);
                        cand = pidx;
                    }
                    cn = pn + cn;
                    // U-turn over the merged level-(l+1) subtree
                    const int k0 = k + 1 - (2 << l);
                    const int slot = (k0 == 0) ? jd : ctz_u32((uint32_t)k0);
                    float bq[RS + 1], br[RS + 1], eq[RS + 1], er[RS + 1];
#pragma unroll
                    for (int r = 0; r <= RS; ++r) {
                        const bool in = r < RS || Dsh > 0;
                        if (l == 0) {  // (read ahead at the leaf's start)
                            bq[r] = aq0[r];
                            br[r] = ar0[r];
                        } else {
                            bq[r] = in ? *at(0, slot, 0, r) : 0.0f;
                            br[r] = in ? *at(0, slot, 1, r) : 0.0f;
                        }
                        eq[r] = r < RS ? R.q[r][0] : sh.q;
                        er[r] = r < RS ? R.p[r][0] : sh.p;
                    }
                    const bool ok = (v > 0) ? no_u_turn_lanes(bq, eq, br, er)
                                            : no_u_turn_lanes(eq, bq, er, br);
                    if (!ok) {
                        s_sub = false;
                        break;
                    }
                }
                MC_STAMP(12);
                if (!s_sub) break;
                if (parked) continue;
                // l reached jd: the depth-jd subtree is complete
            }
            // the working registers back into the end they extended
            if (v > 0) {
                store_end(EP);
                Pqs = sh.q;
                Prs = sh.p;
                Pgs = sh.g;
            } else {
                store_end(EM);
                Mqs = sh.q;
                Mrs = sh.p;
                Mgs = sh.g;
            }

            // ---- top level (nuts.py:262-284) --------------------------------
            if (s_sub) {
                const double den = (double)n > 1.0 ? (double)n : 1.0;
                // U < min(1, cn / den) (nuts.py:269-272); U < 1 always, and U < cn / den
                // as U * den < cn (exact, see the merge)
                if ((double)mc_u01_f32(rd.y) * den < (double)cn) {
#pragma unroll
                    for (int r = 0; r < RS; ++r) {
                        const float q = *at(1, cand, 0, r), g = *at(1, cand, 1, r);
                        Cq[r] = q;
                        Cg[r] = g;
                    }
                    if (Dsh > 0) {
                        Cqs = *at(1, cand, 0, RS);
                        Cgs = *at(1, cand, 1, RS);
                    }
                    lp = rl(pool_lp, cand);
                }
            }
            n += cn;
            if (s_sub) {
                float mq[RS + 1], pq[RS + 1], mr[RS + 1], pr[RS + 1];
#pragma unroll
                for (int r = 0; r < RS; ++r) {
                    mq[r] = EM.q[r];
                    pq[r] = EP.q[r];
                    mr[r] = EM.p[r];
                    pr[r] = EP.p[r];
                }
                mq[RS] = Mqs;
                pq[RS] = Pqs;
                mr[RS] = Mrs;
                pr[RS] = Prs;
                s = no_u_turn_lanes(mq, pq, mr, pr);
            } else {
                s = false;
            }
            jd += 1;
            MC_STAMP(13);
        }

        const double alpha = alpha_sum / (n_alpha > 1 ? (double)n_alpha : 1.0);
        n_grad += leaves;
        sc.n_divergent += divergent;
        sc.alpha_sum += alpha;
        sc.n_accept += (alpha > 0.5) ? 1 : 0;
        sc.n_total += 1;
        sc.depth_sum += jd;
        if (warm && cfg.adapt_step_size) {  // dual averaging, nuts.py:299-310
            const double m = (double)it;
            const double eta = 1.0 / (m + 10.0);
            sc.h_bar = (1.0 - eta) * sc.h_bar + eta * (cfg.target_accept - alpha);
            const float lf = sc.mu - (float)(sqrt(m + 1.0) / 0.05 * sc.h_bar);
            double le = (double)lf;
            if (10.0 < le) le = 10.0;
            if (-10.0 > le) le = -10.0;
            eps = (double)mc_expf_ref((float)le);
            const double m_eta = pow(m + 1.0, -0.75);
            const double lb = m_eta * log(eps) + (1.0 - m_eta) * log(sc.step_size_bar);
            sc.step_size_bar = (double)mc_expf_ref((float)lb);
        }
        if (!warm && samples != nullptr) {
            const int64_t si = it - cfg.num_warmup - cfg.sample_begin;
            if (si >= 0 && si < cfg.sample_capacity) {
                float* out = samples + (c * cfg.sample_capacity + si) * (int64_t)D;
#pragma unroll
                for (int r = 0; r < RS; ++r)
                    if (gk[r] >= 0 && lead) out[gk[r]] = Cq[r];
                if (xone) out[xg] = Cqs;
            }
        }
        if (j == 0) {
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
        if constexpr (PW)  // (the draw wave may now refill this iteration's buffer)
            __hip_atomic_store(dflags + 32, (int)(it - cfg.iter_begin) + 1, __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    MC_STAMP_FLUSH

#pragma unroll
    for (int r = 0; r < RS; ++r) {
        if (gk[r] >= 0 && lead) {
            st_q[c * D + gk[r]] = Cq[r];
            st_g[c * D + gk[r]] = Cg[r];
        }
    }
    if (xone) {
        st_q[c * D + xg] = Cqs;
        st_g[c * D + xg] = Cgs;
    }
    if (j == 0) {
        sc.logp = lp;
        sc.step_size = eps;
        sc.n_grad += n_grad;
        scal[c] = sc;
    }
}

}  // namespace mc
