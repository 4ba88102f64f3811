// hmc.h — persistent HMC kernel: one chain group per chain runs every
// iteration of [iter_begin, iter_begin + iter_count) on chip.
//
// Restates mlx_mcmc/kernels/hmc.py:7-206 per chain:
//   momentum ~ N(0, I)                         hmc.py:116-120
//   H_init = -log p(q) + 0.5 sum p^2           hmc.py:102-111,127
//   L leapfrog steps                           hmc.py:69-100,132-133
//     p += f32(0.5 eps) * grad; q += f32(eps) * p; p += f32(0.5 eps) * grad'
//   accept iff f32 log U < -(H_prop - H_init)  hmc.py:139-153 (NaN -> reject)
//   warmup (i > 10): eps *= 0.95 if cumulative accept rate < target else 1.05
//                                              hmc.py:159-170
//   counters reset at the warmup->sampling edge hmc.py:179-180
// Cost-only differences: the gradient at the end of a leapfrog
// step is reused as the next step's first gradient and the accepted
// proposal's log density / gradient are carried over, so an iteration costs
// L gradient evaluations instead of 2L + 2.  The arithmetic of every value
// is unchanged (two separate half kicks, no FMA contraction).
#pragma once
#include "eval.h"
#include "philox.h"

namespace mc {

template <int WPC, bool LDS_ARENA, bool EX>
__global__ void __launch_bounds__(WPC >= 4 ? 64 * WPC : 256)
k_hmc(DevCtx P, RunArgs A, mc_chain_scalars* scal, float* st_q, float* st_g, float* samples,
      TraceDev tr, float* ws) {
    constexpr int CPB = (WPC >= 4) ? 1 : 4 / WPC;
    constexpr int T = 64 * WPC;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const mc_run_config& cfg = A.cfg;
    const int lc = threadIdx.x / T;
    const int64_t c = (int64_t)blockIdx.x * CPB + lc;
    if (c >= cfg.num_chains) return;

    Group<WPC> G;
    SegScratch S;
    G.tid = threadIdx.x % T;
    float* base = smem + (int64_t)lc * A.lds_floats;
    carve_group<WPC>(base, G, S);
    const int D = P.D;
    const int Dp = A.dpad;
    float* arena = LDS_ARENA ? (base + A.scratch_floats) : (ws + c * 5 * (int64_t)Dp);
    float* qA = arena;
    float* gA = arena + Dp;
    float* qB = arena + 2 * Dp;
    float* gB = arena + 3 * Dp;
    float* p = arena + 4 * Dp;

    MC_STAMP_INIT
    float lp = scal[c].logp;
    double eps = scal[c].step_size;
    int n_acc = scal[c].n_accept, n_tot = scal[c].n_total;
    int warm_acc = scal[c].warmup_accept, warm_tot = scal[c].warmup_total;
    for (int j = G.tid; j < D; j += T) {
        qA[j] = st_q[c * D + j];
        gA[j] = st_g[c * D + j];
    }
    G.sync();

    const uint32_t chain_id = (uint32_t)(cfg.chain_offset + c);
    const int L = cfg.num_leapfrog_steps;
    const int64_t it_end = cfg.iter_begin + cfg.iter_count;
    for (int64_t it = cfg.iter_begin; it < it_end; ++it) {
        if (it == cfg.num_warmup) {  // hmc.py:175-180
            warm_acc = n_acc;
            warm_tot = n_tot;
            n_acc = 0;
            n_tot = 0;
        }
        const bool warm = it < cfg.num_warmup;
        const double eps_used = eps;
        const float h = (float)(0.5 * eps);
        const float e = (float)eps;

        // momentum: 4 normals per Philox block, element j <- index j/4
        float kp = 0.0f;
        for (int m = G.tid; 4 * m < D; m += T) {
            const mc_u32x4 r = mc_draw(cfg.seed, chain_id, (uint32_t)it, MC_RNG_TAG_MOMENTUM, 0,
                                       (uint32_t)m);
            float z[4];
            mc_box_muller(r.x, r.y, &z[0], &z[1]);
            mc_box_muller(r.z, r.w, &z[2], &z[3]);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int j = 4 * m + k;
                if (j < D) {
                    p[j] = z[k];
                    kp += z[k] * z[k];
                }
            }
        }
        const float H0 = -lp + 0.5f * G.sum(kp);
        G.sync();  // momentum written by the Philox-block mapping, read j-strided

        const float* cq = qA;
        const float* cg = gA;
        float lpn = lp;
        for (int l = 0; l < L; ++l) {
            MC_STAMP_DECL
            for (int j = G.tid; j < D; j += T) {
                const float gj = cg[j];
                float pj = p[j];
                if (l > 0) pj = pj + h * gj;  // second half kick of step l-1
                pj = pj + h * gj;             // first half kick of step l
                p[j] = pj;
                qB[j] = cq[j] + e * pj;
                gB[j] = 0.0f;  // the evaluator accumulates into a zeroed gradient
            }
            G.sync();
            MC_STAMP(0);
            lpn = eval_lp_grad<WPC, false, EX>(P, qB, gB, G, S, true);
            MC_STAMP(1);
            cq = qB;
            cg = gB;
        }
        float kp1 = 0.0f;
        for (int j = G.tid; j < D; j += T) {
            const float pj = (L > 0) ? p[j] + h * cg[j] : p[j];
            kp1 += pj * pj;
        }
        const float H1 = -lpn + 0.5f * G.sum(kp1);
        const float ratio = -(H1 - H0);
        const mc_u32x4 ru = mc_draw(cfg.seed, chain_id, (uint32_t)it, MC_RNG_TAG_ACCEPT, 0, 0);
        const float logu = mc_logf_u01(mc_u01_f32(ru.x));
        const bool accepted = logu < ratio;
        if (accepted && L > 0) {
            float* t;
            t = qA; qA = qB; qB = t;
            t = gA; gA = gB; gB = t;
            lp = lpn;
        }
        n_acc += accepted ? 1 : 0;
        n_tot += 1;
        if (warm && cfg.adapt_step_size && it > 10) {
            const double rate = (double)n_acc / (double)n_tot;
            eps = (rate < cfg.target_accept) ? eps * 0.95 : eps * 1.05;
        }
        if (!warm && samples != nullptr) {
            const int64_t s = it - cfg.num_warmup - cfg.sample_begin;
            if (s >= 0 && s < cfg.sample_capacity) {
                float* out = samples + (c * cfg.sample_capacity + s) * (int64_t)D;
                for (int j = G.tid; j < D; j += T) out[j] = qA[j];
            }
        }
        if (G.tid == 0) {
            const int64_t ti = it - tr.iter_begin;
            if (ti >= 0 && ti < tr.capacity) {
                const int64_t o = c * tr.capacity + ti;
                if (tr.accepted) tr.accepted[o] = accepted ? 1 : 0;
                if (tr.accept_stat) tr.accept_stat[o] = ratio;
                if (tr.step_size) tr.step_size[o] = eps_used;
                if (tr.energy) tr.energy[o] = H0;
                if (tr.tree_depth) tr.tree_depth[o] = L;
                if (tr.n_leapfrog) tr.n_leapfrog[o] = L;
            }
        }
        G.sync();
    }

    for (int j = G.tid; j < D; j += T) {
        st_q[c * D + j] = qA[j];
        st_g[c * D + j] = gA[j];
    }
    MC_STAMP_FLUSH
    if (G.tid == 0) {
        mc_chain_scalars& sc = scal[c];
        sc.logp = lp;
        sc.step_size = eps;
        sc.n_accept = n_acc;
        sc.n_total = n_tot;
        sc.warmup_accept = warm_acc;
        sc.warmup_total = warm_tot;
        sc.n_grad += cfg.iter_count * (int64_t)L;
    }
}

}  // namespace mc
