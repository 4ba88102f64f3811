// mh.h — persistent random-walk Metropolis-Hastings kernel: one chain group
// per chain runs every iteration of [iter_begin, iter_begin + iter_count).
//
// Restates mlx_mcmc/kernels/metropolis.py:6-101 per chain:
//   proposal  q' = q + f32(z * f32(scale)),  z ~ N(0, I)     metropolis.py:66-74
//             (mx.random.normal(shape) * proposal_scale, then param + noise)
//   ratio     f32(lp(q') - lp(q))                            metropolis.py:77-78
//   accept    iff f32 log U < ratio (NaN -> reject)          metropolis.py:81-88
//   store     the current point after every iteration        metropolis.py:90-92
// The log density is the forward tape only (eval_lp_grad<WPC, true>): the
// proposal's log density is carried over on acceptance, so one evaluation per
// iteration, exactly the reference's count.
#pragma once
#include "eval.h"
#include "philox.h"

namespace mc {

template <int WPC, bool LDS_ARENA, bool EX>
__global__ void __launch_bounds__(WPC >= 4 ? 64 * WPC : 256)
k_mh(DevCtx P, RunArgs A, float scale, mc_chain_scalars* scal, float* st_q, float* samples,
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
    float* arena = LDS_ARENA ? (base + A.scratch_floats) : (ws + c * 2 * (int64_t)Dp);
    float* qA = arena;       // current point
    float* qB = arena + Dp;  // proposal

    float lp = scal[c].logp;
    int n_acc = scal[c].n_accept, n_tot = scal[c].n_total;
    for (int j = G.tid; j < D; j += T) qA[j] = st_q[c * D + j];
    G.sync();

    const uint32_t chain_id = (uint32_t)(cfg.chain_offset + c);
    const int64_t it_end = cfg.iter_begin + cfg.iter_count;
    for (int64_t it = cfg.iter_begin; it < it_end; ++it) {
        // Gaussian random walk: element j takes normal j % 4 of Philox block j / 4
        for (int m = G.tid; 4 * m < D; m += T) {
            const mc_u32x4 r = mc_draw(cfg.seed, chain_id, (uint32_t)it, MC_RNG_TAG_PROPOSAL, 0,
                                       (uint32_t)m);
            float z[4];
            mc_box_muller(r.x, r.y, &z[0], &z[1]);
            mc_box_muller(r.z, r.w, &z[2], &z[3]);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int j = 4 * m + k;
                if (j < D) qB[j] = qA[j] + z[k] * scale;
            }
        }
        G.sync();
        const float lpn = eval_lp_grad<WPC, true, EX>(P, qB, nullptr, G, S);
        const float ratio = lpn - lp;
        const mc_u32x4 ru = mc_draw(cfg.seed, chain_id, (uint32_t)it, MC_RNG_TAG_ACCEPT, 0, 0);
        const float logu = mc_logf_u01(mc_u01_f32(ru.x));
        const bool accepted = logu < ratio;
        if (accepted) {
            float* t = qA;
            qA = qB;
            qB = t;
            lp = lpn;
        }
        n_acc += accepted ? 1 : 0;
        n_tot += 1;
        if (samples != nullptr) {
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
                if (tr.step_size) tr.step_size[o] = (double)scale;
                if (tr.energy) tr.energy[o] = lp;
                if (tr.tree_depth) tr.tree_depth[o] = 0;
                if (tr.n_leapfrog) tr.n_leapfrog[o] = 0;
            }
        }
        G.sync();  // the next proposal overwrites the buffer just read
    }

    for (int j = G.tid; j < D; j += T) st_q[c * D + j] = qA[j];
    if (G.tid == 0) {
        mc_chain_scalars& sc = scal[c];
        sc.logp = lp;
        sc.n_accept = n_acc;
        sc.n_total = n_tot;
    }
}

}  // namespace mc
