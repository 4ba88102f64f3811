// nuts.h — persistent slice-NUTS kernel (Hoffman & Gelman 2014, Alg. 3 with
// the reference's dual averaging), one chain group per chain.
//
// Restates mlx_mcmc/kernels/nuts.py:16-358 per chain; the recursion of
// build_tree (nuts.py:137-218) becomes an iterative post-order walk over the
// 2^j leaves of a depth-j subtree:
//   leaf k: leapfrog from the trajectory end (nuts.py:160-161), H' (:164),
//           n' = [log u <= -H'] (:166), s' = [log u < f32(1000 - H')] (:170),
//           alpha = min(1, f32 exp(H0 - H')) with Python min semantics, so a
//           NaN energy counts as alpha = 1 (:173)
//   a completed subtree at level l is a first half if bit l of (k+1) is set:
//   it is parked; a second half is merged with the parked first half:
//           keep the second half's candidate iff U < n''/max(n'+n'', 1) (:205)
//           s = s'' and no_u_turn(subtree ends)                      (:214)
//   any s = false ends the subtree at once: the reference builds no further
//   leaf after a failure (:194, :214 short-circuit), so the remaining merges
//   only touch values the caller discards.
// Top level (nuts_step, nuts.py:220-285): direction U < 0.5 -> +1 (:254),
// accept the subtree's candidate iff s' and U < min(1, n'/max(n,1)) (:269-272),
// n += n', s = s' and no_u_turn(trajectory ends) (:275-276).
// Slice (nuts.py:234-237): log u = f32(-H0) + f32 log U in double; in the
// reference mode u = f32 exp(f32 log u) with gradual underflow and then
// log u = f32 log u: u is the smallest denormal (log u ~ -103.28, SURVEY Q7's
// ~-103.3) down to ln 2^-150 ~ -103.97 and 0 below it, where the slice is off
// (log u = -inf)
// (SURVEY Q7).  Dual averaging (nuts.py:298-319) runs in-kernel.
//
// Draw addressing: momentum (TAG_MOMENTUM), slice (TAG_SLICE), per depth j
// one block TAG_DEPTH/j giving the direction (word x) and top-level accept
// (word y) uniforms, per merge TAG_MERGE/j with index (level << 20) | k.
// Each leaf costs one gradient evaluation (the reference's second gradient
// and the H0 recomputation at every leaf are cost-only).
#pragma once
#include "eval.h"
#include "philox.h"

namespace mc {

// per-chain arena (global memory), in units of Dp floats
//   [0,6)                         minus end q r g, plus end q r g
//   [6, 6 + 2(MAXJ+1))            first-leaf (q, r) of a subtree, slot = min(tz(k), j)
//   [.., + 2(MAXJ+2))             candidate pool (q, g)
__host__ __device__ constexpr int64_t nuts_arena_vectors(int max_depth) {
    return 6 + 2 * (int64_t)(max_depth + 1) + 2 * (int64_t)(max_depth + 2);
}
// LDS ints after the group scratch: pending idx / pending n / pool lp
constexpr int kNutsLdsWords = 3 * 32;

template <int WPC>
MC_DEV void vcopy(float* dst, const float* src, int D, const Group<WPC>& G) {
    for (int j = G.tid; j < D; j += Group<WPC>::T) dst[j] = src[j];
}

// reference no_u_turn (nuts.py:119-135): (q+ - q-).r- >= 0 and (q+ - q-).r+ >= 0
template <int WPC>
MC_DEV bool no_u_turn(const float* qm, const float* qp, const float* rm, const float* rp, int D,
                      const Group<WPC>& G) {
    float a = 0.0f, b = 0.0f;
    for (int j = G.tid; j < D; j += Group<WPC>::T) {
        const float d = qp[j] - qm[j];
        a += d * rm[j];
        b += d * rp[j];
    }
    const float dm = G.sum(a);
    const float dp = G.sum(b);
    return dm >= 0.0f && dp >= 0.0f;
}

MC_DEV int ctz_u32(uint32_t x) { return __builtin_ctz(x); }

// LDS_ARENA: the arena lives in the workgroup's LDS after the group scratch
// and the pending words (every trajectory vector one LDS round trip away
// instead of an L2 one); else in the global workspace.
template <int WPC, bool LDS_ARENA, bool EX>
__global__ void __launch_bounds__(WPC >= 4 ? 64 * WPC : 256)
k_nuts(DevCtx P, RunArgs A, mc_chain_scalars* scal, float* st_q, float* st_g, float* samples,
       TraceDev tr, float* ws) {
    constexpr int CPB = (WPC >= 4) ? 1 : 4 / WPC;
    constexpr int T = 64 * WPC;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const mc_run_config& cfg = A.cfg;
    const int lc = threadIdx.x / T;
    const int64_t c = (int64_t)blockIdx.x * CPB + lc;
    // the (read-only) data pool staged in LDS once per workgroup: the tape's
    // per-element operand loads become LDS reads (before any chain returns)
    DevCtx Pd = P;
    if constexpr (LDS_ARENA) {
        if (A.data_lds > 0) {
            float* dl = smem + (int64_t)CPB * A.lds_floats;
            for (int i = threadIdx.x; i < A.data_lds; i += blockDim.x) dl[i] = P.data[i];
            __syncthreads();
            Pd.data = dl;
        }
    }
    if (c >= cfg.num_chains) return;

    Group<WPC> G;
    SegScratch S;
    G.tid = threadIdx.x % T;
    float* base = smem + (int64_t)lc * A.lds_floats;
    carve_group<WPC>(base, G, S);
    int* pend_idx = reinterpret_cast<int*>(base + A.scratch_floats);
    int* pend_n = pend_idx + 32;
    float* pool_lp = reinterpret_cast<float*>(pend_idx + 64);

    const int D = P.D;
    const int64_t Dp = A.dpad;
    const int MAXJ = cfg.max_tree_depth;
    float* ar = LDS_ARENA ? (base + A.scratch_floats + kNutsLdsWords)
                          : (ws + c * nuts_arena_vectors(MAXJ) * Dp);
    float* Mq = ar;
    float* Mr = ar + Dp;
    float* Mg = ar + 2 * Dp;
    float* Pq = ar + 3 * Dp;
    float* Pr = ar + 4 * Dp;
    float* Pg = ar + 5 * Dp;
    float* first = ar + 6 * Dp;                       // slot s: q at 2s, r at 2s+1
    float* pool = first + 2 * (int64_t)(MAXJ + 1) * Dp;  // slot s: q at 2s, g at 2s+1
    float* sq = st_q + c * D;  // current sample (theta0 of the next iteration)
    float* sg = st_g + c * D;

    MC_STAMP_INIT
    mc_chain_scalars sc = scal[c];
    float lp = sc.logp;
    double eps = sc.step_size;
    const uint32_t chain_id = (uint32_t)(cfg.chain_offset + c);
    const int64_t it_end = cfg.iter_begin + cfg.iter_count;
    int64_t n_grad = 0;

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

        // momentum into the minus end, kinetic energy, H0 (nuts.py:223-231)
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
                    Mr[j] = z[k];
                    kp += z[k] * z[k];
                }
            }
        }
        const float H0 = -lp + 0.5f * G.sum(kp);
        G.sync();  // momentum written by the Philox-block mapping, read j-strided
        for (int j = G.tid; j < D; j += T) {
            const float qj = sq[j], gj = sg[j], rj = Mr[j];
            Mq[j] = qj;
            Mg[j] = gj;
            Pq[j] = qj;
            Pr[j] = rj;
            Pg[j] = gj;
        }

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
        int j = 0;
        double alpha_sum = 0.0;
        int n_alpha = 0;
        int leaves = 0;
        int divergent = 0;
        G.sync();
        MC_STAMP(14);

        while (s && j < MAXJ) {
            const mc_u32x4 rd = mc_draw(cfg.seed, chain_id, (uint32_t)it, MC_RNG_TAG_DEPTH,
                                        (uint32_t)j, 0);
            const int v = (mc_u01_f32(rd.x) < 0.5f) ? 1 : -1;
            const double ve = (double)v * eps;
            const float h = (float)(0.5 * ve);
            const float e = (float)ve;
            float* Eq = (v > 0) ? Pq : Mq;
            float* Er = (v > 0) ? Pr : Mr;
            float* Eg = (v > 0) ? Pg : Mg;

            // ---- build_tree(j) iteratively ---------------------------------
            uint32_t freemask = (1u << (MAXJ + 2)) - 1u;
            bool s_sub = true;
            int cand = -1, cn = 0;
            const int nleaf = 1 << j;
            for (int k = 0; k < nleaf; ++k) {
                // leaf: leapfrog_step(theta, r, v*eps) + hamiltonian (nuts.py:160-164)
                for (int jj = G.tid; jj < D; jj += T) {
                    const float pj = Er[jj] + h * Eg[jj];
                    Er[jj] = pj;
                    Eq[jj] = Eq[jj] + e * pj;
                    Eg[jj] = 0.0f;  // the evaluator accumulates into a zeroed gradient
                }
                G.sync();
                MC_STAMP(8);
                const float lpl = eval_lp_grad<WPC, false, EX>(Pd, Eq, Eg, G, S, true);
                MC_STAMP(9);
                float kl = 0.0f;
                for (int jj = G.tid; jj < D; jj += T) {
                    const float pj = Er[jj] + h * Eg[jj];
                    Er[jj] = pj;
                    kl += pj * pj;
                }
                const float Hl = -lpl + 0.5f * G.sum(kl);
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
                float* cq = pool + (int64_t)(2 * f) * Dp;
                float* cgp = pool + (int64_t)(2 * f + 1) * Dp;
                const bool opens = (j >= 1) && ((k & 1) == 0);
                const int fslot = (k == 0) ? j : ctz_u32((uint32_t)k);
                float* fq = first + (int64_t)(2 * fslot) * Dp;
                float* fr = first + (int64_t)(2 * fslot + 1) * Dp;
                for (int jj = G.tid; jj < D; jj += T) {
                    const float qv = Eq[jj];
                    cq[jj] = qv;
                    cgp[jj] = Eg[jj];
                    if (opens) {
                        fq[jj] = qv;
                        fr[jj] = Er[jj];
                    }
                }
                if (G.tid == 0) pool_lp[f] = lpl;
                G.sync();
                MC_STAMP(11);
                if (!s_leaf) {
                    s_sub = false;
                    break;
                }
                cand = f;
                cn = n_leaf;

                // merge completed subtrees upward
                bool parked = false;
                for (int l = 0; l < j; ++l) {
                    if (((k + 1) >> l) & 1) {
                        if (G.tid == 0) {
                            pend_idx[l] = cand;
                            pend_n[l] = cn;
                        }
                        G.sync();
                        parked = true;
                        break;
                    }
                    const int pidx = pend_idx[l];
                    const int pn = pend_n[l];
                    const mc_u32x4 rm = mc_draw(cfg.seed, chain_id, (uint32_t)it,
                                                MC_RNG_TAG_MERGE, (uint32_t)j,
                                                ((uint32_t)l << 20) | (uint32_t)k);
                    const double den = (double)(pn + cn) > 1.0 ? (double)(pn + cn) : 1.0;
                    // U < cn / den (nuts.py:205) as U * den < cn: exact in f64 (U a
                    // multiple of 2^-24, den < 2^24), the same decision as the
                    // rounded quotient (no representable U lies between the two)
                    const bool take_second = (double)mc_u01_f32(rm.x) * den < (double)cn;
                    if (take_second) {
                        freemask |= (1u << pidx);
                    } else {
                        freemask |= (1u << cand);
                        cand = pidx;
                    }
                    cn = pn + cn;
                    // U-turn over the merged level-(l+1) subtree
                    const int k0 = k + 1 - (2 << l);
                    const int slot = (k0 == 0) ? j : ctz_u32((uint32_t)k0);
                    const float* bq = first + (int64_t)(2 * slot) * Dp;
                    const float* br = first + (int64_t)(2 * slot + 1) * Dp;
                    const bool ok = (v > 0) ? no_u_turn<WPC>(bq, Eq, br, Er, D, G)
                                            : no_u_turn<WPC>(Eq, bq, Er, br, D, G);
                    if (!ok) {
                        s_sub = false;
                        break;
                    }
                }
                MC_STAMP(12);
                if (!s_sub) break;
                if (parked) continue;
                // l reached j: the depth-j subtree is complete
            }

            // ---- top level (nuts.py:262-284) --------------------------------
            if (s_sub) {
                const double den = (double)n > 1.0 ? (double)n : 1.0;
                // U < min(1, cn / den) (nuts.py:269-272); U < 1 always, and U < cn / den
                // as U * den < cn (exact, see the merge)
                if ((double)mc_u01_f32(rd.y) * den < (double)cn) {
                    const float* cq = pool + (int64_t)(2 * cand) * Dp;
                    const float* cgp = pool + (int64_t)(2 * cand + 1) * Dp;
                    for (int jj = G.tid; jj < D; jj += T) {
                        sq[jj] = cq[jj];
                        sg[jj] = cgp[jj];
                    }
                    lp = pool_lp[cand];
                }
            }
            n += cn;
            s = s_sub && no_u_turn<WPC>(Mq, Pq, Mr, Pr, D, G);
            j += 1;
            G.sync();
            MC_STAMP(13);
        }

        const double alpha = alpha_sum / (n_alpha > 1 ? (double)n_alpha : 1.0);
        n_grad += leaves;
        sc.n_divergent += divergent;
        sc.alpha_sum += alpha;
        sc.n_accept += (alpha > 0.5) ? 1 : 0;
        sc.n_total += 1;
        sc.depth_sum += j;
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
                for (int jj = G.tid; jj < D; jj += T) out[jj] = sq[jj];
            }
        }
        if (G.tid == 0) {
            const int64_t ti = it - tr.iter_begin;
            if (ti >= 0 && ti < tr.capacity) {
                const int64_t o = c * tr.capacity + ti;
                if (tr.accepted) tr.accepted[o] = (alpha > 0.5) ? 1 : 0;
                if (tr.accept_stat) tr.accept_stat[o] = (float)alpha;
                if (tr.step_size) tr.step_size[o] = eps_used;
                if (tr.energy) tr.energy[o] = H0;
                if (tr.tree_depth) tr.tree_depth[o] = j;
                if (tr.n_leapfrog) tr.n_leapfrog[o] = leaves;
            }
        }
        G.sync();
        MC_STAMP(15);
    }
    MC_STAMP_FLUSH

    if (G.tid == 0) {
        sc.logp = lp;
        sc.step_size = eps;
        sc.n_grad += n_grad;
        scal[c] = sc;
    }
}

}  // namespace mc
