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
#pragma once
#include <hip/hip_runtime.h>
#include "internal.h"

#define MC_DEV __device__ __forceinline__

namespace mc {

MC_DEV float wave_sum(float x) {
    // xor butterfly: every lane ends with the bit-identical total
    // (each stage adds a pair in both orders; fp add is commutative).
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}

// A chain group: WPC wavefronts that together own one chain.  With WPC == 1
// several chains share a workgroup and never use the workgroup barrier.
template <int WPC>
struct Group {
    static constexpr int T = 64 * WPC;
    int tid;
    float* red;  // LDS scratch, WPC floats

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

// LDS scratch used by the deterministic segmented sum of a sorted gather.
struct SegScratch {
    int* kf;    // first run's segment of each thread's piece (-1: empty)
    float* af;  // its partial cotangent
    int* kl;    // last run's segment (== kf when the piece has one run)
    float* al;
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

MC_DEV bool is_vec(int kind) {
    return kind == MC_OP_DATA || kind == MC_OP_PVEC || kind == MC_OP_GATHER;
}

MC_DEV float uniform_value(const DevOperand& o, const float* q) {
    if (o.kind == MC_OP_PSCALAR) return q[o.poff];
    if (o.kind == MC_OP_CONST) return o.cval;
    return 0.0f;
}

MC_DEV int gidx(const DevOperand& o, const DevCtx& P, int64_t i) {
    return P.index[o.pool + i];
}

MC_DEV float fetch(const DevOperand& o, int64_t i, float uni, const float* q, const DevCtx& P) {
    switch (o.kind) {
        case MC_OP_DATA:
            return P.data[o.pool + i];
        case MC_OP_PVEC:
            return q[o.poff + i];
        case MC_OP_GATHER:
            return q[o.poff + gidx(o, P, i)];
        default:
            return uni;
    }
}

// Accumulate a per-element cotangent for operand o (not the sorted primary).
MC_DEV void accum(const DevOperand& o, int64_t i, float c, float& scalar_part, float* g,
                  const DevCtx& P) {
    switch (o.kind) {
        case MC_OP_PSCALAR:
            scalar_part += c;
            break;
        case MC_OP_PVEC:
            g[o.poff + i] += c;
            break;
        case MC_OP_GATHER:
            g[o.poff + gidx(o, P, i)] += c;
            break;
        default:
            break;
    }
}

template <int WPC>
MC_DEV void eval_term(const DevTerm& T, const DevCtx& P, const float* q, float* g,
                      const Group<WPC>& G, float& lp_acc, const SegScratch& S) {
    const float uv = uniform_value(T.op[0], q);
    const float um = uniform_value(T.op[1], q);
    const float us = uniform_value(T.op[2], q);
    const bool scale_vec = is_vec(T.op[2].kind);
    const float ulogs = scale_vec ? 0.0f : logf(us);
    const float w = T.weight;
    const bool normal = (T.dist == MC_DIST_NORMAL);

    for (int pass = 0; pass < T.npass; ++pass) {
        const uint32_t mask =
            pass == 0 ? T.pass_mask[0] : (pass == 1 ? T.pass_mask[1] : T.pass_mask[2]);
        float pv = 0.0f, pm = 0.0f, ps = 0.0f;

        // one element: forward + VJP, accumulate everything except the
        // sorted primary gather; returns the primary's cotangent.
        auto element = [&](int64_t i) -> float {
            const float v = fetch(T.op[0], i, uv, q, P);
            const float m = fetch(T.op[1], i, um, q, P);
            const float s = fetch(T.op[2], i, us, q, P);
            const float logs = scale_vec ? logf(s) : ulogs;
            const ElemOut e = normal ? elem_normal(T.c0, v, m, s, logs)
                                     : elem_halfnormal(T.c0, v, s, logs);
            if (mask & PASS_LP) lp_acc += w * e.lp;
            const float cv = w * e.dv, cm = w * e.dm, cs = w * e.ds;
            float cprim = 0.0f;
            if (mask & PASS_VALUE) {
                if (T.primary == 0) cprim = cv;
                else accum(T.op[0], i, cv, pv, g, P);
            }
            if (mask & PASS_LOC) {
                if (T.primary == 1) cprim = cm;
                else accum(T.op[1], i, cm, pm, g, P);
            }
            if (mask & PASS_SCALE) {
                if (T.primary == 2) cprim = cs;
                else accum(T.op[2], i, cs, ps, g, P);
            }
            return cprim;
        };

        if (T.primary < 0) {
            for (int64_t i = G.tid; i < T.n; i += G.T) (void)element(i);
        } else {
            // Elements are sorted by the primary index: each thread takes a
            // contiguous piece and sums runs of equal index in registers.
            // Runs strictly inside a piece are owned by the thread; the first
            // and last run of each piece are combined in thread order below.
            const DevOperand po =
                T.primary == 0 ? T.op[0] : (T.primary == 1 ? T.op[1] : T.op[2]);
            const bool acc_prim = (mask & (1u << T.primary)) != 0;
            const int64_t n = T.n;
            const int tact = (int)(n < (int64_t)G.T ? n : (int64_t)G.T);
            int kf = -1, kl = -1;
            float af = 0.0f, al = 0.0f;
            if (G.tid < tact) {
                const int64_t b = (n * G.tid) / tact;
                const int64_t e = (n * (G.tid + 1)) / tact;
                int kcur = -1, nruns = 0;
                float acc = 0.0f;
                for (int64_t i = b; i < e; ++i) {
                    const float c = element(i);
                    if (acc_prim) {
                        const int k = gidx(po, P, i);
                        if (k != kcur) {
                            if (kcur >= 0) {
                                if (nruns == 1) {
                                    kf = kcur;
                                    af = acc;
                                } else {
                                    g[po.poff + kcur] += acc;
                                }
                            }
                            kcur = k;
                            acc = 0.0f;
                            ++nruns;
                        }
                        acc += c;
                    }
                }
                if (acc_prim) {
                    if (nruns == 1) {
                        kf = kcur;
                        af = acc;
                    }
                    kl = kcur;
                    al = acc;
                }
            }
            if (acc_prim) {
                S.kf[G.tid] = kf;
                S.af[G.tid] = af;
                S.kl[G.tid] = kl;
                S.al[G.tid] = al;
                G.sync();
                if (G.tid < tact) {
                    const bool single = (kf == kl);
                    const bool lead_f = (G.tid == 0) || (S.kl[G.tid - 1] != kf);
                    // a leader sums the pieces that continue its segment, in order
                    auto chain = [&](int k, float s) -> float {
                        for (int t2 = G.tid + 1; t2 < tact && S.kf[t2] == k; ++t2) {
                            s += S.af[t2];
                            if (S.kl[t2] != S.kf[t2]) break;
                        }
                        return s;
                    };
                    if (single) {
                        if (lead_f) g[po.poff + kf] += chain(kf, af);
                    } else {
                        if (lead_f) g[po.poff + kf] += af;
                        g[po.poff + kl] += chain(kl, al);
                    }
                }
            }
        }

        // broadcast-parameter cotangents: fixed-order group reduction
        if ((mask & PASS_VALUE) && T.op[0].kind == MC_OP_PSCALAR) {
            const float t = G.sum(pv);
            if (G.tid == 0) g[T.op[0].poff] += t;
        }
        if ((mask & PASS_LOC) && T.op[1].kind == MC_OP_PSCALAR) {
            const float t = G.sum(pm);
            if (G.tid == 0) g[T.op[1].poff] += t;
        }
        if ((mask & PASS_SCALE) && T.op[2].kind == MC_OP_PSCALAR) {
            const float t = G.sum(ps);
            if (G.tid == 0) g[T.op[2].poff] += t;
        }
        G.sync();
    }
}

// Log density at q and its gradient into g (g may not alias q).  Every thread
// of the group returns the same value.
template <int WPC>
MC_DEV float eval_lp_grad(const DevCtx& P, const float* q, float* g, const Group<WPC>& G,
                          const SegScratch& S) {
    for (int j = G.tid; j < P.D; j += G.T) g[j] = 0.0f;
    G.sync();
    float lp_acc = 0.0f;
    for (int t = 0; t < P.n_terms; ++t) {
        const DevTerm T = P.terms[t];
        eval_term<WPC>(T, P, q, g, G, lp_acc, S);
    }
    return G.sum(lp_acc) + P.lp_const;
}

// LDS floats a chain group needs for reductions + segmented-sum scratch.
__host__ __device__ constexpr int group_scratch_floats(int wpc) { return 16 + 4 * 64 * wpc; }

template <int WPC>
MC_DEV void carve_group(float* base, Group<WPC>& G, SegScratch& S) {
    constexpr int T = 64 * WPC;
    G.red = base;
    S.kf = reinterpret_cast<int*>(base + 16);
    S.af = base + 16 + T;
    S.kl = reinterpret_cast<int*>(base + 16 + 2 * T);
    S.al = base + 16 + 3 * T;
}

}  // namespace mc
