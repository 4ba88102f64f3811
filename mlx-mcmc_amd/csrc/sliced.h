// sliced.h — sliced HMC: each chain's log density is split into S data
// slices, and one workgroup evaluates one slice for a block of NB chains.
// Same sampler as k_hmc (hmc.h; reference hmc.py:7-206), different work
// decomposition:
//
//   * the parameters are partitioned: a parameter whose cotangent only comes
//     from elements of one slice is *private* to that slice (theta_g of the
//     groups whose observations the slice holds); a parameter used as a
//     broadcast operand (mu, tau, sigma) is *shared* and replicated in every
//     slice;
//   * a workgroup keeps q, p, grad of its private + shared parameters for its
//     NB chains in LDS, and its slice of the data (plus the slice's run
//     tables) in LDS, loaded once per launch;
//   * wave w evaluates chains 2w and 2w+1: each lane walks its runs once and
//     updates both chains from registers, so every data element is read from
//     LDS once per two chains (LDS bandwidth is the binding resource at one
//     chain per lane);
//   * per leapfrog step the S workgroups of a chain block exchange one small
//     record per chain — the slice's log p partial, its cotangent partials of
//     the shared parameters and its kinetic-energy partials — as tagged 8-byte
//     granules (write-through stores, polled with L1-bypassing loads; no
//     fences, no atomics on the data path).  Every workgroup then sums the S
//     records in slice order, so all copies of a shared parameter stay
//     bit-identical and the accept decision is the same in every slice.
//
// Private parameters advance with their own (complete) gradient; nothing else
// crosses workgroups.  Summation order is fixed (no float atomics): a run is
// bit-reproducible and a chain's trajectory does not depend on NB, on the
// chain's position in its block or on how chains are split over launches.
#pragma once
#include "eval.h"
#include "philox.h"

namespace mc {

enum : int32_t { SK_NONE = 0, SK_CONST = 1, SK_SHARED = 2, SK_DATA = 3, SK_PP = 4 };

constexpr int kSlLanes = 64;  // run slots per chain pair (one wave serves two chains)
constexpr int kSlItr = 8;     // run iterations per combine round
constexpr int kSlVc = kSlLanes * kSlItr;  // staged run cotangents per chain and round
constexpr int kSlShReg = 4;   // shared parameters whose cotangents stay in registers

// One term restricted to one slice.  Its elements are grouped into runs of
// equal per-element parameter ("pp", the PVEC/GATHER operand) — or plain
// chunks when the term has none.  Runs are dealt to the 64 lanes of a wave
// longest first; lane j's it-th run is "run (it, j)".  Data operands are tiled
// per iteration: element u of run (it, j) at off[it] + (u/4)*256 + 4j + u%4.
// All tables live in the slice's block next to its data (LDS).
struct SlTerm {
    int32_t dist;
    int32_t mode;      // 0: broadcast scale (moment sums), 1: per-element scale
    int32_t pp;        // operand slot of the per-element parameter, or -1
    int32_t direct;    // pp runs have distinct parameters: write gradients directly
    int32_t niter;     // run iterations per lane (0: no elements in this slice)
    float weight;
    float c0;
    float clogs;       // CONST scale: f32 log(scale)
    int32_t kind[3];   // SK_* of value, loc, scale
    int32_t kloc[3];   // SK_SHARED: local slot
    int32_t jsh[3];    // SK_SHARED: ordinal among the shared parameters
    int32_t doff[3];   // SK_DATA: float offset in the slice's block
    float cval[3];     // SK_CONST
    float cinv, cinv2; // CONST scale: f32 1/scale, 1/scale^2
    float clg;         // Gamma / Beta with constant shapes: gammaln normaliser
    // int32 tables at these word offsets in the slice block
    int32_t tile_off;   // per iteration: {data offset, len_max, len_min / 4}
    int32_t lane_off;   // per (iteration, lane): {local slot or -1, len} (len 0: none)
    int32_t round_off;  // ceil(niter / kSlItr) + 1 offsets into the combine entries
    int32_t comb_off;   // entries {local slot, position-list offset, count}
    int32_t pos_off;    // positions ((it % kSlItr) * 64 + lane) of each entry's runs
};

struct SlCtx {
    const SlTerm* terms;    // [S][n_terms]
    const float* data;      // slice blocks
    const int32_t* index;   // (unused: the tables are in the blocks)
    const int64_t* blocks;  // per slice {data offset, data floats, private count, active terms}
    const int32_t* gidx;    // [S][Lp] global parameter of each local slot, -1: padding
    int32_t n_terms;
    int32_t S;
    int32_t Lp;             // local slots per chain: private (< Pmax) then shared
    int32_t Pmax;
    int32_t Dsh;
    int32_t D;
    int32_t nitems;         // exchange record per chain: lp, Dsh cotangents, K0, K1
    int32_t sdata_floats;   // LDS floats reserved for a slice's block
    float lp_const;
    int32_t combine;        // some slice term has split runs (needs the staging area)
    const SlTerm* sterms;   // scalar terms (constants / broadcast parameters only),
    int32_t n_sterms;       //   niter = element count; evaluated after the exchange
    int32_t pad;
};

// LDS layout of a sliced workgroup (floats).
template <int NB>
struct SlLayout {
    int sd, q2, g2, pm, vpart, sacc, xin, ob, der, sst, cs, total;
    __host__ __device__ SlLayout(const SlCtx& P) {
        int o = 0;
        sd = o;    o += (P.sdata_floats + 3) / 4 * 4;
        q2 = o;    o += 2 * NB * P.Lp;
        g2 = o;    o += 2 * NB * P.Lp;
        pm = o;    o += NB * P.Lp;
        vpart = o; o += P.combine ? NB * kSlVc : 0;
        sacc = o;  o += NB * (P.Dsh + 1);
        xin = o;   o += (P.S > 16 || P.nitems * NB * 16 > 4 * (kSlLanes * NB / 2))
                             ? P.S * P.nitems * NB : 0;
        ob = o;    o += P.nitems * NB;
        o = (o + 3) / 4 * 4;
        der = o;   o += 4 * NB * (P.Dsh > 0 ? P.Dsh : 1);
        sst = o;   o += (P.Dsh + 1) * NB * P.n_sterms;
        o = (o + 1) / 2 * 2;
        cs = o;    o += 24 * NB + 8;
        total = o;
    }
};

// per-chain scalars kept in LDS (index into the cs area, stride NB)
enum : int {
    CS_EPS = 0,    // double, 2 words
    CS_LP = 2, CS_LPN, CS_LPP, CS_H, CS_E, CS_K0P, CS_K1P, CS_K0, CS_K1,
    CS_NACC, CS_NTOT, CS_WACC, CS_WTOT, CS_K0S, CS_COUNT
};

MC_DEV int slot_of(uint32_t mask, int b, int NB, int Lp) {
    return ((int)((mask >> b) & 1u) * NB + b) * Lp;
}

// A slice-term read once per term from the constant address space (a few
// batched scalar loads instead of a separately waited load at every use).
MC_DEV SlTerm load_slterm(const MC_CONST SlTerm* p) {
    SlTerm t;
    t.dist = p->dist;
    t.mode = p->mode;
    t.pp = p->pp;
    t.direct = p->direct;
    t.niter = p->niter;
    t.weight = p->weight;
    t.c0 = p->c0;
    t.clogs = p->clogs;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        t.kind[a] = p->kind[a];
        t.kloc[a] = p->kloc[a];
        t.jsh[a] = p->jsh[a];
        t.doff[a] = p->doff[a];
        t.cval[a] = p->cval[a];
    }
    t.cinv = p->cinv;
    t.cinv2 = p->cinv2;
    t.clg = p->clg;
    t.tile_off = p->tile_off;
    t.lane_off = p->lane_off;
    t.round_off = p->round_off;
    t.comb_off = p->comb_off;
    t.pos_off = p->pos_off;
    return t;
}

// value of operand a for this thread's chain when it is not per-element
MC_DEV float sl_uni(const SlTerm& T, int a, const float* qc) {
    return T.kind[a] == SK_SHARED ? qc[T.kloc[a]] : (T.kind[a] == SK_CONST ? T.cval[a] : 0.0f);
}

// Moment sums of one run for two chains (broadcast scale): d = value - loc,
// formed exactly as the reference's (value - loc): x - m, v - y, x - y or v - m.
// DC bit 0: value is data, bit 1: loc is data; vv/mm: the chains' run values
// of the non-data operands.
template <int DC>
MC_DEV float sl_diff(float x, float y, float vv, float mm) {
    return (DC == 0) ? (vv - mm) : (DC == 1) ? (x - mm) : (DC == 2) ? (vv - y) : (x - y);
}

// Four float4 rows per batch (loads issued before the arithmetic); each
// element feeds two chains.
template <int DC>
MC_DEV void run_moments2(const float* xv, const float* xm, int len, int lmin4, const float (&vv)[2],
                         const float (&mm)[2], float (&s1)[2], float (&s2)[2]) {
    float a1[2] = {0.f, 0.f}, a2[2] = {0.f, 0.f};
    auto elem = [&](float x, float y) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const float d = sl_diff<DC>(x, y, vv[c], mm[c]);
            a1[c] += d;
            a2[c] = fmaf(d, d, a2[c]);
        }
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
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        s1[c] += a1[c];
        s2[c] += a2[c];
    }
}

// Scalar terms (every operand a constant or a broadcast parameter): lane b
// of wave t % NW evaluates term t for chain b into its staging row {lp,
// dvalue, dloc, dscale}; the exchange adds the rows in term order to the
// total log p and the shared gradient totals, identically in every slice.
template <int NB>
MC_DEV void sl_scalar_stage(const SlCtx& P, const float* q2, uint32_t pmask, float* st, int tid) {
    constexpr int NW = NB / 2;  // waves: term t on wave t % NW (uniform descriptor
                                // loads), lane b = chain b
    const int wave = tid >> 6, b = tid & 63;
    const int Dc = P.Dsh + 1;
    for (int t = wave; t < P.n_sterms && b < NB; t += NW) {
        const float* qc = q2 + slot_of(pmask, b, NB, P.Lp);
        const SlTerm T = load_slterm(cptr(P.sterms) + t);
        const float v = sl_uni(T, 0, qc), m = sl_uni(T, 1, qc), sc = sl_uni(T, 2, qc);
        const float ls = (T.kind[2] == SK_CONST) ? T.clogs : logf(sc);
        const float lg = (T.kind[1] == SK_SHARED || T.kind[2] == SK_SHARED)
                             ? lgamma_norm(T.dist, m, sc) : T.clg;
        const ElemOut e = elem_eval(T.dist, T.c0, v, m, sc, ls, lg);
        const float wn = T.weight * (float)T.niter;
        // row (t, b): column 0 log p, column 1 + j shared parameter j
        float* row = st + (t * NB + b) * Dc;
        for (int c = 0; c < Dc; ++c) row[c] = 0.0f;
        row[0] = wn * e.lp;
        if (T.kind[0] == SK_SHARED) row[1 + T.jsh[0]] += wn * e.dv;
        if (T.kind[1] == SK_SHARED) row[1 + T.jsh[1]] += wn * e.dm;
        if (T.kind[2] == SK_SHARED) row[1 + T.jsh[2]] += wn * e.ds;
    }
}

// One term of one slice; wave w evaluates chains b0 = 2w and 2w+1, lane j
// walks runs (it, j).  Adds to lp[] (the lanes' log p partials), writes
// (direct) or stages and combines (split runs) the per-element parameter
// cotangents, and deposits the wave totals of the broadcast-operand
// cotangents into sacc[b][jsh].
template <int NB>
MC_DEV void sl_term(const SlCtx& P, const SlTerm& T, const float* sd, const float* q2, float* g2,
                    uint32_t pmask, int b0, int j, float* vpart, float* sacc, const float4* der,
                    int tid, float (&lp)[2], float (&acc)[kSlShReg][2]) {
    MC_STAMP_DECL
    constexpr int NT = kSlLanes * NB / 2;
    const int Lp = P.Lp;
    int qb[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) qb[c] = slot_of(pmask, b0 + c, NB, Lp);
    const int k0 = T.kind[0], k1 = T.kind[1], k2 = T.kind[2];
    const float w = T.weight, c0 = T.c0;
    const int32_t* tab = (const int32_t*)sd;
    const int32_t* tiles = tab + T.tile_off;
    const int32_t* lanes = tab + T.lane_off;
    const int nrounds = (T.niter + kSlItr - 1) / kSlItr;
    const bool combine = T.pp >= 0 && !T.direct;

    // the chains' broadcast operand values and derived scale values
    float uv[2], um[2], us[2], is[2], iv[2], lg[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const float* qc = q2 + qb[c];
        uv[c] = sl_uni(T, 0, qc);
        um[c] = sl_uni(T, 1, qc);
        us[c] = sl_uni(T, 2, qc);
        is[c] = T.cinv;
        iv[c] = T.cinv2;
        lg[c] = T.clogs;
        if (k2 == SK_SHARED) {
            const float4 d = der[(b0 + c) * P.Dsh + T.jsh[2]];
            is[c] = d.y;
            iv[c] = d.z;
            lg[c] = d.w;
        }
    }
    float pv[2] = {0.f, 0.f}, pm[2] = {0.f, 0.f}, ps[2] = {0.f, 0.f};
    MC_STAMP(12);

    for (int rd = 0; rd < nrounds; ++rd) {
        MC_STAMP(23);
        const int it_end = min(T.niter, (rd + 1) * kSlItr);
        for (int it = rd * kSlItr; it < it_end; ++it) {
            const int toff = tiles[3 * it], lmin4 = tiles[3 * it + 2];
            const int2 rec = *(const int2*)(lanes + 2 * (it * kSlLanes + j));
            const int k = rec.x, len = rec.y;
            float th[2];
#pragma unroll
            for (int c = 0; c < 2; ++c) th[c] = (len > 0 && k >= 0) ? q2[qb[c] + k] : 0.0f;
            const float* x0 = sd + T.doff[0] + toff + 4 * j;
            const float* x1 = sd + T.doff[1] + toff + 4 * j;
            const float* x2 = sd + T.doff[2] + toff + 4 * j;
            float rc[2] = {0.f, 0.f};
            MC_STAMP(13);
            if (len > 0) {
                if (T.mode == 0) {
                    float s1[2] = {0.f, 0.f}, s2[2] = {0.f, 0.f}, cnt[2];
                    bool neg[2] = {false, false};
                    if (T.dist == MC_DIST_NORMAL) {
                        {
                            float vv[2], mm[2];
#pragma unroll
                            for (int c = 0; c < 2; ++c) {
                                vv[c] = (k0 == SK_PP) ? th[c] : uv[c];
                                mm[c] = (k1 == SK_PP) ? th[c] : um[c];
                            }
                            const int dc = (k0 == SK_DATA ? 1 : 0) | (k1 == SK_DATA ? 2 : 0);
                            if (dc == 1) run_moments2<1>(x0, x1, len, lmin4, vv, mm, s1, s2);
                            else if (dc == 0) run_moments2<0>(x0, x1, len, lmin4, vv, mm, s1, s2);
                            else if (dc == 2) run_moments2<2>(x0, x1, len, lmin4, vv, mm, s1, s2);
                            else run_moments2<3>(x0, x1, len, lmin4, vv, mm, s1, s2);
                        }
                        cnt[0] = cnt[1] = (float)len;
                        MC_STAMP(14);
                    } else {
                        // HalfNormal: moments of the value over value >= 0 (the
                        // VJP of mx.where sends nothing through the -inf branch)
                        cnt[0] = cnt[1] = 0.0f;
                        for (int u = 0; u < len; ++u) {
                            const float x = (k0 == SK_DATA) ? x0[(u >> 2) * 256 + (u & 3)] : 0.0f;
#pragma unroll
                            for (int c = 0; c < 2; ++c) {
                                const float d = (k0 == SK_DATA) ? x : ((k0 == SK_PP) ? th[c] : uv[c]);
                                if (d >= 0.0f) {
                                    s1[c] += d;
                                    s2[c] = fmaf(d, d, s2[c]);
                                    cnt[c] += 1.0f;
                                } else {
                                    neg[c] = true;
                                }
                            }
                        }
                    }
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        const float lpt = neg[c] ? -__builtin_inff()
                                                 : cnt[c] * (c0 - lg[c]) - (0.5f * s2[c]) * iv[c];
                        lp[c] += w * lpt;
                        const float t = w * (s1[c] * iv[c]);
                        rc[c] = (T.pp == 0) ? -t : t;
                        pv[c] += -t;
                        pm[c] += t;
                        ps[c] += w * ((s2[c] * iv[c] - cnt[c]) * is[c]);
                    }
                } else {
                    // per-element scale: the reference's formula per element
                    // (chain by chain, explicit indices: no arrays behind a loop)
                    auto elemwise = [&](float thc, float uvc, float umc, float usc, float lgc,
                                        float& lpc, float& rcc, float& pvc, float& pmc,
                                        float& psc) {
                        const float lsc = (k2 == SK_PP) ? logf(thc) : lgc;
                        // gammaln normaliser: per element when a shape varies by
                        // element, else once per chain
                        const bool lgv = (k1 == SK_DATA || k1 == SK_PP || k2 == SK_DATA ||
                                          k2 == SK_PP);
                        const float lgu = (k1 == SK_SHARED || k2 == SK_SHARED)
                                              ? lgamma_norm(T.dist, umc, usc) : T.clg;
                        for (int u = 0; u < len; ++u) {
                            const int o = (u >> 2) * 256 + (u & 3);
                            const float v = (k0 == SK_DATA) ? x0[o] : (k0 == SK_PP ? thc : uvc);
                            const float m = (k1 == SK_DATA) ? x1[o] : (k1 == SK_PP ? thc : umc);
                            const float sc = (k2 == SK_DATA) ? x2[o] : (k2 == SK_PP ? thc : usc);
                            const float ls = (k2 == SK_DATA) ? logf(sc) : lsc;
                            const float lg = lgv ? lgamma_norm(T.dist, m, sc) : lgu;
                            const ElemOut e = elem_eval(T.dist, c0, v, m, sc, ls, lg);
                            lpc += w * e.lp;
                            rcc += w * (T.pp == 0 ? e.dv : (T.pp == 1 ? e.dm : e.ds));
                            pvc += w * e.dv;
                            pmc += w * e.dm;
                            psc += w * e.ds;
                        }
                    };
                    elemwise(th[0], uv[0], um[0], us[0], lg[0], lp[0], rc[0], pv[0], pm[0], ps[0]);
                    elemwise(th[1], uv[1], um[1], us[1], lg[1], lp[1], rc[1], pv[1], pm[1], ps[1]);
                }
                if (T.pp >= 0 && T.direct) {  // the run owns its parameter
                    g2[qb[0] + k] += rc[0];
                    g2[qb[1] + k] += rc[1];
                }
            }
            if (combine) {
                const int ps_ = (it - rd * kSlItr) * kSlLanes + j;
                vpart[b0 * kSlVc + ps_] = rc[0];
                vpart[(b0 + 1) * kSlVc + ps_] = rc[1];
            }
        }
        if (combine) {
            // the runs of one parameter summed in run order, then added to its slot
            __syncthreads();
            const int32_t* rounds = tab + T.round_off;
            const int32_t* comb = tab + T.comb_off;
            const int32_t* pos = tab + T.pos_off;
            const int e0 = rounds[rd], ne = rounds[rd + 1] - e0;
            for (int idx = tid; idx < ne * NB; idx += NT) {
                const int bb = idx % NB, e = e0 + idx / NB;
                const int kk = comb[3 * e], po = comb[3 * e + 1], cntr = comb[3 * e + 2];
                const float* vp = vpart + bb * kSlVc;
                float s = vp[pos[po]];
                for (int q = 1; q < cntr; ++q) s += vp[pos[po + q]];
                g2[slot_of(pmask, bb, NB, Lp) + kk] += s;
            }
            __syncthreads();
        }
    }
    MC_STAMP(15);
    if (P.Dsh <= kSlShReg) {
        // broadcast-operand cotangents stay per lane until the end of the
        // evaluation (one reduction per shared parameter, not per term)
#pragma unroll
        for (int q = 0; q < kSlShReg; ++q) {
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                if (k0 == SK_SHARED && T.jsh[0] == q) acc[q][c] += pv[c];
                if (k1 == SK_SHARED && T.jsh[1] == q) acc[q][c] += pm[c];
                if (k2 == SK_SHARED && T.jsh[2] == q) acc[q][c] += ps[c];
            }
        }
    } else {
        // wave totals per term, one writer per chain
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            float* row = sacc + (b0 + c) * (P.Dsh + 1);
            if (k0 == SK_SHARED) {
                const float x = wave_sum(pv[c]);
                if (j == 0) row[T.jsh[0]] += x;
            }
            if (k1 == SK_SHARED) {
                const float x = wave_sum(pm[c]);
                if (j == 0) row[T.jsh[1]] += x;
            }
            if (k2 == SK_SHARED) {
                const float x = wave_sum(ps[c]);
                if (j == 0) row[T.jsh[2]] += x;
            }
        }
    }
    MC_STAMP(16);
}

// Log density partial of this slice and its gradient contributions, for all
// NB chains at their proposal slots (mask bit b: chain b's proposal buffer).
// g2 at the proposal slots must be zero on entry.  Private gradients are
// complete on return; shared ones hold this slice's partial; cs[LPP] = the
// slice's log p partial.
template <int NB>
MC_DEV void sl_eval(const SlCtx& P, int slice, int nact, const float* sd, const float* q2,
                    float* g2, uint32_t pmask, float* vpart, float* sacc, float4* der, float* sst,
                    float* ob, int tid) {
    constexpr int NT = kSlLanes * NB / 2;
    const int Lp = P.Lp, Dc = P.Dsh + 1;
    const int b0 = 2 * (tid >> 6), j = tid & 63;
    const MC_CONST SlTerm* tt = cptr(P.terms) + (int64_t)slice * P.n_terms;
    MC_STAMP_DECL
    // per chain and shared parameter: {x, 1/x, 1/x^2, f32 log x} (the scale
    // operands' derived values, computed once instead of in every lane)
    for (int idx = tid; idx < NB * P.Dsh; idx += NT) {
        const int bb = idx / P.Dsh, jj = idx - bb * P.Dsh;
        const float x = q2[slot_of(pmask, bb, NB, Lp) + P.Pmax + jj];
        der[idx] = make_float4(x, 1.0f / x, 1.0f / (x * x), logf(x));
    }
    __syncthreads();
    float lp[2] = {0.0f, 0.0f};
    float acc[kSlShReg][2];
#pragma unroll
    for (int q = 0; q < kSlShReg; ++q) acc[q][0] = acc[q][1] = 0.0f;
    for (int t = 0; t < nact; ++t) {  // the slice's active terms, compacted
        const SlTerm T = load_slterm(tt + t);
        MC_STAMP(22);
        // no barrier between terms: a parameter's direct runs are on the same
        // lane in every term (the planner's lane map), split runs are combined
        // between barriers of their own
        sl_term<NB>(P, T, sd, q2, g2, pmask, b0, j, vpart, sacc, der, tid, lp, acc);
        MC_STAMP(4 + (t < 7 ? t : 7));
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const float x = wave_sum(lp[c]);
        if (j == 0) ob[b0 + c] = x;  // record item 0: log p partial
    }
    if (P.Dsh <= kSlShReg) {
#pragma unroll
        for (int q = 0; q < kSlShReg; ++q) {
            if (q < P.Dsh) {
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    const float x = wave_sum(acc[q][c]);
                    if (j == 0) sacc[(b0 + c) * Dc + q] = x;
                }
            }
        }
    }
    // scalar terms need only this step's shared values: evaluate them in the
    // slack before the barrier (the exchange adds them to the totals)
    sl_scalar_stage<NB>(P, q2, pmask, sst, tid);
    __syncthreads();
    MC_STAMP(11);
    // record items 1..Dsh: this slice's shared cotangent partials (per-element
    // contributions already in the slots plus the broadcast-operand totals)
    for (int idx = tid; idx < NB * P.Dsh; idx += NT) {
        const int bb = idx / P.Dsh, jj = idx - bb * P.Dsh;
        float* a = &sacc[bb * Dc + jj];
        ob[(1 + jj) * NB + bb] = g2[slot_of(pmask, bb, NB, Lp) + P.Pmax + jj] + *a;
        *a = 0.0f;
    }
    __syncthreads();
}

// ---------------------------------------------------------------------------
// exchange
// ---------------------------------------------------------------------------
typedef __attribute__((address_space(1))) unsigned long long gu64_t;

MC_DEV void granule_store(unsigned long long* p, uint32_t tag, float v) {
    __hip_atomic_store((gu64_t*)p, ((unsigned long long)tag << 32) | __float_as_uint(v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
constexpr uint32_t kSpinLimit = 1u << 23;  // ~seconds: then status = 1, exit

MC_DEV unsigned long long granule_load(unsigned long long* p) {
    return __hip_atomic_load((gu64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- same-XCD exchange (round 5) ---------------------------------------------
// granule_store's agent-scope store carries sc1, which drops the line from
// the producer XCD's L2: a consumer on the same XCD then polls it at the
// cross-XCD rate.  A workgroup-scope store (no sc1) writes through the
// producer CU's L1 into its XCD's L2 and keeps the line there, where the
// consumer's sc1 poll (L1 bypassed, L2-served) finds it — valid only when
// every partner of the exchange sits on the same XCD, which the launch
// verifies first (xcd_announce / xcd_agree); across XCDs such a store could stay
// invisible.  The granule stays one 8-byte atomic store: no tearing, no
// ordering needed (the tag validates it).  Same-box A/B, config 3: 113.4 ->
// 120.4 M steps/s; medium 189 -> 225 M (profiles/r5/xcd).
MC_DEV void granule_store_xcd(unsigned long long* p, uint32_t tag, float v) {
    __hip_atomic_store((gu64_t*)p, ((unsigned long long)tag << 32) | __float_as_uint(v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
MC_DEV void granule_put(unsigned long long* p, uint32_t tag, float v, bool xcd_local) {
    if (xcd_local) granule_store_xcd(p, tag, v);
    else granule_store(p, tag, v);
}
// the XCD (XCC) this wave runs on
MC_DEV uint32_t xcc_id() {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x;
}
// Launch-start check that the S workgroups of one exchange group share an
// XCD, in two halves so that its round trip hides behind the first sweep:
// xcd_announce stores this slice's XCC id (agent scope, at slots[16 slice],
// tag = a tag of this launch) and issues the loads of all S slots; xcd_agree
// completes them (re-polling the slots not yet arrived) and returns, the same
// in every wave of every slice, whether the S ids agree; `ok` false on a
// timeout (a partner never arrived).
struct XcdPoll {
    unsigned long long y;
};
MC_DEV XcdPoll xcd_announce(unsigned long long* slots, int S, int slice, uint32_t tag, bool writer) {
    const int j = threadIdx.x & 63;
    if (writer) granule_store(slots + 16 * slice, tag, __uint_as_float(xcc_id()));
    XcdPoll h;
    h.y = j < S ? granule_load(slots + 16 * j) : 0ull;
    return h;
}
MC_DEV bool xcd_agree(XcdPoll h, unsigned long long* slots, int S, uint32_t tag, bool& ok) {
    const int j = threadIdx.x & 63;
    unsigned long long y = h.y;
    bool need = j < S && (uint32_t)(y >> 32) != tag;
    uint32_t spins = 0;
    while (__ballot(need)) {
        if (++spins > kSpinLimit) {
            ok = false;
            return false;
        }
        if (need) {
            y = granule_load(slots + 16 * j);
            need = (uint32_t)(y >> 32) != tag;
        }
    }
    const uint32_t x = (uint32_t)y, x0 = (uint32_t)__shfl((int)x, 0);
    return __ballot(j < S && x != x0) == 0;
}


// Publish this slice's record for every chain (the outbox ob[item][b]);
// collect: wait for all S records of the block and sum them.  Items: 0 log p, 1..Dsh shared
// cotangents, Dsh+1 K0 partial, Dsh+2 K1 partial.  With S <= 16 thread x
// polls the granule of (item x/16, slice x%16) and a 16-lane DPP row sums the
// item straight from registers (a fixed tree, identical in every slice);
// otherwise the records go through LDS and are summed in slice order.  The
// scalar terms' staged rows are added in term order.  Returns false on timeout.
template <int NB>
MC_DEV void sl_publish(const SlCtx& P, int slice, unsigned long long* xg, uint32_t tag,
                       const float* ob, int tid) {
    constexpr int NT = kSlLanes * NB / 2;
    const int n_items = P.nitems * NB;
    for (int idx = tid; idx < n_items; idx += NT)
        granule_store(xg + (int64_t)slice * n_items + idx, tag, ob[idx]);
}

constexpr int kMaxPass = 4;  // granules per thread on the fast (register) path

// Polled granules of one exchange, held in registers between issue and
// completion so that the memory round trip overlaps other work.
struct SlPoll {
    unsigned long long y[kMaxPass];
};

template <int NB>
MC_DEV bool sl_fast_path(const SlCtx& P) {
    constexpr int NT = kSlLanes * NB / 2;
    return P.S <= 16 && (P.nitems * NB * 16 + NT - 1) / NT <= kMaxPass;
}

// Issue this thread's granule loads of the exchange (no wait).
template <int NB>
MC_DEV void sl_poll_issue(const SlCtx& P, unsigned long long* xg, SlPoll& R, int tid) {
    constexpr int NT = kSlLanes * NB / 2;
    if (!sl_fast_path<NB>(P)) return;
    const int n_items = P.nitems * NB;
    const int npass = (n_items * 16 + NT - 1) / NT;
#pragma unroll
    for (int p = 0; p < kMaxPass; ++p) {
        const int x = p * NT + tid, idx = x >> 4, sl = x & 15;
        R.y[p] = 0;
        if (p < npass && idx < n_items && sl < P.S) R.y[p] = granule_load(xg + sl * n_items + idx);
    }
}

// Complete the exchange: re-poll the granules whose tags were stale, sum
// every item over the slices (a 16-lane DPP row per item: a fixed tree,
// identical in every slice; or in slice order through LDS when S > 16) and
// add the scalar terms' staged rows in term order.  Returns false on timeout.
template <int NB>
MC_DEV bool sl_collect(const SlCtx& P, unsigned long long* xg, uint32_t tag, float* g2,
                       uint32_t pmask, float* xin, const float* sst, float* cs, int* flags,
                       int* status, SlPoll& R, int tid) {
    constexpr int NT = kSlLanes * NB / 2;
    const int nI = P.nitems, Dsh = P.Dsh, Lp = P.Lp;
    const int n_items = nI * NB;
    MC_STAMP_DECL
    auto finish_item = [&](int idx, float s) {
        const int i = idx / NB, b = idx - i * NB;
        if (i <= Dsh)
            for (int t = 0; t < P.n_sterms; ++t) s += sst[(t * NB + b) * (Dsh + 1) + i];
        if (i == 0) cs[CS_LPN * NB + b] = s + P.lp_const;
        else if (i <= Dsh) g2[slot_of(pmask, b, NB, Lp) + P.Pmax + i - 1] = s;
        else if (i == Dsh + 1) cs[CS_K0 * NB + b] = s;
        else cs[CS_K1 * NB + b] = s;
    };
    bool ok = true;
    const bool fast = sl_fast_path<NB>(P);
    if (fast) {
        const int npass = (n_items * 16 + NT - 1) / NT;
        float v[kMaxPass];
        uint32_t need = 0;
#pragma unroll
        for (int p = 0; p < kMaxPass; ++p) {
            v[p] = 0.0f;
            const int x = p * NT + tid, idx = x >> 4, sl = x & 15;
            if (p < npass && idx < n_items && sl < P.S) {
                if ((uint32_t)(R.y[p] >> 32) == tag) v[p] = __uint_as_float((uint32_t)R.y[p]);
                else need |= 1u << p;
            }
        }
        uint32_t spins = 0;
        while (need) {
            if (++spins > kSpinLimit) {
                ok = false;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            unsigned long long y[kMaxPass];
#pragma unroll
            for (int p = 0; p < kMaxPass; ++p) {
                const int x = p * NT + tid, idx = x >> 4, sl = x & 15;
                if ((need >> p) & 1u) y[p] = granule_load(xg + sl * n_items + idx);
            }
#pragma unroll
            for (int p = 0; p < kMaxPass; ++p) {
                if (((need >> p) & 1u) && (uint32_t)(y[p] >> 32) == tag) {
                    v[p] = __uint_as_float((uint32_t)y[p]);
                    need &= ~(1u << p);
                }
            }
        }
#pragma unroll
        for (int p = 0; p < kMaxPass; ++p) {
            if (p < npass) {
                const int x = p * NT + tid, idx = x >> 4, sl = x & 15;
                float t = v[p];
                t += dpp_row<0xB1>(t);
                t += dpp_row<0x4E>(t);
                t += dpp_row<0x141>(t);
                t += dpp_row<0x140>(t);
                if (idx < n_items && sl == 0) finish_item(idx, t);
            }
        }
    } else {
        for (int g = tid; g < P.S * n_items && ok; g += NT) {
            uint32_t spins = 0;
            for (;;) {
                const unsigned long long x = granule_load(xg + g);
                if ((uint32_t)(x >> 32) == tag) {
                    xin[g] = __uint_as_float((uint32_t)x);
                    break;
                }
                if (++spins > kSpinLimit) {
                    ok = false;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
    }
    if (!ok) {
        flags[1] = 1;
        __hip_atomic_store(status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    MC_STAMP(19);
    if (flags[1]) return false;
    if (!fast) {
        for (int idx = tid; idx < n_items; idx += NT) {
            float v = xin[idx];
            for (int sl = 1; sl < P.S; ++sl) v += xin[sl * n_items + idx];
            finish_item(idx, v);
        }
        __syncthreads();
    }
    MC_STAMP(21);
    return true;
}

// Kinetic partial over the private slots [0, Ps) of every chain; wave w
// reduces chains 2w and 2w+1 (fixed order).  With final_kick the momentum is
// first advanced by the last half kick (p + h_b * g).
template <int NB>
MC_DEV void sl_kinetic(const float* pm, const float* g2, uint32_t gmask, const float* cs,
                       bool final_kick, int Ps, int Lp, float* out, int tid) {
    const int b0 = 2 * (tid >> 6), j = tid & 63;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const int b = b0 + c;
        const float h = cs[CS_H * NB + b];
        const int go = slot_of(gmask, b, NB, Lp);
        float x = 0.0f;
        for (int k = j; k < Ps; k += kSlLanes) {
            float p = pm[b * Lp + k];
            if (final_kick) p = p + h * g2[go + k];
            x += p * p;
        }
        x = wave_sum(x);
        if (j == 0) out[b] = x;
    }
}

// ---------------------------------------------------------------------------
// the sampler
// ---------------------------------------------------------------------------
template <int NB>
__global__ void __launch_bounds__(512)
k_hmc_sl(SlCtx P, RunArgs A, int64_t chain_base, int64_t n_groups, mc_chain_scalars* scal,
         float* st_q, float* st_g, float* samples, TraceDev tr, unsigned long long* xch,
         int* status) {
    constexpr int NT = kSlLanes * NB / 2;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    if (A.fault && blockIdx.x == gridDim.x - 1) return;  // test hook: never publishes
    const mc_run_config& cfg = A.cfg;
    const int tid = threadIdx.x;
    const int S = P.S, Lp = P.Lp, D = P.D;
    // workgroup -> (chain block, slice); blocks of one chain block share an
    // XCD when the grid allows it (speed only, nothing depends on placement)
    int64_t grp;
    int slice;
    {
        const int64_t w = blockIdx.x, nwg = gridDim.x;
        if (nwg % 8 == 0 && (nwg / 8) % S == 0) {
            const int64_t x = w & 7, r = w >> 3;
            grp = x * ((nwg / 8) / S) + r / S;
            slice = (int)(r % S);
        } else {
            grp = w / S;
            slice = (int)(w % S);
        }
    }
    const int64_t C = cfg.num_chains;
    const int64_t cbase = chain_base + grp * NB;  // first chain of the block

    const SlLayout<NB> Lo(P);
    float* sd = smem + Lo.sd;
    float* q2 = smem + Lo.q2;
    float* g2 = smem + Lo.g2;
    float* pm = smem + Lo.pm;
    float* vpart = smem + Lo.vpart;
    float* sacc = smem + Lo.sacc;
    float* xin = smem + Lo.xin;
    float* ob = smem + Lo.ob;
    float4* der = (float4*)(smem + Lo.der);
    float* sst = smem + Lo.sst;
    float* cs = smem + Lo.cs;
    double* eps = (double*)cs;  // CS_EPS: NB doubles = 2*NB floats
    int* ci = (int*)cs;
    int* flags = (int*)(cs + CS_COUNT * NB);  // [0] current-buffer mask, [1] abort

    const int64_t* blk = P.blocks + 4 * (int64_t)slice;
    const int nact = (int)blk[3];
    const int64_t doff = blk[0];
    const int dlen = (int)blk[1];
    const int Ps = (int)blk[2];
    const int32_t* gmap = P.gidx + (int64_t)slice * Lp;

    MC_STAMP_INIT
    // ---- launch prologue: slice block and chain state into LDS ----------------
    for (int i = tid; 4 * i < dlen; i += NT)
        *(float4*)(sd + 4 * i) = *(const float4*)(P.data + doff + 4 * i);
    for (int i = tid; i < NB * (P.Dsh + 1); i += NT) sacc[i] = 0.0f;
    for (int idx = tid; idx < NB * Lp; idx += NT) {
        const int b = idx / Lp, k = idx - b * Lp;
        const int64_t c = min(cbase + b, C - 1);
        const int g = gmap[k];
        q2[idx] = g >= 0 ? st_q[c * D + g] : 0.0f;  // buffer 0 of chain b
        g2[idx] = g >= 0 ? st_g[c * D + g] : 0.0f;
        q2[NB * Lp + idx] = 0.0f;
        g2[NB * Lp + idx] = 0.0f;
        pm[idx] = 0.0f;
    }
    if (tid < NB) {
        const int64_t c = min(cbase + tid, C - 1);
        eps[tid] = scal[c].step_size;
        cs[CS_LP * NB + tid] = scal[c].logp;
        ci[CS_NACC * NB + tid] = scal[c].n_accept;
        ci[CS_NTOT * NB + tid] = scal[c].n_total;
        ci[CS_WACC * NB + tid] = scal[c].warmup_accept;
        ci[CS_WTOT * NB + tid] = scal[c].warmup_total;
    }
    if (tid == 0) {
        flags[0] = 0;
        flags[1] = 0;
    }
    __syncthreads();

    const int L = cfg.num_leapfrog_steps;
    const int nI = P.nitems;
    uint32_t epoch = 0;
    const int64_t it_end = cfg.iter_begin + cfg.iter_count;
    for (int64_t it = cfg.iter_begin; it < it_end; ++it) {
        const bool warm = it < cfg.num_warmup;
        if (tid < NB) {
            if (it == cfg.num_warmup) {  // hmc.py:175-180
                ci[CS_WACC * NB + tid] = ci[CS_NACC * NB + tid];
                ci[CS_WTOT * NB + tid] = ci[CS_NTOT * NB + tid];
                ci[CS_NACC * NB + tid] = 0;
                ci[CS_NTOT * NB + tid] = 0;
            }
            cs[CS_H * NB + tid] = (float)(0.5 * eps[tid]);
            cs[CS_E * NB + tid] = (float)eps[tid];
        }
        // momentum: parameter g takes normal g % 4 of Philox block g / 4
        for (int idx = tid; idx < NB * Lp; idx += NT) {
            const int b = idx / Lp, k = idx - b * Lp;
            const int g = gmap[k];
            float z = 0.0f;
            if (g >= 0) {
                const uint32_t chain_id = (uint32_t)(cfg.chain_offset + min(cbase + b, C - 1));
                const mc_u32x4 r = mc_draw(cfg.seed, chain_id, (uint32_t)it, MC_RNG_TAG_MOMENTUM,
                                           0, (uint32_t)(g >> 2));
                float z0, z1;
                if ((g & 3) < 2) mc_box_muller(r.x, r.y, &z0, &z1);
                else mc_box_muller(r.z, r.w, &z0, &z1);
                z = (g & 1) ? z1 : z0;
            }
            pm[idx] = z;
        }
        __syncthreads();
        uint32_t cur = (uint32_t)flags[0];
        sl_kinetic<NB>(pm, g2, cur, cs, false, Ps, Lp, ob + (P.Dsh + 1) * NB, tid);
        if (tid < NB) {
            // the shared parameters' part of K0 (every slice holds them)
            float k0s = 0.0f;
            for (int jj = 0; jj < P.Dsh; ++jj) {
                const float p = pm[tid * Lp + P.Pmax + jj];
                k0s += p * p;
            }
            cs[CS_K0S * NB + tid] = k0s;
            ob[(P.Dsh + 2) * NB + tid] = 0.0f;
        }
        __syncthreads();

        const uint32_t prop = ~cur;  // proposal buffer of every chain
        SlPoll poll;
        auto xbuf = [&](uint32_t ep) {
            return xch + ((int64_t)(ep & 1) * n_groups + grp) * S * nI * NB;
        };
        // position update of slots [k_lo, k_hi) of every chain: step 0 starts
        // from the current point, later steps update the proposal in place
        // (each slot is read and written by one thread)
        auto advance = [&](int l, int k_lo, int k_hi) {
            const uint32_t from = (l == 0) ? cur : prop;
            const int w = k_hi - k_lo;
            for (int idx = tid; idx < NB * w; idx += NT) {
                const int b = idx / w, k = k_lo + (idx - b * w);
                const int src = slot_of(from, b, NB, Lp) + k;
                const int dst = slot_of(prop, b, NB, Lp) + k;
                const float h = cs[CS_H * NB + b], e = cs[CS_E * NB + b];
                const float gj = g2[src];
                float pj = pm[b * Lp + k];
                if (l > 0) pj = pj + h * gj;  // second half kick of step l-1
                pj = pj + h * gj;             // first half kick of step l
                pm[b * Lp + k] = pj;
                q2[dst] = q2[src] + e * pj;
                g2[dst] = 0.0f;
            }
        };
        if (L == 0) {
            ++epoch;
            if (tid < NB) ob[tid] = 0.0f;
            __syncthreads();
            sl_publish<NB>(P, slice, xbuf(epoch), epoch, ob, tid);
            sl_poll_issue<NB>(P, xbuf(epoch), poll, tid);
            if (!sl_collect<NB>(P, xbuf(epoch), epoch, g2, prop, xin, sst, cs, flags, status,
                                poll, tid))
                return;
        }
        MC_STAMP_DECL
        for (int l = 0; l < L; ++l) {
            // private slots of step l > 0 were advanced while the previous
            // exchange was in flight (their gradients were complete)
            if (l == 0) advance(0, 0, Lp);
            else advance(l, P.Pmax, P.Pmax + P.Dsh);
            __syncthreads();
            MC_STAMP(0);
            sl_eval<NB>(P, slice, nact, sd, q2, g2, prop, vpart, sacc, der, sst, ob, tid);
            MC_STAMP(1);
            if (l == L - 1) {
                sl_kinetic<NB>(pm, g2, prop, cs, true, Ps, Lp, ob + (P.Dsh + 2) * NB, tid);
                __syncthreads();
            }
            ++epoch;
            sl_publish<NB>(P, slice, xbuf(epoch), epoch, ob, tid);
            if (l + 1 < L) advance(l + 1, 0, P.Pmax);  // overlaps the records' flight
            sl_poll_issue<NB>(P, xbuf(epoch), poll, tid);
            if (!sl_collect<NB>(P, xbuf(epoch), epoch, g2, prop, xin, sst, cs, flags, status,
                                poll, tid))
                return;
            MC_STAMP(2);
        }

        // ---- accept / adapt (identical in every slice of the block) ----------
        if (tid < 64) {
            bool acc = false;
            if (tid < NB) {
                const int b = tid;
                const int go = slot_of(prop, b, NB, Lp);
                const float h = cs[CS_H * NB + b];
                const float k0s = cs[CS_K0S * NB + b];
                float k1s = 0.0f;
                for (int jj = 0; jj < P.Dsh; ++jj) {
                    const float p = pm[b * Lp + P.Pmax + jj];
                    const float p1 = (L > 0) ? p + h * g2[go + P.Pmax + jj] : p;
                    k1s += p1 * p1;
                }
                const float lp = cs[CS_LP * NB + b];
                const float H0 = -lp + 0.5f * (cs[CS_K0 * NB + b] + k0s);
                const float lpn = (L > 0) ? cs[CS_LPN * NB + b] : lp;
                const float K1 = (L > 0) ? cs[CS_K1 * NB + b] : cs[CS_K0 * NB + b];
                const float H1 = -lpn + 0.5f * (K1 + (L > 0 ? k1s : k0s));
                const float ratio = -(H1 - H0);
                const int64_t c = cbase + b;
                const uint32_t chain_id = (uint32_t)(cfg.chain_offset + min(c, C - 1));
                const mc_u32x4 ru =
                    mc_draw(cfg.seed, chain_id, (uint32_t)it, MC_RNG_TAG_ACCEPT, 0, 0);
                const float logu = mc_logf_u01(mc_u01_f32(ru.x));
                const bool accepted = logu < ratio;
                acc = accepted && L > 0;
                if (acc) cs[CS_LP * NB + b] = lpn;
                const int n_acc = ci[CS_NACC * NB + b] + (accepted ? 1 : 0);
                const int n_tot = ci[CS_NTOT * NB + b] + 1;
                ci[CS_NACC * NB + b] = n_acc;
                ci[CS_NTOT * NB + b] = n_tot;
                const double eps_used = eps[b];
                if (warm && cfg.adapt_step_size && it > 10) {
                    const double rate = (double)n_acc / (double)n_tot;
                    eps[b] = (rate < cfg.target_accept) ? eps_used * 0.95 : eps_used * 1.05;
                }
                if (slice == 0 && c < C) {
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
            }
            const unsigned long long bal = __ballot(acc);
            if (tid == 0) flags[0] = (int)((uint32_t)flags[0] ^ (uint32_t)bal);
        }
        __syncthreads();
        cur = (uint32_t)flags[0];
        if (!warm && samples != nullptr) {
            const int64_t s = it - cfg.num_warmup - cfg.sample_begin;
            if (s >= 0 && s < cfg.sample_capacity) {
                for (int idx = tid; idx < NB * Lp; idx += NT) {
                    const int b = idx / Lp, k = idx - b * Lp;
                    const int g = gmap[k];
                    const int64_t c = cbase + b;
                    const bool mine = k < Ps || (slice == 0 && k >= P.Pmax);
                    if (g >= 0 && mine && c < C)
                        samples[(c * cfg.sample_capacity + s) * (int64_t)D + g] =
                            q2[slot_of(cur, b, NB, Lp) + k];
                }
            }
        }
    }

    // ---- launch epilogue: state back to HBM -------------------------------------
    const uint32_t cur = (uint32_t)flags[0];
    for (int idx = tid; idx < NB * Lp; idx += NT) {
        const int b = idx / Lp, k = idx - b * Lp;
        const int g = gmap[k];
        const int64_t c = cbase + b;
        const bool mine = k < Ps || (slice == 0 && k >= P.Pmax);
        if (g >= 0 && mine && c < C) {
            st_q[c * D + g] = q2[slot_of(cur, b, NB, Lp) + k];
            st_g[c * D + g] = g2[slot_of(cur, b, NB, Lp) + k];
        }
    }
    MC_STAMP_FLUSH
    if (slice == 0 && tid < NB && cbase + tid < C) {
        mc_chain_scalars& sc = scal[cbase + tid];
        sc.logp = cs[CS_LP * NB + tid];
        sc.step_size = eps[tid];
        sc.n_accept = ci[CS_NACC * NB + tid];
        sc.n_total = ci[CS_NTOT * NB + tid];
        sc.warmup_accept = ci[CS_WACC * NB + tid];
        sc.warmup_total = ci[CS_WTOT * NB + tid];
        sc.n_grad += cfg.iter_count * (int64_t)L;
    }
}

}  // namespace mc
