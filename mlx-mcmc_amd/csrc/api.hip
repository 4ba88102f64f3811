// api.hip — libmcmc355.so: program builder, slice / lane planners, tape,
// state and diagnostics launches and the rest of the C-ABI of
// include/mcmc355.h (the sampler launches are in run_hmc.hip, run_mh.hip,
// run_nuts.hip).
#include "host.h"
#include "jit.h"

static thread_local bool g_program_host_only;
#include "diag.h"  // (non-template kernels: this unit only)
static bool is_vec_kind(int k) { return k == MC_OP_DATA || k == MC_OP_PVEC || k == MC_OP_GATHER; }
static bool is_acc_vec(int k) { return k == MC_OP_PVEC || k == MC_OP_GATHER; }

// f32 constants exactly as the reference forms them (normal.py:31,
// halfnormal.py:31-32): log_norm = -0.5 * f32 log(f32(2*pi)), log2 = f32 log 2.
static float c_log_norm() {
    const float two_pi = (float)(2.0 * 3.141592653589793);
    const float l = (float)std::log((double)two_pi);
    return -0.5f * l;
}
static float c_log2() { return (float)std::log(2.0); }
static float dist_c0(int dist) {
    if (dist == MC_DIST_NORMAL) return c_log_norm();
    if (dist == MC_DIST_HALFNORMAL) return c_log2() + c_log_norm();
    return 0.0f;
}

static int choose_wpc(int64_t max_n) {
    if (max_n <= 512) return 1;
    if (max_n <= 16384) return 4;
    return 8;
}

// Segment-tiled layout of a term sorted by its primary (non-injective) gather
// index; see DevTerm in internal.h.  Runs of equal index ("segments") are
// split into at most ceil(len / Lt) near-equal virtual segments so that a
// chain group of T threads has ~2T lanes of work even for few, long groups;
// with >= 2T segments nothing is split and each lane writes its group's
// gradient directly.
// prim_pool: index-pool offset of the sorted primary index; others: the
// term's other vector operands, tiled beside it (DATA copied, PVEC turned
// into identity gathers, GATHER indices copied); tsplit: with fewer groups
// than that, runs are split into ~tsplit virtual segments; nprim: partials per
// virtual segment (an expression term keeps one per gathered leaf), so that
// nprim x (virtual segments) fit the evaluator's 4T segment-partial floats.
static int build_segments_ops(DevTerm& dt, int64_t prim_pool, const std::vector<DevOperand*>& others,
                              int64_t tsplit, int nprim, std::vector<float>& dpool,
                              std::vector<int32_t>& ipool, int T) {
    const int64_t n = dt.n;
    const int64_t ip = prim_pool;
    std::vector<int64_t> sstart;
    std::vector<int32_t> sk;
    for (int64_t i = 0; i < n; ++i)
        if (i == 0 || ipool[ip + i] != ipool[ip + i - 1]) {
            sstart.push_back(i);
            sk.push_back(ipool[ip + i]);
        }
    const int64_t G = (int64_t)sstart.size();
    sstart.push_back(n);
    // split only when there are fewer groups than tsplit (then <= 2 tsplit
    // virtual segments); otherwise each lane owns whole groups
    struct V {
        int32_t k;
        int64_t start;
        int32_t len;
    };
    std::vector<V> vs;
    std::vector<int32_t> comb;
    bool split = false;
    auto plan_runs = [&](int64_t Lt) {
        vs.clear();
        comb.clear();
        split = false;
        for (int64_t g = 0; g < G; ++g) {
            const int64_t len = sstart[g + 1] - sstart[g];
            const int64_t pieces = (Lt == INT64_MAX) ? 1 : (len + Lt - 1) / Lt;
            if (pieces > 1) split = true;
            const int64_t base = len / pieces, rem = len % pieces;
            comb.push_back(sk[g]);
            comb.push_back((int32_t)vs.size());
            comb.push_back((int32_t)pieces);
            int64_t st = sstart[g];
            for (int64_t pc = 0; pc < pieces; ++pc) {
                const int64_t pl = base + (pc < rem ? 1 : 0);
                if (pl > INT32_MAX) return fail(MC_ERR_UNSUPPORTED, "segment too long");
                vs.push_back({sk[g], st, (int32_t)pl});
                st += pl;
            }
        }
        return MC_OK;
    };
    int rc = plan_runs((G >= tsplit) ? INT64_MAX : std::max<int64_t>(1, (n + tsplit - 1) / tsplit));
    if (rc) return rc;
    // the split's partial rows (nprim per virtual segment) must fit the
    // evaluator's 4T floats of segment scratch; tsplit keeps them within it,
    // and should a plan not, the runs stay whole (no hard error)
    if (split && (int64_t)vs.size() * nprim > 4 * (int64_t)T) {
        rc = plan_runs(INT64_MAX);
        if (rc) return rc;
    }
    const int64_t nv = (int64_t)vs.size();
    const int64_t ntiles = (nv + 63) / 64;
    std::vector<int32_t> tiles(3 * ntiles), lanes(2 * nv);
    int64_t total = 0;
    for (int64_t t = 0; t < ntiles; ++t) {
        int32_t lmax = 0, lmin = INT32_MAX;
        for (int l = 0; l < 64; ++l) {
            const int64_t v = t * 64 + l;
            if (v >= nv) break;  // lanes past the end are masked off in-kernel
            lmax = std::max(lmax, vs[v].len);
            lmin = std::min(lmin, vs[v].len);
        }
        const int32_t lpad = (lmax + 3) / 4 * 4;
        if (total > INT32_MAX - 64 * (int64_t)lpad)
            return fail(MC_ERR_UNSUPPORTED, "segmented term too large");
        tiles[3 * t] = (int32_t)total;
        tiles[3 * t + 1] = lpad;
        tiles[3 * t + 2] = lmin;
        total += 64 * (int64_t)lpad;
    }
    for (int64_t v = 0; v < nv; ++v) {
        lanes[2 * v] = vs[v].k;
        lanes[2 * v + 1] = vs[v].len;
    }
    // parameter slices become identity gathers so that they can be tiled too
    for (DevOperand* dp : others) {
        DevOperand& d = *dp;
        if (d.kind != MC_OP_PVEC) continue;
        const int64_t base = (int64_t)ipool.size();
        for (int64_t i = 0; i < n; ++i) ipool.push_back((int32_t)i);
        d.kind = MC_OP_GATHER;
        d.pool = base;
        d.unique = 1;
    }
    // tiled copies of every other vector operand (and an affine loc's data x)
    for (DevOperand* dp : others) {
        DevOperand& d = *dp;
        if (d.kind != MC_OP_DATA && d.kind != MC_OP_GATHER) continue;
        if (d.kind == MC_OP_DATA) {
            while (dpool.size() % 64) dpool.push_back(0.0f);
            const int64_t base = (int64_t)dpool.size();
            dpool.resize(base + total, 0.0f);
            for (int64_t v = 0; v < nv; ++v) {
                const int64_t t = v / 64, l = v % 64;
                for (int32_t u = 0; u < vs[v].len; ++u)
                    dpool[base + tiles[3 * t] + (u >> 2) * 256 + l * 4 + (u & 3)] =
                        dpool[d.pool + vs[v].start + u];
            }
            d.pool = base;
        } else {
            while (ipool.size() % 64) ipool.push_back(0);
            const int64_t base = (int64_t)ipool.size();
            ipool.resize(base + total, 0);
            for (int64_t v = 0; v < nv; ++v) {
                const int64_t t = v / 64, l = v % 64;
                for (int32_t u = 0; u < vs[v].len; ++u)
                    ipool[base + tiles[3 * t] + (u >> 2) * 256 + l * 4 + (u & 3)] =
                        ipool[d.pool + vs[v].start + u];
            }
            d.pool = base;
        }
    }
    dt.ntiles = (int32_t)ntiles;
    dt.nvirt = (int32_t)nv;
    dt.ncomb = split ? (int32_t)G : 0;
    dt.tile_base = (int64_t)ipool.size();
    ipool.insert(ipool.end(), tiles.begin(), tiles.end());
    while (ipool.size() % 2) ipool.push_back(0);  // lane records are read as int2
    dt.lane_base = (int64_t)ipool.size();
    ipool.insert(ipool.end(), lanes.begin(), lanes.end());
    dt.comb_base = (int64_t)ipool.size();
    if (split) ipool.insert(ipool.end(), comb.begin(), comb.end());
    return MC_OK;
}

static int build_segments(DevTerm& dt, std::vector<float>& dpool, std::vector<int32_t>& ipool,
                          int T) {
    const int a = dt.primary;
    std::vector<DevOperand*> others;
    for (int b = 0; b < 3; ++b)
        if (b != a) others.push_back(&dt.op[b]);
    if (dt.affine) others.push_back(&dt.ax);
    return build_segments_ops(dt, dt.op[a].pool, others, T, 1, dpool, ipool, T);
}

// ---------------------------------------------------------------------------
// sliced layout planner (sliced.h)
// ---------------------------------------------------------------------------
static void free_slices(SlicePlan& P) {
    if (P.d_terms) (void)hipFree(P.d_terms);
    if (P.d_sterms) (void)hipFree(P.d_sterms);
    if (P.d_data) (void)hipFree(P.d_data);
    if (P.d_index) (void)hipFree(P.d_index);
    if (P.d_blocks) (void)hipFree(P.d_blocks);
    if (P.d_gidx) (void)hipFree(P.d_gidx);
    P = SlicePlan();
}


static int sl_lds_bytes(const mc_program* p, int nb) {
    const SlCtx c = slctx_of(p);
    return 4 * (nb == 16 ? SlLayout<16>(c).total : SlLayout<8>(c).total);
}


static int64_t pp_index(const DevTerm& t, int a, int64_t i, const std::vector<int32_t>& ip) {
    const DevOperand& o = t.op[a];
    return o.kind == MC_OP_PVEC ? (int64_t)o.poff + i : (int64_t)o.poff + ip[o.pool + i];
}

// The parameter / element partition plan_slices computes, kept for the
// lane-resident planner (plan_lanes).
struct SlPartition {
    std::vector<int> shxf;                // per shared ordinal: mc_transform_kind
    std::vector<int> sterm_raw;           // per scalar term: LrSterm::raw bits
    std::vector<int> ppr;                 // per term: slot of its per-element parameter, or -1
    std::vector<char> shared, scalar;     // per parameter / per term
    std::vector<int> jsh;                 // per parameter: shared ordinal, or -1
    std::vector<std::vector<int>> priv;   // per slice: its private parameters
    std::vector<int> shl;                 // shared parameters by ordinal
    std::vector<std::vector<std::vector<int64_t>>> elems;  // [slice][term] element ids
};


static int plan_slices(mc_program* p, int S, SlicePlan& P, SlPartition* part = nullptr) {
    const std::vector<DevTerm>& raw = p->raw;
    if (has_expr(p) && !expr_lanes_ok(p))
        return fail(MC_ERR_UNSUPPORTED, "expression terms other than data / broadcast "
                    "parameter / constant leaves (a parameter vector, a gather, more than %d "
                    "data leaves) run on the chain-per-workgroup kernels (not sliceable)",
                    kLrExprData);
    if (has_affine(p) && !affine_lanes_ok(p))
        return fail(MC_ERR_UNSUPPORTED, "affine loc operands other than `loc + b * x` over "
                    "data x (x a parameter vector, a non-Normal term, a per-element scale) run "
                    "on the chain-per-workgroup kernels (not sliceable)");
    const bool xf = has_transform(p);
    if (xf && !transform_on_shared_only(p))
        return fail(MC_ERR_UNSUPPORTED, "transformed parameter operands (mx.exp / mx.log) of "
                    "per-element parameters, and identity terms over them, run on the "
                    "chain-per-workgroup kernels (not sliceable)");
    const std::vector<float>& dp = p->h_data;
    const std::vector<int32_t>& ip = p->h_index;
    const int D = p->D;
    const int nT = (int)raw.size();
    const int T = kSlLanes;  // run slots per chain pair
    std::vector<int> ppr(nT, -1);
    for (int t = 0; t < nT; ++t)
        for (int a = 0; a < 3; ++a)
            if (raw[t].op[a].kind == MC_OP_PVEC || raw[t].op[a].kind == MC_OP_GATHER) {
                if (ppr[t] >= 0)
                    return fail(MC_ERR_UNSUPPORTED,
                                "term %d has two per-element parameter operands: not sliceable", t);
                ppr[t] = a;
            }
    // shared (broadcast) parameters and the private parameters' costs
    std::vector<char> shared(D, 0);
    for (const DevTerm& t : raw) {
        for (int a = 0; a < 3; ++a)
            if (t.op[a].kind == MC_OP_PSCALAR) shared[t.op[a].poff] = 1;
        if (t.affine && t.ab.kind == MC_OP_PSCALAR) shared[t.ab.poff] = 1;  // the slope
        if (t.dist == MC_DIST_EXPR)  // an expression's broadcast leaves
            for (int k = 0; k < t.expr_n; ++k) {
                const DevExprNode& d = p->nodes[t.expr_base + k];
                if (d.op == MC_EX_LEAF && d.leaf.kind == MC_OP_PSCALAR) shared[d.leaf.poff] = 1;
            }
    }
    std::vector<int64_t> cost(D, 1);
    for (int t = 0; t < nT; ++t)
        if (ppr[t] >= 0)
            for (int64_t i = 0; i < raw[t].n; ++i) {
                const int64_t j = pp_index(raw[t], ppr[t], i, ip);
                if (!shared[j]) cost[j] += 1;
            }
    int64_t total = 0;
    for (int j = 0; j < D; ++j)
        if (!shared[j]) total += cost[j];
    std::vector<int> owner(D, 0), lidx(D, 0), jsh(D, -1);
    std::vector<std::vector<int>> priv(S);
    std::vector<int> shl;
    {
        int64_t run = 0;
        for (int j = 0; j < D; ++j) {
            if (shared[j]) {
                jsh[j] = (int)shl.size();
                shl.push_back(j);
                continue;
            }
            const int s = (int)std::min<int64_t>(S - 1, (2 * run + cost[j]) * S / (2 * std::max<int64_t>(total, 1)));
            owner[j] = s;
            lidx[j] = (int)priv[s].size();
            priv[s].push_back(j);
            run += cost[j];
        }
    }
    // the transform of each shared parameter: every transformed use agrees;
    // terms that are not scalar read it through the transform only (a scalar
    // term may also read the raw parameter: the raw bits below)
    std::vector<int> shxf(shl.size(), MC_XF_NONE);
    if (xf) {
        for (const DevTerm& t : raw)
            for (int a = 0; a < 3; ++a) {
                const DevOperand& o = t.op[a];
                if (o.kind != MC_OP_PSCALAR || o.xf == MC_XF_NONE) continue;
                int& x = shxf[jsh[o.poff]];
                if (x != MC_XF_NONE && x != o.xf)
                    return fail(MC_ERR_UNSUPPORTED, "a broadcast parameter read through two "
                                "different transforms (mx.exp and mx.log): not sliceable");
                x = o.xf;
            }
        for (int t = 0; t < nT; ++t) {
            bool sc = raw[t].dist != MC_DIST_EXPR;
            for (int a = 0; a < 3; ++a) {
                const int k = raw[t].op[a].kind;
                if (k != MC_OP_CONST && k != MC_OP_PSCALAR && k != MC_OP_NONE) sc = false;
            }
            if (sc) continue;
            for (int a = 0; a < 3; ++a) {
                const DevOperand& o = raw[t].op[a];
                if (o.kind == MC_OP_PSCALAR && o.xf != shxf[jsh[o.poff]])
                    return fail(MC_ERR_UNSUPPORTED, "a broadcast parameter read both raw and "
                                "through mx.exp / mx.log by per-element terms: not sliceable");
            }
            // an expression reads a transformed broadcast parameter only
            // through the matching node (mx.exp(log_sigma) for an exp
            // transform): the lane code reads the transformed value there and
            // its cotangent is the value's (jit.hip gen_lane_term)
            if (raw[t].dist == MC_DIST_EXPR) {
                const DevExprNode* N = p->nodes.data() + raw[t].expr_base;
                for (int k = 0; k < raw[t].expr_n; ++k) {
                    if (N[k].op == MC_EX_LEAF) continue;
                    const int args[3] = {N[k].a, N[k].b, N[k].c};
                    for (int x = 0; x < 3; ++x) {
                        const int a = args[x];
                        if (a < 0 || N[a].op != MC_EX_LEAF || N[a].leaf.kind != MC_OP_PSCALAR) continue;
                        const int xfk = shxf[jsh[N[a].leaf.poff]];
                        if (xfk == MC_XF_NONE) continue;
                        const int want = xfk == MC_XF_EXP ? MC_EX_EXP : MC_EX_LOG;
                        if (N[k].op != want || x != 0)
                            return fail(MC_ERR_UNSUPPORTED, "a broadcast parameter read raw by an "
                                        "expression and through mx.exp / mx.log by a fused term: "
                                        "not sliceable");
                    }
                }
            }
        }
    }
    P.S = S;
    P.Dsh = (int)shl.size();
    P.Pmax = 0;
    for (int s = 0; s < S; ++s) P.Pmax = std::max<int>(P.Pmax, (int)priv[s].size());
    P.Lp = std::max(4, (P.Pmax + P.Dsh + 3) / 4 * 4);
    P.nitems = P.Dsh + 3;
    P.gidx.assign((size_t)S * P.Lp, -1);
    for (int s = 0; s < S; ++s)
        for (size_t k = 0; k < priv[s].size(); ++k) P.gidx[(size_t)s * P.Lp + k] = priv[s][k];
    for (int s = 0; s < S; ++s)
        for (int j = 0; j < P.Dsh; ++j) P.gidx[(size_t)s * P.Lp + P.Pmax + j] = shl[j];
    P.terms.assign((size_t)S * nT, SlTerm());
    P.blocks.assign(4 * (size_t)S, 0);
    P.sdata_floats = 0;

    // operand kinds of a slice term (SK_*)
    auto make_slterm = [&](const DevTerm& rt, int t) {
        SlTerm st;
        std::memset(&st, 0, sizeof(st));
        st.dist = rt.dist;
        st.pp = ppr[t];
        st.weight = rt.weight;
        st.c0 = rt.c0;
        if (rt.op[2].kind == MC_OP_CONST) {
            const float c = rt.op[2].cval;
            st.clogs = (float)std::log((double)c);
            st.cinv = 1.0f / c;
            st.cinv2 = 1.0f / (c * c);
        }
        for (int a = 0; a < 3; ++a) {
            const DevOperand& o = rt.op[a];
            st.kloc[a] = -1;
            switch (o.kind) {
                case MC_OP_CONST: st.kind[a] = SK_CONST; st.cval[a] = o.cval; break;
                case MC_OP_PSCALAR:
                    st.kind[a] = SK_SHARED;
                    st.jsh[a] = jsh[o.poff];
                    st.kloc[a] = P.Pmax + jsh[o.poff];
                    break;
                case MC_OP_DATA: st.kind[a] = SK_DATA; break;
                case MC_OP_PVEC:
                case MC_OP_GATHER: st.kind[a] = SK_PP; break;
                default: st.kind[a] = SK_NONE; break;
            }
        }
        // moment sums for Normal / HalfNormal with a broadcast scale, else
        // the per-element formula
        st.mode = (st.kind[2] == SK_DATA || st.kind[2] == SK_PP ||
                   (rt.dist != MC_DIST_NORMAL && rt.dist != MC_DIST_HALFNORMAL)) ? 1 : 0;
        st.clg = rt.clg;
        return st;
    };
    // scalar terms (only constants and broadcast parameters): evaluated once
    // per chain after every exchange, in every slice, not split into slices
    std::vector<char> scalar(nT, 0);
    std::vector<int> sterm_raw;
    P.sterms.clear();
    for (int t = 0; t < nT; ++t) {
        bool sc = raw[t].dist != MC_DIST_EXPR;  // (an expression term is sliced by element)
        for (int a = 0; a < 3; ++a) {
            const int k = raw[t].op[a].kind;
            if (k != MC_OP_CONST && k != MC_OP_PSCALAR && k != MC_OP_NONE) sc = false;
        }
        scalar[t] = sc;
        if (sc) {
            SlTerm st = make_slterm(raw[t], t);
            if (raw[t].n > INT32_MAX) return fail(MC_ERR_UNSUPPORTED, "scalar term too long");
            st.niter = (int32_t)raw[t].n;  // element count
            P.sterms.push_back(st);
            int rb = 0;
            for (int a = 0; a < 3; ++a) {
                const DevOperand& o = raw[t].op[a];
                if (o.kind == MC_OP_PSCALAR && o.xf == MC_XF_NONE && shxf[jsh[o.poff]] != MC_XF_NONE)
                    rb |= 1 << a;
            }
            sterm_raw.push_back(rb);
        }
    }

    // element -> slice
    std::vector<std::vector<std::vector<int64_t>>> elems(S, std::vector<std::vector<int64_t>>(nT));
    for (int t = 0; t < nT; ++t) {
        if (scalar[t]) continue;
        const int64_t n = raw[t].n;
        for (int64_t i = 0; i < n; ++i) {
            int s;
            if (ppr[t] >= 0) {
                const int64_t j = pp_index(raw[t], ppr[t], i, ip);
                s = shared[j] ? 0 : owner[j];
            } else if (n < 256) {
                s = t % S;  // small terms go whole to one slice, round robin
            } else {
                s = (int)(i * S / n);
            }
            elems[s][t].push_back(i);
        }
    }
    if (part) {
        part->shxf = shxf;
        part->sterm_raw = sterm_raw;
        part->ppr = ppr;
        part->shared = shared;
        part->scalar = scalar;
        part->jsh = jsh;
        part->priv = priv;
        part->shl = shl;
        part->elems = elems;
    }

    struct Run {
        int32_t k;
        int64_t first;
        int32_t len;
    };
    for (int s = 0; s < S; ++s) {
        while (P.data.size() % 4) P.data.push_back(0.0f);
        const int64_t blk0 = (int64_t)P.data.size();
        // ---- runs of every term of this slice ----
        std::vector<std::vector<Run>> runs(nT);
        std::vector<char> direct(nT, 0);
        for (int t = 0; t < nT; ++t) {
            const DevTerm& rt = raw[t];
            const std::vector<int64_t>& E = elems[s][t];
            const int64_t nE = (int64_t)E.size();
            std::vector<Run>& R = runs[t];
            if (nE > 0 && ppr[t] >= 0) {
                std::vector<Run> nat;
                for (int64_t e = 0; e < nE; ++e) {
                    const int64_t j = pp_index(rt, ppr[t], E[e], ip);
                    const int32_t k = shared[j] ? P.Pmax + jsh[j] : lidx[j];
                    if (e > 0 && nat.back().k == k && nat.back().len < INT32_MAX) {
                        ++nat.back().len;
                    } else {
                        nat.push_back({k, e, 1});
                    }
                }
                // few long runs: split them so that the lanes get near-equal
                // work (m runs per lane); otherwise keep whole runs
                int64_t Lt = INT64_MAX;
                const int64_t nn = (int64_t)nat.size();
                if (nn <= 4 * T) {
                    const int64_t m = (nn + T - 1) / T;
                    int64_t lo = 1, hi = 1;
                    for (const Run& r : nat) hi = std::max<int64_t>(hi, r.len);
                    while (lo < hi) {
                        const int64_t mid = (lo + hi) / 2;
                        int64_t pieces = 0;
                        for (const Run& r : nat) pieces += (r.len + mid - 1) / mid;
                        if (pieces <= T * m) hi = mid; else lo = mid + 1;
                    }
                    Lt = lo;
                }
                for (const Run& r : nat) {
                    const int64_t pieces = (Lt == INT64_MAX) ? 1 : (r.len + Lt - 1) / Lt;
                    const int64_t base = r.len / pieces, rem = r.len % pieces;
                    int64_t f = r.first;
                    for (int64_t pc = 0; pc < pieces; ++pc) {
                        const int32_t pl = (int32_t)(base + (pc < rem ? 1 : 0));
                        R.push_back({r.k, f, pl});
                        f += pl;
                    }
                }
                std::vector<int32_t> ks;
                for (const Run& r : R) ks.push_back(r.k);
                std::sort(ks.begin(), ks.end());
                direct[t] = std::adjacent_find(ks.begin(), ks.end()) == ks.end();
            } else if (nE > 0) {
                const int64_t nch = std::min<int64_t>(T, nE);
                int64_t f = 0;
                for (int64_t c = 0; c < nch; ++c) {
                    const int32_t pl = (int32_t)(nE / nch + (c < nE % nch ? 1 : 0));
                    R.push_back({-1, f, pl});
                    f += pl;
                }
            }
            if ((int64_t)R.size() > INT32_MAX / 4)
                return fail(MC_ERR_UNSUPPORTED, "slice term too large");
        }
        // ---- runs -> lanes.  A parameter's direct runs share one lane in
        // every term (so direct-write terms need no barrier between them):
        // the map is built from the largest direct term first, longest run
        // first onto the least loaded lane; other runs likewise per term ----
        std::vector<std::vector<int32_t>> rl(nT), rit(nT);
        std::vector<int32_t> lane_of_k(P.Lp, -1);
        {
            std::vector<int> order(nT);
            std::iota(order.begin(), order.end(), 0);
            auto total = [&](int t) {
                int64_t x = 0;
                for (const Run& r : runs[t]) x += r.len;
                return x;
            };
            std::stable_sort(order.begin(), order.end(),
                             [&](int a2, int b2) { return total(a2) > total(b2); });
            std::vector<int64_t> kload(T, 0);  // load of the shared k->lane map
            for (int t : order) {
                const std::vector<Run>& R = runs[t];
                const int64_t nr = (int64_t)R.size();
                rl[t].assign(nr, 0);
                rit[t].assign(nr, 0);
                std::vector<int64_t> ord(nr);
                std::iota(ord.begin(), ord.end(), 0);
                std::stable_sort(ord.begin(), ord.end(),
                                 [&](int64_t a2, int64_t b2) { return R[a2].len > R[b2].len; });
                std::vector<int64_t> load(T, 0);
                std::vector<int32_t> cnt(T, 0);
                for (int64_t r : ord) {
                    int lane;
                    if (direct[t] && lane_of_k[R[r].k] >= 0) {
                        lane = lane_of_k[R[r].k];
                    } else {
                        std::vector<int64_t>& L = direct[t] ? kload : load;
                        lane = 0;
                        for (int l = 1; l < T; ++l)
                            if (L[l] < L[lane]) lane = l;
                        if (direct[t]) lane_of_k[R[r].k] = lane;
                    }
                    if (direct[t]) kload[lane] += R[r].len;
                    load[lane] += R[r].len;
                    rl[t][r] = lane;
                    rit[t][r] = cnt[lane]++;
                }
            }
        }
        // ---- per-term tables and tiled data, in program order; the slice's
        // active terms are stored first, compacted ----
        int nact = 0;
        for (int t = 0; t < nT; ++t) {
            const DevTerm& rt = raw[t];
            const std::vector<int64_t>& E = elems[s][t];
            const std::vector<Run>& R = runs[t];
            const int64_t nr = (int64_t)R.size();
            SlTerm st = make_slterm(rt, t);
            st.direct = direct[t];
            int32_t niter = 0;
            for (int64_t r = 0; r < nr; ++r) niter = std::max(niter, rit[t][r] + 1);
            st.niter = scalar[t] ? 0 : niter;
            // tiles per iteration
            std::vector<int32_t> tiles(3 * (size_t)niter, 0);
            std::vector<int64_t> toff(niter, 0);
            {
                std::vector<int32_t> lmax(niter, 0), lmin(niter, INT32_MAX);
                for (int64_t r = 0; r < nr; ++r) {
                    const int32_t it = rit[t][r];
                    lmax[it] = std::max(lmax[it], R[r].len);
                    lmin[it] = std::min(lmin[it], R[r].len);
                }
                int64_t tot = 0;
                for (int32_t it = 0; it < niter; ++it) {
                    const int64_t lpad = (lmax[it] + 3) / 4 * 4;
                    toff[it] = tot;
                    tiles[3 * it + 1] = lmax[it];
                    tiles[3 * it + 2] = lmax[it] > 0 ? lmin[it] / 4 : 0;
                    tot += (int64_t)T * lpad;
                }
                // tiled data operands (offsets relative to the slice block)
                for (int a = 0; a < 3; ++a) {
                    if (st.kind[a] != SK_DATA) continue;
                    while (P.data.size() % 4) P.data.push_back(0.0f);
                    const int64_t base = (int64_t)P.data.size();
                    P.data.resize(base + tot, 0.0f);
                    const int64_t src = rt.op[a].pool;
                    for (int64_t r = 0; r < nr; ++r) {
                        const int64_t o = base + toff[rit[t][r]] + rl[t][r] * 4;
                        for (int32_t u = 0; u < R[r].len; ++u)
                            P.data[o + (u >> 2) * (4 * T) + (u & 3)] =
                                dp[src + E[R[r].first + u]];
                    }
                    st.doff[a] = (int32_t)(base - blk0);
                }
                for (int32_t it = 0; it < niter; ++it) {
                    if (toff[it] > INT32_MAX / 2)
                        return fail(MC_ERR_UNSUPPORTED, "slice data too large");
                    tiles[3 * it] = (int32_t)toff[it];
                }
            }
            // lane records per (iteration, lane); empty {-1, 0}
            std::vector<int32_t> lanes(2 * (size_t)niter * T, 0);
            for (int64_t x = 0; x < (int64_t)niter * T; ++x) lanes[2 * x] = -1;
            for (int64_t r = 0; r < nr; ++r) {
                const int64_t x = (int64_t)rit[t][r] * T + rl[t][r];
                lanes[2 * x] = R[r].k;
                lanes[2 * x + 1] = R[r].len;
            }
            // combine entries per round of kSlItr iterations (split runs only):
            // the runs of one parameter, positions in run order
            std::vector<int32_t> roff, ents, plist;
            const int32_t nrounds = (niter + kSlItr - 1) / kSlItr;
            for (int32_t rd = 0; rd < nrounds; ++rd) {
                roff.push_back((int32_t)(ents.size() / 3));
                if (st.direct || ppr[t] < 0) continue;
                for (int64_t r = 0; r < nr;) {
                    int64_t q = r;
                    while (q < nr && R[q].k == R[r].k) ++q;
                    std::vector<int32_t> ps;
                    for (int64_t x = r; x < q; ++x)
                        if (rit[t][x] / kSlItr == rd)
                            ps.push_back((int32_t)((rit[t][x] % kSlItr) * T + rl[t][x]));
                    if (!ps.empty()) {
                        ents.push_back(R[r].k);
                        ents.push_back((int32_t)plist.size());
                        ents.push_back((int32_t)ps.size());
                        plist.insert(plist.end(), ps.begin(), ps.end());
                    }
                    r = q;
                }
            }
            roff.push_back((int32_t)(ents.size() / 3));
            // the tables go into the slice block as int32 words
            auto put = [&](const std::vector<int32_t>& v, bool even) -> int32_t {
                while (P.data.size() % (even ? 2 : 1)) P.data.push_back(0.0f);
                const int64_t o = (int64_t)P.data.size();
                P.data.resize(o + v.size());
                if (!v.empty()) std::memcpy(&P.data[o], v.data(), v.size() * 4);
                return (int32_t)(o - blk0);
            };
            st.tile_off = put(tiles, false);
            st.lane_off = put(lanes, true);
            st.round_off = put(roff, false);
            st.comb_off = put(ents, false);
            st.pos_off = put(plist, false);
            if (st.pp >= 0 && !st.direct && st.niter > 0) P.combine = 1;
            if (st.niter > 0) P.terms[(size_t)s * nT + nact++] = st;
        }
        while (P.data.size() % 4) P.data.push_back(0.0f);
        const int64_t blen = (int64_t)P.data.size() - blk0;
        P.blocks[4 * s] = blk0;
        P.blocks[4 * s + 1] = blen;
        P.blocks[4 * s + 2] = (int64_t)priv[s].size();
        P.blocks[4 * s + 3] = nact;
        if (blen > INT32_MAX / 8) return fail(MC_ERR_UNSUPPORTED, "slice data too large");
        P.sdata_floats = std::max<int>(P.sdata_floats, (int)blen);
    }
    if (P.index.empty()) P.index.push_back(0);
    if (P.data.empty()) P.data.assign(4, 0.0f);
    return MC_OK;
}


// ---------------------------------------------------------------------------
// lane-resident layout planner (lanes.h)
// ---------------------------------------------------------------------------
static void free_lanes(LanePlan& L) {
    if (L.d_terms) (void)hipFree(L.d_terms);
    if (L.d_data) (void)hipFree(L.d_data);
    if (L.d_blocks) (void)hipFree(L.d_blocks);
    if (L.d_gidx) (void)hipFree(L.d_gidx);
    if (L.d_sterms) (void)hipFree(L.d_sterms);
    if (L.d_rng) (void)hipFree(L.d_rng);
    L = LanePlan();
}


// Deal every slice's private parameters to (lane, slot), longest first onto
// the least loaded lane with a free slot, and tile each term's elements per
// (slot, lane).  Returns MC_ERR_UNSUPPORTED (with L.why) when the program does
// not qualify; the term interpreter (k_hmc_sl) then runs it.
// The compile-time form of a fast-form plan (lanes_fast.h LF_* bits): every
// slice holds the same swept / direct terms with the same shared operands,
// the shared roles (swept scale, direct loc, direct scale) are distinct
// parameters and every shared parameter has one; -1 otherwise, or when the
// form has no compiled kernel (k_hmc_lf<..., -1> reads it at run time).
static int lanes_form(const LanePlan& L, int nT) {
    int form = -2, o_sw = -1, o_dm = -1, o_ds = -1;
    for (int s = 0; s < L.S; ++s) {
        const int nsw = (int)(L.blocks[4 * s + 3] & 255), ndir = (int)((L.blocks[4 * s + 3] >> 8) & 255);
        const LrTerm* t = &L.terms[(size_t)s * nT];
        int f = 0, a = -1, b = -1, c = -1;
        if (nsw > 0) {
            f |= LF_SW;
            if (t[0].kind[2] == SK_SHARED) f |= LF_SWS, a = t[0].jsh[2];
        }
        if (ndir > 0) {
            const LrTerm& u = t[nsw];
            f |= LF_DIR;
            if (u.kind[1] == SK_SHARED) f |= LF_DM, b = u.jsh[1];
            if (u.kind[2] == SK_SHARED) f |= LF_DS, c = u.jsh[2];
        }
        if (form == -2) {
            form = f, o_sw = a, o_dm = b, o_ds = c;
        } else if (f != form || a != o_sw || b != o_dm || c != o_ds) {
            return -1;
        }
    }
    if (form < 0) return -1;
    const int roles = lf_nroles(form);
    if (roles != L.Dsh) return -1;
    if ((o_sw >= 0 && (o_sw == o_dm || o_sw == o_ds)) || (o_dm >= 0 && o_dm == o_ds)) return -1;
    return (form == (LF_SW | LF_SWS | LF_DIR | LF_DM | LF_DS) || form == LF_DIR) ? form : -1;
}

// The lane RNG plan of k_hmc_lf (lanes_fast.h lf_rng_*).  A wave's draws per
// iteration are the momentum normals of its two chains' private parameters
// (normal g % 4 of Philox block g / 4, the tape kernels' mapping), of the
// lanes' shared parameters (lane 2 k + c: parameter k of chain c), and one
// accept uniform per chain.  Every lane of a slice holds the same parameters
// in every wave, so the distinct (chain, block) pairs can be dealt to lanes
// once: lane i computes one Philox block and both Box-Muller pairs of it, two
// more lanes the chains' accept draws (their first Box-Muller log is the
// accept log), and each lane fetches its normals from the lanes that hold
// them — one Philox block and two Box-Muller pairs per lane and iteration
// instead of three blocks and three pairs, plus two blocks and logs per lane
// for the accept.  Per lane four words:
//   x: job (0 none, 1 / 2 momentum block of chain 0 / 1, 3 / 4 accept draw
//      of chain 0 / 1) | block << 3
//   y: slots 0, 1: source lane of chain 0, chain 1 (6 bits each) and the
//      component (2 bits), per slot 14 bits
//   z: slots 2, 3 likewise
//   w: the accept lane of chain 0 << 8 | of chain 1 << 14 | 1 << 30 (valid)
// (the blocks of every shared parameter of both chains are among the jobs;
// a lane finds its shared parameter's block lane once per launch)
// Empty when more than 62 distinct blocks are needed (the kernel then draws
// per lane).
static void plan_lane_rng(LanePlan& L, int S) {
    if (const char* e = std::getenv("MC_LANES_RNG"))  // 0: per-lane draws (A/B)
        if (std::atoi(e) == 0) return;
    std::vector<int32_t> rng((size_t)S * 64 * 4, 0);
    for (int s = 0; s < S; ++s) {
        std::map<std::pair<int, int32_t>, int> lane_of_block;  // (chain, block) -> lane
        std::vector<std::pair<int, int32_t>> jobs;
        auto job = [&](int c, int32_t b) {
            const auto key = std::make_pair(c, b);
            auto it = lane_of_block.find(key);
            if (it != lane_of_block.end()) return it->second;
            const int l = (int)jobs.size();
            jobs.push_back(key);
            lane_of_block[key] = l;
            return l;
        };
        int32_t* R = &rng[(size_t)s * 64 * 4];
        for (int j = 0; j < 64; ++j) {
            for (int r = 0; r < L.rs && r < kLrMaxSlots; ++r) {
                const int32_t g = L.gidx[((size_t)s * kLrMaxSlots + r) * 64 + j];
                if (g < 0) continue;
                if (g >= (1 << 28)) return;  // (block << 3 must fit the word)
                const int l0 = job(0, g >> 2), l1 = job(1, g >> 2);
                const int32_t v = l0 | (l1 << 6) | ((g & 3) << 12);
                R[4 * j + 1 + (r >> 1)] |= v << (14 * (r & 1));
            }
            if (j < 2 * L.Dsh) {  // every shared parameter k = j / 2 of chain j % 2 (the
                                  // kernel finds its block's lane: lane layouts differ)
                const int32_t g = L.shl[j >> 1];
                if (g >= (1 << 28)) return;
                (void)job(j & 1, g >> 2);
            }
        }
        if ((int)jobs.size() + 2 > 64) return;  // (no plan: per-lane draws)
        const int acc0 = (int)jobs.size(), acc1 = acc0 + 1;
        for (size_t i = 0; i < jobs.size(); ++i)
            R[4 * i] = (jobs[i].first + 1) | (jobs[i].second << 3);
        R[4 * acc0] = 3;
        R[4 * acc1] = 4;
        for (int j = 0; j < 64; ++j) R[4 * j + 3] |= (acc0 << 8) | (acc1 << 14) | (1 << 30);
    }
    L.rng.swap(rng);
}

static int plan_lanes(const mc_program* p, const SlicePlan& SP, const SlPartition& part,
                      LanePlan& L) {
    const std::vector<DevTerm>& raw = p->raw;
    const std::vector<float>& dp = p->h_data;
    const std::vector<int32_t>& ip = p->h_index;
    const int nT = (int)raw.size();
    const int S = SP.S;
    auto no = [&](const char* why) {
        L.why = why;
        return MC_ERR_UNSUPPORTED;
    };
    if (S > kLrSlices) return no("more than 16 slices");
    if (SP.Dsh > kLrMaxShared) return no("more than 4 broadcast parameters");
    int rs = 1;
    for (int s = 0; s < S; ++s) {
        const int need = ((int)part.priv[s].size() + 63) / 64;
        if (need > kLrMaxSlots) return no("more than 256 private parameters in a slice");
        rs = std::max(rs, need);
    }
    if (rs == 3) rs = 4;
    // replication (lanes.h LrCtx::rep): with at most 32 private parameters per
    // slice, each is dealt to a group of `rep` lanes (the largest power of two
    // <= 16 that still fits every parameter) and its elements are split over
    // the group: a lone wave's sweep runs n / rep elements instead of n (the
    // README "Small" shape: 7 groups of ~143 observations, 7 busy lanes of 64).
    // MC_LANES_REP=<k> caps it (1: off; A/B and tests).
    int rep = 1;
    if (rs == 1) {
        size_t maxp = 1;
        for (int s = 0; s < S; ++s) maxp = std::max(maxp, part.priv[s].size());
        int np2 = 1;
        while ((size_t)np2 < maxp) np2 <<= 1;
        rep = std::max(1, std::min(16, 64 / np2));
        if (const char* e = std::getenv("MC_LANES_REP")) {
            const int cap = std::atoi(e);
            while (rep > 1 && rep > cap) rep >>= 1;
        }
    }
    const int ngroups = 64 / rep;
    for (int t = 0; t < nT; ++t) {
        if (part.scalar[t] || part.ppr[t] < 0) continue;
        for (int64_t i = 0; i < raw[t].n; ++i)
            if (part.shared[pp_index(raw[t], part.ppr[t], i, ip)])
                return no("a per-element operand reads a broadcast parameter");
    }
    L.rs = rs;
    L.rep = rep;
    L.S = S;
    L.Dsh = SP.Dsh;
    L.nitems = SP.nitems;
    for (int k = 0; k < SP.Dsh; ++k) L.shl[k] = part.shl[k];
    L.has_xf = has_transform(p) ? 1 : 0;
    for (int k = 0; k < SP.Dsh; ++k) L.shxf[k] = part.shxf.empty() ? 0 : part.shxf[k];
    L.terms.assign((size_t)S * nT, LrTerm());
    L.blocks.assign(4 * (size_t)S, 0);
    L.gidx.assign((size_t)S * kLrMaxSlots * 64, -1);
    L.sdata_floats = 0;
    std::vector<int> lane_of(p->D, -1), slot_of_p(p->D, -1);
    bool any_rest = false, any_rest_nonexpr = false;
    for (int s = 0; s < S; ++s) {
        // ---- parameters -> (lane, slot) ----
        const std::vector<int>& pv = part.priv[s];
        std::vector<int64_t> cost(pv.size(), 0);
        std::vector<int> lpos(p->D, -1);
        for (size_t k = 0; k < pv.size(); ++k) lpos[pv[k]] = (int)k;
        for (int t = 0; t < nT; ++t) {
            if (part.scalar[t] || part.ppr[t] < 0) continue;
            for (int64_t i : part.elems[s][t]) cost[lpos[pp_index(raw[t], part.ppr[t], i, ip)]]++;
        }
        std::vector<int> ord(pv.size());
        std::iota(ord.begin(), ord.end(), 0);
        std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return cost[a] > cost[b]; });
        // (lane groups of `rep` lanes; lane_of = the group's leader lane)
        std::vector<int64_t> load(ngroups, 0);
        std::vector<int> used(ngroups, 0);
        for (int k : ord) {
            int best = -1;
            for (int l = 0; l < ngroups; ++l)
                if (used[l] < rs && (best < 0 || load[l] < load[best])) best = l;
            lane_of[pv[k]] = best * rep;
            slot_of_p[pv[k]] = used[best]++;
            load[best] += cost[k];
            for (int x = 0; x < rep; ++x)
                L.gidx[((size_t)s * kLrMaxSlots + slot_of_p[pv[k]]) * 64 + best * rep + x] = pv[k];
        }
        // ---- terms: the swept ones (lanes.h kLrSweep) first ----
        while (L.data.size() % 4) L.data.push_back(0.0f);
        const int64_t blk0 = (int64_t)L.data.size();
        int nact = 0;
        std::vector<LrTerm> swept, direct, rest;
        for (int t = 0; t < nT; ++t) {
            if (part.scalar[t]) continue;
            const DevTerm& rt = raw[t];
            const std::vector<int64_t>& E = part.elems[s][t];
            if (E.empty()) continue;
            LrTerm lt;
            std::memset(&lt, 0, sizeof(lt));
            lt.dist = rt.dist;
            lt.pp = part.ppr[t];
            lt.weight = rt.weight;
            lt.c0 = rt.c0;
            lt.clg = rt.clg;
            if (rt.op[2].kind == MC_OP_CONST) {
                const float c = rt.op[2].cval;
                lt.clogs = (float)std::log((double)c);
                lt.cinv = 1.0f / c;
                lt.cinv2 = 1.0f / (c * c);
            }
            for (int a = 0; a < 3; ++a) {
                const DevOperand& o = rt.op[a];
                lt.jsh[a] = 0;
                switch (o.kind) {
                    case MC_OP_CONST: lt.kind[a] = SK_CONST; lt.cval[a] = o.cval; break;
                    case MC_OP_PSCALAR: lt.kind[a] = SK_SHARED; lt.jsh[a] = part.jsh[o.poff]; break;
                    case MC_OP_DATA: lt.kind[a] = SK_DATA; break;
                    case MC_OP_PVEC:
                    case MC_OP_GATHER: lt.kind[a] = SK_PP; break;
                    default: lt.kind[a] = SK_NONE; break;
                }
            }
            lt.mode = (lt.kind[2] == SK_DATA || lt.kind[2] == SK_PP ||
                       (rt.dist != MC_DIST_NORMAL && rt.dist != MC_DIST_HALFNORMAL)) ? 1 : 0;
            lt.sig = LS_GENERIC;
            if (rt.dist == MC_DIST_NORMAL && lt.mode == 0) {
                const int a = lt.kind[0], b = lt.kind[1], c = lt.kind[2];
                if (a == SK_DATA && b == SK_PP) lt.sig = c == SK_SHARED ? LS_DATA_PP_SH : LS_DATA_PP_C;
                else if (a == SK_PP && b == SK_SHARED && c == SK_SHARED) lt.sig = LS_PP_SH_SH;
                else if (a == SK_PP && b == SK_CONST && c == SK_CONST) lt.sig = LS_PP_C_C;
                else if (a == SK_PP && b == SK_DATA && c == SK_SHARED) lt.sig = LS_PP_DATA_SH;
                else if (a == SK_DATA && b == SK_SHARED && c == SK_SHARED) lt.sig = LS_DATA_SH_SH;
            }
            // an affine loc (loc + b * x over data x): lanes.h lr_affine_term
            if (rt.affine) {
                if (rt.dist != MC_DIST_NORMAL || lt.mode != 0 || lt.kind[0] != SK_DATA ||
                    rt.ax.kind != MC_OP_DATA)
                    return no("an affine loc the lane kernels do not take");
                lt.sig = LS_AFF;
                lt.kb = rt.ab.kind == MC_OP_PSCALAR ? SK_SHARED : SK_CONST;
                lt.jb = rt.ab.kind == MC_OP_PSCALAR ? part.jsh[rt.ab.poff] : 0;
                lt.cb = rt.ab.kind == MC_OP_CONST ? rt.ab.cval : 0.0f;
            }
            // Normal with a per-element data scale, one of value / loc private
            // (theta ~ N(m, s_i), y_i ~ N(theta_g, s_i)): lanes.h lr_dscale_term
            if (rt.dist == MC_DIST_NORMAL && lt.kind[2] == SK_DATA && lt.pp >= 0 && lt.pp <= 1 &&
                lt.kind[lt.pp] == SK_PP && lt.kind[1 - lt.pp] != SK_PP &&
                lt.kind[1 - lt.pp] != SK_NONE && !rt.affine)
                lt.sig = LS_DSCALE;
            // an expression term (a chunk term: its data leaves tiled below)
            if (rt.dist == MC_DIST_EXPR) {
                lt.sig = LS_EXPR;
                lt.expr_base = rt.expr_base;
                lt.expr_n = rt.expr_n;
                L.has_expr = 1;
            }
            // element lists per (slot, lane), in element order
            std::vector<std::vector<int64_t>> lists((size_t)kLrMaxSlots * 64);
            int nslot = 1;
            if (lt.pp >= 0) {
                for (int64_t i : E) {
                    const int64_t g = pp_index(rt, lt.pp, i, ip);
                    const int r = slot_of_p[g];
                    lists[(size_t)r * 64 + lane_of[g]].push_back(i);
                    nslot = std::max(nslot, r + 1);
                }
                // a replicated parameter's elements: near-equal contiguous
                // chunks over its group (a lone element stays with the leader)
                if (rep > 1)
                    for (int r = 0; r < nslot; ++r)
                        for (int l0 = 0; l0 < 64; l0 += rep) {
                            std::vector<int64_t> all;
                            all.swap(lists[(size_t)r * 64 + l0]);
                            const int64_t n = (int64_t)all.size();
                            int64_t f = 0;
                            for (int x = 0; x < rep; ++x) {
                                const int64_t len = n / rep + (x < n % rep ? 1 : 0);
                                lists[(size_t)r * 64 + l0 + x].assign(all.begin() + f,
                                                                       all.begin() + f + len);
                                f += len;
                            }
                        }
            } else {  // chunk term: contiguous near-equal chunks over the lanes (slot 0)
                const int64_t nE = (int64_t)E.size(), nch = std::min<int64_t>(64, nE);
                int64_t f = 0;
                for (int64_t c = 0; c < nch; ++c) {
                    const int64_t len = nE / nch + (c < nE % nch ? 1 : 0);
                    for (int64_t u = 0; u < len; ++u) lists[(size_t)c].push_back(E[f + u]);
                    f += len;
                }
            }
            lt.nslot = nslot;
            int64_t tot = 0;
            std::vector<int32_t> lens((size_t)nslot * 64, 0);
            for (int r = 0; r < nslot; ++r) {
                int64_t lmax = 0, lmin = INT64_MAX;
                for (int l = 0; l < 64; ++l) {
                    const int64_t n = (int64_t)lists[(size_t)r * 64 + l].size();
                    if (n > INT32_MAX / 256) return no("a lane run is too long");
                    lens[(size_t)r * 64 + l] = (int32_t)n;
                    lmax = std::max(lmax, n);
                    if (n > 0) lmin = std::min(lmin, n);
                }
                if (tot > INT32_MAX / 4) return no("slice data too large");
                lt.toff[r] = (int32_t)tot;
                lt.lmin4[r] = lmax > 0 ? (int32_t)(lmin / 4) : 0;
                tot += 64 * ((lmax + 3) / 4 * 4);
            }
            for (int a = 0; a < 4; ++a) {  // (a = 3: an affine term's x)
                if (a < 3 ? lt.kind[a] != SK_DATA : lt.sig != LS_AFF) continue;
                while (L.data.size() % 4) L.data.push_back(0.0f);
                const int64_t base = (int64_t)L.data.size();
                L.data.resize(base + tot, 0.0f);
                const int64_t src = a < 3 ? rt.op[a].pool : rt.ax.pool;
                for (int r = 0; r < nslot; ++r)
                    for (int l = 0; l < 64; ++l) {
                        const std::vector<int64_t>& li = lists[(size_t)r * 64 + l];
                        for (size_t u = 0; u < li.size(); ++u)
                            L.data[base + lt.toff[r] + (u >> 2) * 256 + 4 * l + (u & 3)] =
                                dp[src + li[u]];
                    }
                if (a < 3) lt.doff[a] = (int32_t)(base - blk0);
                else lt.xoff = (int32_t)(base - blk0);
            }
            if (lt.sig == LS_EXPR) {  // the data leaves' arrays, in node order (one tile each)
                int e = 0;
                std::vector<int64_t> seen;
                for (int k = 0; k < rt.expr_n; ++k) {
                    const DevExprNode& d = p->nodes[rt.expr_base + k];
                    if (d.op != MC_EX_LEAF || d.leaf.kind != MC_OP_DATA) continue;
                    if (std::find(seen.begin(), seen.end(), d.leaf.pool) != seen.end()) continue;
                    seen.push_back(d.leaf.pool);
                    if (e >= kLrExprData) return no("an expression with too many data leaves");
                    while (L.data.size() % 4) L.data.push_back(0.0f);
                    const int64_t base = (int64_t)L.data.size();
                    L.data.resize(base + tot, 0.0f);
                    const int64_t src = d.leaf.pool;
                    for (int r = 0; r < nslot; ++r)
                        for (int l = 0; l < 64; ++l) {
                            const std::vector<int64_t>& li = lists[(size_t)r * 64 + l];
                            for (size_t u = 0; u < li.size(); ++u)
                                L.data[base + lt.toff[r] + (u >> 2) * 256 + 4 * l + (u & 3)] =
                                    dp[src + li[u]];
                        }
                    lt.eoff[e++] = (int32_t)(base - blk0);
                }
            }
            if (lt.sig == LS_DSCALE) {
                // the scale tile becomes 1/s^2 and the private operand's (free)
                // tile holds f32 log s, per element, as the constant-scale
                // terms' cinv2 / clogs
                const int64_t sb = blk0 + lt.doff[2];
                while (L.data.size() % 4) L.data.push_back(0.0f);
                const int64_t base = (int64_t)L.data.size();
                L.data.resize(base + tot, 0.0f);
                for (int r = 0; r < nslot; ++r)
                    for (int l = 0; l < 64; ++l) {
                        const size_t nl = lists[(size_t)r * 64 + l].size();
                        for (size_t u = 0; u < nl; ++u) {
                            const int64_t o = lt.toff[r] + (u >> 2) * 256 + 4 * l + (u & 3);
                            const float sc = L.data[sb + o];
                            L.data[base + o] = (float)std::log((double)sc);
                            L.data[sb + o] = 1.0f / (sc * sc);
                        }
                    }
                lt.doff[lt.pp] = (int32_t)(base - blk0);
            }
            const int64_t lo = (int64_t)L.data.size();
            L.data.resize(lo + lens.size());
            std::memcpy(&L.data[lo], lens.data(), lens.size() * 4);
            lt.len_off = (int32_t)(lo - blk0);
            int32_t maxlen = 0;
            for (int32_t x : lens) maxlen = std::max(maxlen, x);
            const bool dir = (lt.sig == LS_PP_SH_SH || lt.sig == LS_PP_C_C) && maxlen <= 1;
            const bool sw = lt.sig == LS_DATA_PP_SH || lt.sig == LS_DATA_PP_C ||
                            lt.sig == LS_PP_C_C || lt.sig == LS_PP_DATA_SH;
            if (dir && (int)direct.size() < kLrDirect) direct.push_back(lt);
            else if (sw && (int)swept.size() < kLrSweep) swept.push_back(lt);
            else rest.push_back(lt);
        }
        // fast form (lanes_fast.h): one swept term with data value and private
        // loc at most, one direct term at most, nothing else
        const bool core = !(swept.size() > 1 || direct.size() > 1 ||
                            (!swept.empty() && swept[0].sig != LS_DATA_PP_SH &&
                             swept[0].sig != LS_DATA_PP_C));
        if (!rest.empty() || !core) any_rest = true;
        bool rest_expr = true;  // every other term an expression term (LanePlan::nuts_expr)
        for (const LrTerm& lt : rest) rest_expr &= lt.sig == LS_EXPR;
        if (!rest_expr || !core) any_rest_nonexpr = true;
        for (const LrTerm& lt : swept) L.terms[(size_t)s * nT + nact++] = lt;
        for (const LrTerm& lt : direct) L.terms[(size_t)s * nT + nact++] = lt;
        for (const LrTerm& lt : rest) L.terms[(size_t)s * nT + nact++] = lt;
        while (L.data.size() % 4) L.data.push_back(0.0f);
        const int64_t blen = (int64_t)L.data.size() - blk0;
        if (blen > INT32_MAX / 8) return no("slice data too large");
        L.blocks[4 * s] = blk0;
        L.blocks[4 * s + 1] = blen;
        L.blocks[4 * s + 2] = nact;
        L.blocks[4 * s + 3] = (int64_t)swept.size() | ((int64_t)direct.size() << 8);
        L.sdata_floats = std::max<int>(L.sdata_floats, (int)blen);
    }
    // the scalar terms, compact (LDS copy in every workgroup)
    uint32_t own_mask = 0;
    int lf_generic = 0;  // scalar terms k_hmc_lf cannot take
    for (size_t it = 0; it < SP.sterms.size(); ++it) {
        const SlTerm& st = SP.sterms[it];
        LrSterm x;
        std::memset(&x, 0, sizeof(x));
        x.raw = part.sterm_raw.empty() ? 0 : part.sterm_raw[it];
        x.dist = st.dist;
        x.kinds = st.kind[0] | (st.kind[1] << 4) | (st.kind[2] << 8);
        x.jsh = (st.kind[0] == SK_SHARED ? st.jsh[0] : 0) |
                ((st.kind[1] == SK_SHARED ? st.jsh[1] : 0) << 4) |
                ((st.kind[2] == SK_SHARED ? st.jsh[2] : 0) << 8);
        x.c0 = st.c0;
        for (int a = 0; a < 3; ++a) x.cval[a] = st.cval[a];
        x.clogs = st.clogs;
        x.clg = st.clg;
        x.wn = st.weight * (float)st.niter;
        // one "own" prior per shared parameter (lanes.h LrOwn)
        x.own = st.kind[0] == SK_SHARED &&
                (st.dist == MC_DIST_NORMAL || st.dist == MC_DIST_HALFNORMAL) &&
                (st.kind[1] == SK_CONST || st.kind[1] == SK_NONE) && st.kind[2] == SK_CONST &&
                !(own_mask >> st.jsh[0] & 1) && !(x.raw & 1);
        if (x.own) own_mask |= 1u << st.jsh[0];
        x.cinv = st.kind[2] == SK_CONST ? 1.0f / st.cval[2] : 0.0f;
        if (!x.own) ++L.n_generic;
        // an identity term over a raw shared parameter (its log-Jacobian):
        // k_hmc_lf adds it in the holder lane (LrCtx::shid); k_hmc_lr runs it
        // with the other generic scalar terms
        const bool raw_id = st.dist == MC_DIST_IDENTITY && st.kind[0] == SK_SHARED &&
                            ((x.raw & 1) || L.shxf[st.jsh[0]] == MC_XF_NONE);
        if (raw_id) L.shid[st.jsh[0]] += x.wn;
        else if (!x.own) ++lf_generic;
        L.sterms.push_back(x);
    }
    L.sdata_floats = (L.sdata_floats + 3) / 4 * 4;  // the scalar terms follow, 16-byte aligned
    if ((int64_t)L.sdata_floats * 4 + (int64_t)L.sterms.size() * (int64_t)sizeof(LrSterm) >
        kSlLdsBudget)
        return no("slice data exceed the LDS budget");
    if (L.data.empty()) L.data.assign(4, 0.0f);
    plan_lane_rng(L, S);
    L.fast = (!any_rest && lf_generic == 0) ? 1 : 0;
    L.nuts_expr = (L.has_expr && !any_rest_nonexpr && lf_generic == 0) ? 1 : 0;
    L.form = L.fast ? lanes_form(L, nT) : -1;
    L.ok = 1;
    return MC_OK;
}

template <typename T>
static hipError_t upload(T** dst, const std::vector<T>& v) {
    hipError_t e = hipMalloc(dst, v.size() * sizeof(T));
    if (e == hipSuccess) e = hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
    return e;
}
static hipError_t upload_lanes(LanePlan& LP) {
    hipError_t e = upload(&LP.d_terms, LP.terms);
    if (e == hipSuccess) e = upload(&LP.d_data, LP.data);
    if (e == hipSuccess) e = upload(&LP.d_blocks, LP.blocks);
    if (e == hipSuccess) e = upload(&LP.d_gidx, LP.gidx);
    if (e == hipSuccess && !LP.sterms.empty()) e = upload(&LP.d_sterms, LP.sterms);
    if (e == hipSuccess && !LP.rng.empty()) e = upload(&LP.d_rng, LP.rng);
    return e;
}

// Element count of a program (the planner's size measure).
static int64_t program_elements(const mc_program* p) {
    int64_t n = 0;
    for (const DevTerm& t : p->raw) n += t.n;
    return n;
}
// The automatic slice count.  Programs of 2 K - 8 K elements are sliced (4
// ways) only when the lane-resident kernel takes them (measured at 256
// chains: the D = 100 / N = 10 k and D = 10 / N = 1 k hierarchical models run
// 2.1x / 1.7x faster than on the chain-per-workgroup kernel); smaller ones
// stay unsliced (a per-step exchange costs more than the whole evaluation).
// 8 - 64 K elements: 8 slices (one wave per SIMD, every CU busy at 256
// chains; the D = 100 / N = 10 k model: 165 -> 185 M steps/s against 4
// slices, 79 M with 16, profiles/r4/slices).
static constexpr int64_t kLrAutoMinElements = 2048;
static int auto_slices(const mc_program* p) {
    if ((has_expr(p) && !expr_lanes_ok(p)) || (has_affine(p) && !affine_lanes_ok(p)) ||
        (has_transform(p) && !transform_on_shared_only(p)))
        return 1;
    const int64_t n = program_elements(p);
    if (n >= 65536) return 16;
    if (n >= 8192) return 8;
    if (n >= kLrAutoMinElements) return 4;
    return 1;
}

// Plan an unsliced program onto the lane-resident kernel (one slice).
static int plan_lanes1(mc_program* p) {
    free_lanes(p->lr);
    // expression programs below the slicing threshold stay on the tape (the
    // one-slice lane kernel is not measured on them)
    if (has_expr(p))
        return fail(MC_ERR_UNSUPPORTED, "lane-resident kernel: an unsliced expression program "
                    "runs on the tape");
    SlicePlan P;
    SlPartition part;
    const int rc = plan_slices(p, 1, P, &part);
    if (rc != MC_OK) {
        p->note = "lane-resident kernel: " + g_last_error;
        return rc;
    }
    if (plan_lanes(p, P, part, p->lr) != MC_OK) {
        const std::string why = p->lr.why;
        free_lanes(p->lr);
        p->lr.why = why;
        p->note = "lane-resident kernel: " + why;
        return fail(MC_ERR_UNSUPPORTED, "lane-resident kernel: %s", why.c_str());
    }
    p->note.clear();
    const hipError_t e = upload_lanes(p->lr);
    if (e != hipSuccess) {
        free_lanes(p->lr);
        return fail(e == hipErrorOutOfMemory ? MC_ERR_NOMEM : MC_ERR_HIP,
                    "lane plan upload failed: %s", hipGetErrorString(e));
    }
    return MC_OK;
}

extern "C" int mc_program_set_slices(mc_program* p, int32_t S) {
    if (!p) return fail(MC_ERR_INVALID, "program is NULL");
    if (S < 0 || S > 64) return fail(MC_ERR_INVALID, "num_slices must be in [0, 64]");
    const bool automatic = (S == 0);
    if (automatic) S = auto_slices(p);
    free_slices(p->sl);
    free_lanes(p->lr);
    p->note.clear();
    if (S <= 1) {
        // automatic: the lane-resident kernel with one slice when the program
        // qualifies (1.4-4.5x k_hmc on D = 2..100 models at 64-1024 chains,
        // scripts/bench_unsliced.py); an explicit 1 keeps k_hmc
        if (automatic && p->slice_kernel != 1) (void)plan_lanes1(p);
        return MC_OK;
    }
    SlicePlan P;
    SlPartition part;
    int rc = plan_slices(p, S, P, &part);
    if (rc == MC_OK) {
        p->sl = P;  // host tables; geometry below needs them in place
        auto fit = [&]() {
            return sl_lds_bytes(p, 16) <= kSlLdsBudget ? 16
                 : (sl_lds_bytes(p, 8) <= kSlLdsBudget ? 8 : 0);
        };
        p->sl.nb_max = fit();
        if (p->sl.nb_max == 0)
            rc = fail(MC_ERR_UNSUPPORTED, "slice state (%d bytes) exceeds the LDS budget",
                      sl_lds_bytes(p, 8));
    }
    if (rc != MC_OK) {
        free_slices(p->sl);
        if (!automatic) return rc;
        p->note = "data slicing: " + g_last_error;
        return MC_OK;  // automatic: stay on the unsliced kernels
    }
    SlicePlan& Q = p->sl;
    hipError_t e = upload(&Q.d_terms, Q.terms);
    if (e == hipSuccess && !Q.sterms.empty()) e = upload(&Q.d_sterms, Q.sterms);
    if (e == hipSuccess) e = upload(&Q.d_data, Q.data);
    if (e == hipSuccess) e = upload(&Q.d_index, Q.index);
    if (e == hipSuccess) e = upload(&Q.d_blocks, Q.blocks);
    if (e == hipSuccess) e = upload(&Q.d_gidx, Q.gidx);
    if (e != hipSuccess) {
        free_slices(p->sl);
        return fail(e == hipErrorOutOfMemory ? MC_ERR_NOMEM : MC_ERR_HIP,
                    "slice upload failed: %s", hipGetErrorString(e));
    }
    // the lane-resident layout of the same slices, when the program qualifies
    LanePlan& LP = p->lr;
    if (plan_lanes(p, Q, part, LP) == MC_OK) {
        e = upload_lanes(LP);
        if (e != hipSuccess) {
            free_lanes(LP);
            free_slices(p->sl);
            return fail(e == hipErrorOutOfMemory ? MC_ERR_NOMEM : MC_ERR_HIP,
                        "slice upload failed: %s", hipGetErrorString(e));
        }
    } else {
        const std::string why = LP.why;
        free_lanes(LP);
        LP.why = why;
        p->note = "lane-resident kernel: " + why;
        if (!interp_ok(p)) {  // the term interpreter has no transforms / affine locs
            free_slices(p->sl);
            if (!automatic)
                return fail(MC_ERR_UNSUPPORTED, "lane-resident kernel: %s (a program with "
                            "transformed operands or affine locs is sliced onto it only)",
                            why.c_str());
            return MC_OK;
        }
        if (automatic && program_elements(p) < 16384) {  // only worth it on the lanes kernel
            free_slices(p->sl);
            if (p->slice_kernel != 1) (void)plan_lanes1(p);
            return MC_OK;
        }
    }
    return MC_OK;
}

extern "C" int mc_program_set_slice_kernel(mc_program* p, int32_t kernel) {
    if (!p) return fail(MC_ERR_INVALID, "program is NULL");
    if (kernel < 0 || kernel > 2) return fail(MC_ERR_INVALID, "slice kernel must be 0, 1 or 2");
    if (p->sl.S < 2) {
        // an unsliced program: 0 and 2 run it on the lane-resident kernel with
        // one slice (no exchange) — 0 when it qualifies, 2 or an error; 1 keeps
        // the chain-per-workgroup kernel (k_hmc)
        free_lanes(p->lr);
        if (kernel != 1) {
            const int rc = plan_lanes1(p);
            if (rc != MC_OK && kernel == 2) return rc;
        }
        p->slice_kernel = kernel;
        return MC_OK;
    }
    if (kernel == 2 && !p->lr.ok)
        return fail(MC_ERR_UNSUPPORTED, "lane-resident kernel: %s", p->lr.why.c_str());
    if (kernel == 1 && !interp_ok(p))
        return fail(MC_ERR_UNSUPPORTED, "the term interpreter does not run transformed operands "
                    "(mx.exp / mx.log), identity terms or affine locs");
    p->slice_kernel = kernel;
    return MC_OK;
}

extern "C" int32_t mc_program_slice_kernel(const mc_program* p) {
    if (!p) return -1;
    // expression terms on the lane layout run there only with their JIT-compiled
    // kernel: without it (off, or its compilation failed) the tape runs them
    if (p->lr.ok && p->lr.has_expr && p->slice_kernel != 1 &&
        (!jit_enabled() || !jit_error(p).empty()))
        return 0;
    if (p->sl.S < 2) return (p->lr.ok && p->lr.S == 1) ? 2 : 0;
    if (p->slice_kernel == 1 || !p->lr.ok) return 1;
    return 2;
}

extern "C" int32_t mc_program_lanes_fast(const mc_program* p) {
    if (!p) return -1;
    const int32_t k = mc_program_slice_kernel(p);
    return (k == 2 && p->lr.fast && lanes_fast_enabled()) ? 1 : 0;
}

extern "C" int32_t mc_program_num_slices(const mc_program* p) { return p ? p->sl.S : -1; }

extern "C" const char* mc_program_kernel_note(const mc_program* p) {
    if (!p) return "";
    const std::string je = jit_error(p);
    if (!je.empty()) {  // (the interpreter runs the expression terms)
        static thread_local std::string buf;
        buf = "expression JIT: compilation failed, the interpreter runs: " + je;
        return buf.c_str();
    }
    return (mc_program_slice_kernel(p) == 2) ? "" : p->note.c_str();
}

extern "C" int mc_program_create(const mc_term* terms, int32_t n_terms, int32_t n_params,
                                 float lp_const, const float* data, int64_t n_data,
                                 const int32_t* index, int64_t n_index, mc_program** out) {
    // the non-affine entry point ignores mc_term.affine (it was reserved0
    // before affine locs existed, and callers were free to leave it unset)
    if (n_terms < 0 || (n_terms > 0 && !terms)) return fail(MC_ERR_INVALID, "terms");
    std::vector<mc_term> t(terms, terms + n_terms);
    for (mc_term& x : t) x.affine = 0;
    return mc_program_create_affine(t.data(), n_terms, nullptr, 0, n_params, lp_const, data,
                                    n_data, index, n_index, out);
}

extern "C" int mc_program_create_affine(const mc_term* terms, int32_t n_terms,
                                        const mc_affine* affines, int32_t n_affines,
                                        int32_t n_params, float lp_const, const float* data,
                                        int64_t n_data, const int32_t* index, int64_t n_index,
                                        mc_program** out) {
    if (n_terms < 0 || (n_terms > 0 && !terms)) return fail(MC_ERR_INVALID, "bad term array");
    for (int32_t t = 0; t < n_terms; ++t)
        if (terms[t].dist == MC_DIST_EXPR)
            return fail(MC_ERR_INVALID, "term %d: expression terms need mc_program_create_expr", t);
    return mc_program_create_expr(terms, n_terms, affines, n_affines, nullptr, 0, nullptr, 0,
                                  n_params, lp_const, data, n_data, index, n_index, out);
}

// Validate and lay out one expression term (MC_DIST_EXPR): its nodes are
// appended to `gnodes` (dt.expr_base ..), a non-injective gather orders the
// term into the segment-tiled layout (build_segments_ops, whole runs), and
// vector leaves with overlapping parameter ranges deposit in different passes.
static int build_expr_term(int32_t t, const mc_term& src, const mc_expr* exprs, int32_t n_exprs,
                           const mc_expr_node* nodes, int32_t n_nodes, int32_t n_params,
                           int64_t n_data, int64_t n_index, std::vector<float>& dpool,
                           std::vector<int32_t>& ipool, std::vector<DevExprNode>& gnodes,
                           DevTerm& dt, int wpc) {
    // (leaf ranges are checked against the caller's pools, n_data / n_index:
    // dpool / ipool already hold the library's own tiled copies of earlier terms)
    if (src.affine < 1 || src.affine > n_exprs)
        return fail(MC_ERR_INVALID, "term %d: expression index %d out of range", t, src.affine);
    if (src.value.kind != MC_OP_NONE || src.loc.kind != MC_OP_NONE || src.scale.kind != MC_OP_NONE)
        return fail(MC_ERR_INVALID, "term %d: an expression term takes no value / loc / scale", t);
    const mc_expr& ex = exprs[src.affine - 1];
    if (ex.count < 1 || ex.count > kExMaxNodes)
        return fail(MC_ERR_UNSUPPORTED, "term %d: an expression holds 1 .. %d nodes (got %d)", t,
                    kExMaxNodes, ex.count);
    if (ex.first < 0 || (int64_t)ex.first + ex.count > n_nodes)
        return fail(MC_ERR_INVALID, "term %d: expression nodes out of range", t);
    const int64_t n = src.n;
    const int nn = ex.count;
    std::vector<DevExprNode> en(nn);
    std::vector<int> nonunique;  // non-injective gather leaves
    for (int k = 0; k < nn; ++k) {
        const mc_expr_node& s = nodes[ex.first + k];
        DevExprNode& d = en[k];
        std::memset(&d, 0, sizeof(d));
        d.op = s.op;
        d.a = s.a;
        d.b = s.b;
        d.c = s.c;
        d.leaf.kind = MC_OP_NONE;
        d.leaf.slot = -1;
        if (s.op < MC_EX_LEAF || s.op > MC_EX_LE)
            return fail(MC_ERR_INVALID, "term %d node %d: unknown op %d", t, k, s.op);
        if (s.op == MC_EX_LEAF) {
            const mc_operand& o = s.leaf;
            d.leaf.kind = o.kind;
            d.leaf.poff = o.param_offset;
            d.leaf.pool = o.pool_offset;
            d.leaf.cval = o.value;
            d.leaf.unique = 1;
            d.leaf.xf = MC_XF_NONE;
            if (o.transform != MC_XF_NONE)
                return fail(MC_ERR_INVALID, "term %d node %d: expression leaves take no transform "
                            "(exp / log are nodes)", t, k);
            switch (o.kind) {
                case MC_OP_CONST:
                    break;
                case MC_OP_PSCALAR:
                    if (o.param_offset < 0 || o.param_offset >= n_params)
                        return fail(MC_ERR_INVALID, "term %d node %d: param %d out of range", t, k,
                                    o.param_offset);
                    break;
                case MC_OP_DATA:
                    if (o.pool_offset < 0 || o.pool_offset + n > n_data)
                        return fail(MC_ERR_INVALID, "term %d node %d: data range out of pool", t, k);
                    break;
                case MC_OP_PVEC:
                    if (o.param_offset < 0 || (int64_t)o.param_offset + n > n_params)
                        return fail(MC_ERR_INVALID, "term %d node %d: param slice out of range", t,
                                    k);
                    break;
                case MC_OP_GATHER: {
                    if (o.pool_offset < 0 || o.pool_offset + n > n_index)
                        return fail(MC_ERR_INVALID, "term %d node %d: index range out of pool", t,
                                    k);
                    std::vector<int32_t> v(ipool.begin() + o.pool_offset,
                                           ipool.begin() + o.pool_offset + n);
                    for (int32_t x : v)
                        if (x < 0 || (int64_t)o.param_offset + x >= n_params)
                            return fail(MC_ERR_INVALID,
                                        "term %d node %d: gather index %d out of range", t, k, x);
                    std::sort(v.begin(), v.end());
                    d.leaf.unique = (std::adjacent_find(v.begin(), v.end()) == v.end()) ? 1 : 0;
                    if (!d.leaf.unique) nonunique.push_back(k);
                    break;
                }
                default:
                    return fail(MC_ERR_INVALID, "term %d node %d: bad leaf kind %d", t, k, o.kind);
            }
            d.a = d.b = d.c = -1;
            continue;
        }
        // arity: which arguments the op reads
        bool ua = true, ub = false, uc = false;
        switch (s.op) {
            case MC_EX_ADD: case MC_EX_SUB: case MC_EX_MUL: case MC_EX_DIV: case MC_EX_POW:
            case MC_EX_GT: case MC_EX_GE: case MC_EX_LT: case MC_EX_LE:
                ub = true;
                break;
            case MC_EX_NORMAL_LP: case MC_EX_WHERE: case MC_EX_GAMMA_LP: case MC_EX_BETA_LP:
                ub = uc = true;
                break;
            case MC_EX_HALFNORMAL_LP: case MC_EX_EXPONENTIAL_LP:
                uc = true;
                break;
            default:
                break;
        }
        auto arg_ok = [&](int x, bool used) { return used ? (x >= 0 && x < k) : x == -1; };
        if (!arg_ok(s.a, ua) || !arg_ok(s.b, ub) || !arg_ok(s.c, uc))
            return fail(MC_ERR_INVALID, "term %d node %d: bad arguments (%d, %d, %d) for op %d", t,
                        k, s.a, s.b, s.c, s.op);
        if (s.op == MC_EX_WHERE &&
            !(en[s.a].op == MC_EX_LEAF &&
              (en[s.a].leaf.kind == MC_OP_CONST || en[s.a].leaf.kind == MC_OP_DATA)) &&
            !(en[s.a].op >= MC_EX_GT && en[s.a].op <= MC_EX_LE))
            return fail(MC_ERR_UNSUPPORTED, "term %d node %d: a where mask must be data, a "
                        "constant or a comparison", t, k);
        // the distribution nodes' f32 normalisers (elem_normal / elem_halfnormal)
        if (s.op == MC_EX_NORMAL_LP) d.leaf.cval = dist_c0(MC_DIST_NORMAL);
        if (s.op == MC_EX_HALFNORMAL_LP) d.leaf.cval = dist_c0(MC_DIST_HALFNORMAL);
    }
    dt.dist = MC_DIST_EXPR;
    dt.n = n;
    dt.weight = src.weight;
    dt.affine = 0;
    dt.wave_task = -1;
    dt.primary = -1;
    // a non-injective gather: every such leaf through the same index values
    int64_t prim_pool = -1;
    if (!nonunique.empty()) {
        const int64_t p0 = en[nonunique[0]].leaf.pool;
        for (size_t r = 0; r < nonunique.size(); ++r) {
            const int k = nonunique[r];
            const int64_t pk = en[k].leaf.pool;
            if (pk != p0 && !std::equal(ipool.begin() + pk, ipool.begin() + pk + n,
                                        ipool.begin() + p0))
                return fail(MC_ERR_UNSUPPORTED, "term %d: an expression gathers through two "
                            "different non-injective index arrays", t);
            en[k].prim = 1 + (int)r;  // 1 + its row of split-run partials
        }
        prim_pool = p0;
        dt.primary = 0;  // (a flag for expression terms: segmented)
    }
    // passes: accumulating vector leaves with overlapping parameter ranges
    // deposit in different sweeps (ranges before any tiling)
    {
        std::vector<std::vector<std::pair<int64_t, int64_t>>> pr;  // per pass
        for (int k = 0; k < nn; ++k) {
            DevExprNode& d = en[k];
            if (d.op != MC_EX_LEAF || !is_acc_vec(d.leaf.kind)) continue;
            int64_t lo, hi;
            if (d.leaf.kind == MC_OP_PVEC) {
                lo = d.leaf.poff;
                hi = d.leaf.poff + n - 1;
            } else {
                const int32_t* ix = ipool.data() + d.leaf.pool;
                lo = d.leaf.poff + *std::min_element(ix, ix + n);
                hi = d.leaf.poff + *std::max_element(ix, ix + n);
            }
            int placed = -1;
            for (size_t ps = 0; ps < pr.size() && placed < 0; ++ps) {
                bool clash = false;
                for (auto& r : pr[ps])
                    if (!(hi < r.first || r.second < lo)) clash = true;
                if (!clash) placed = (int)ps;
            }
            if (placed < 0) {
                placed = (int)pr.size();
                pr.emplace_back();
            }
            pr[placed].push_back({lo, hi});
            d.pass = placed;
        }
        if (pr.size() > 16)
            return fail(MC_ERR_UNSUPPORTED, "term %d: more than 16 overlapping vector leaves", t);
        dt.npass = std::max<int>(1, (int)pr.size());
    }
    if (prim_pool >= 0) {
        // order the term by the index (stable), then tile it by runs
        bool sorted = true;
        for (int64_t i = 1; i < n && sorted; ++i) sorted = ipool[prim_pool + i - 1] <= ipool[prim_pool + i];
        if (!sorted) {
            std::vector<int64_t> perm(n);
            std::iota(perm.begin(), perm.end(), 0);
            std::stable_sort(perm.begin(), perm.end(), [&](int64_t x, int64_t y) {
                return ipool[prim_pool + x] < ipool[prim_pool + y];
            });
            std::map<std::pair<int, int64_t>, int64_t> moved;  // (kind, old pool) -> new pool
            for (int k = 0; k < nn; ++k) {
                DevOperand& d = en[k].leaf;
                if (en[k].op != MC_EX_LEAF) continue;
                if (d.kind == MC_OP_DATA || d.kind == MC_OP_GATHER) {
                    const auto key = std::make_pair((int)d.kind, d.pool);
                    auto it = moved.find(key);
                    if (it != moved.end()) {
                        d.pool = it->second;
                        continue;
                    }
                    int64_t base;
                    if (d.kind == MC_OP_DATA) {
                        base = (int64_t)dpool.size();
                        for (int64_t i = 0; i < n; ++i) dpool.push_back(dpool[d.pool + perm[i]]);
                    } else {
                        base = (int64_t)ipool.size();
                        for (int64_t i = 0; i < n; ++i) ipool.push_back(ipool[d.pool + perm[i]]);
                    }
                    moved[key] = base;
                    d.pool = base;
                } else if (d.kind == MC_OP_PVEC) {
                    const int64_t base = (int64_t)ipool.size();
                    for (int64_t i = 0; i < n; ++i) ipool.push_back((int32_t)perm[i]);
                    d.kind = MC_OP_GATHER;
                    d.pool = base;
                    d.unique = 1;
                }
            }
            prim_pool = en[nonunique[0]].leaf.pool;
        }
        std::vector<DevOperand*> others;
        for (int k = 0; k < nn; ++k)
            if (en[k].op == MC_EX_LEAF && !en[k].prim && is_vec_kind(en[k].leaf.kind))
                others.push_back(&en[k].leaf);
        // long runs split as the fused terms' are, with one partial row per
        // gathered leaf (nprim rows of <= 2 tsplit virtual segments: 4T floats)
        const int T = 64 * wpc;
        const int nprim = (int)nonunique.size();
        const int64_t tsplit = std::max<int64_t>(1, std::min<int64_t>(T, 2 * T / nprim));
        const int rc = build_segments_ops(dt, prim_pool, others, tsplit, nprim, dpool, ipool, T);
        if (rc) return rc;
    }
    dt.expr_base = (int32_t)gnodes.size();
    dt.expr_n = nn;
    gnodes.insert(gnodes.end(), en.begin(), en.end());
    return MC_OK;
}

extern "C" int mc_program_create_expr(const mc_term* terms, int32_t n_terms,
                                      const mc_affine* affines, int32_t n_affines,
                                      const mc_expr* exprs, int32_t n_exprs,
                                      const mc_expr_node* nodes, int32_t n_nodes,
                                      int32_t n_params, float lp_const, const float* data,
                                      int64_t n_data, const int32_t* index, int64_t n_index,
                                      mc_program** out) {
    if (!out) return fail(MC_ERR_INVALID, "out is NULL");
    if (n_affines < 0 || (n_affines > 0 && !affines))
        return fail(MC_ERR_INVALID, "bad affine array");
    if (n_exprs < 0 || (n_exprs > 0 && !exprs)) return fail(MC_ERR_INVALID, "bad expression array");
    if (n_nodes < 0 || (n_nodes > 0 && !nodes)) return fail(MC_ERR_INVALID, "bad node array");
    *out = nullptr;
    if (n_params <= 0) return fail(MC_ERR_INVALID, "n_params must be positive (got %d)", n_params);
    if (n_terms < 0 || (n_terms > 0 && !terms)) return fail(MC_ERR_INVALID, "bad term array");
    if (n_data < 0 || (n_data > 0 && !data)) return fail(MC_ERR_INVALID, "bad data pool");
    if (n_index < 0 || (n_index > 0 && !index)) return fail(MC_ERR_INVALID, "bad index pool");

    std::vector<float> dpool(data, data + n_data);
    std::vector<int32_t> ipool(index, index + n_index);
    std::vector<DevTerm> dts, raws;
    std::vector<DevExprNode> gnodes;
    int64_t max_n = 0;
    for (int32_t t = 0; t < n_terms; ++t) max_n = std::max<int64_t>(max_n, terms[t].n);
    const int wpc = choose_wpc(max_n);

    for (int32_t t = 0; t < n_terms; ++t) {
        const mc_term& src = terms[t];
        if (src.dist < MC_DIST_NORMAL || src.dist > MC_DIST_EXPR)
            return fail(MC_ERR_INVALID, "term %d: unknown distribution %d", t, src.dist);
        if (src.n < 1) return fail(MC_ERR_INVALID, "term %d: n must be >= 1", t);
        const int64_t n = src.n;
        DevTerm dt;
        std::memset(&dt, 0, sizeof(dt));
        if (src.dist == MC_DIST_EXPR) {
            const int rc = build_expr_term(t, src, exprs, n_exprs, nodes, n_nodes, n_params,
                                           n_data, n_index, dpool, ipool, gnodes, dt, wpc);
            if (rc) return rc;
            raws.push_back(dt);
            dts.push_back(dt);
            continue;
        }
        dt.dist = src.dist;
        dt.n = n;
        dt.weight = src.weight;
        dt.c0 = dist_c0(src.dist);
        const mc_operand* ops[5] = {&src.value, &src.loc, &src.scale, nullptr, nullptr};
        int nops = 3;
        if (src.affine != 0) {
            if (src.affine < 0 || src.affine > n_affines)
                return fail(MC_ERR_INVALID, "term %d: affine index %d out of range", t,
                            src.affine);
            if (src.dist != MC_DIST_NORMAL)
                return fail(MC_ERR_UNSUPPORTED, "term %d: an affine loc needs a Normal term", t);
            const mc_affine& af = affines[src.affine - 1];
            if (af.slope.kind != MC_OP_CONST && af.slope.kind != MC_OP_PSCALAR)
                return fail(MC_ERR_UNSUPPORTED, "term %d: affine slope must be a constant or a "
                            "scalar parameter", t);
            if (af.x.kind != MC_OP_DATA && af.x.kind != MC_OP_PVEC && af.x.kind != MC_OP_GATHER)
                return fail(MC_ERR_UNSUPPORTED, "term %d: affine x must be data, a parameter "
                            "vector or a gather", t);
            ops[3] = &af.slope;
            ops[4] = &af.x;
            nops = 5;
            dt.affine = 1;
        }
        for (int a = 0; a < nops; ++a) {
            const mc_operand& o = *ops[a];
            DevOperand& d = a < 3 ? dt.op[a] : (a == 3 ? dt.ab : dt.ax);
            d.kind = o.kind;
            d.poff = o.param_offset;
            d.pool = o.pool_offset;
            d.cval = o.value;
            d.unique = 1;
            d.xf = o.transform;
            if (o.transform < MC_XF_NONE || o.transform > MC_XF_LOG)
                return fail(MC_ERR_INVALID, "term %d op %d: unknown transform %d", t, a,
                            o.transform);
            if (o.transform != MC_XF_NONE && o.kind != MC_OP_PSCALAR && o.kind != MC_OP_PVEC &&
                o.kind != MC_OP_GATHER)
                return fail(MC_ERR_INVALID, "term %d op %d: a transform applies to parameter "
                            "operands only", t, a);
            const bool need =
                !(a == 1 && (src.dist == MC_DIST_HALFNORMAL || src.dist == MC_DIST_EXPONENTIAL)) &&
                !(src.dist == MC_DIST_IDENTITY && (a == 1 || a == 2));
            if (!need) {
                if (o.kind != MC_OP_NONE && o.kind != MC_OP_CONST)
                    return fail(MC_ERR_INVALID, "term %d: %s takes no %s operand", t,
                                src.dist == MC_DIST_HALFNORMAL
                                    ? "HalfNormal"
                                    : (src.dist == MC_DIST_EXPONENTIAL ? "Exponential"
                                                                       : "an identity term"),
                                a == 1 ? "loc" : "scale");
                d.kind = MC_OP_NONE;
                d.xf = MC_XF_NONE;
                continue;
            }
            switch (o.kind) {
                case MC_OP_CONST:
                    break;
                case MC_OP_PSCALAR:
                    if (o.param_offset < 0 || o.param_offset >= n_params)
                        return fail(MC_ERR_INVALID, "term %d op %d: param %d out of range", t, a,
                                    o.param_offset);
                    break;
                case MC_OP_DATA:
                    if (o.pool_offset < 0 || o.pool_offset + n > n_data)
                        return fail(MC_ERR_INVALID, "term %d op %d: data range out of pool", t, a);
                    break;
                case MC_OP_PVEC:
                    if (o.param_offset < 0 || (int64_t)o.param_offset + n > n_params)
                        return fail(MC_ERR_INVALID, "term %d op %d: param slice out of range", t,
                                    a);
                    break;
                case MC_OP_GATHER: {
                    if (o.pool_offset < 0 || o.pool_offset + n > n_index)
                        return fail(MC_ERR_INVALID, "term %d op %d: index range out of pool", t,
                                    a);
                    std::vector<int32_t> v(ipool.begin() + o.pool_offset,
                                           ipool.begin() + o.pool_offset + n);
                    for (int32_t x : v)
                        if (x < 0 || (int64_t)o.param_offset + x >= n_params)
                            return fail(MC_ERR_INVALID,
                                        "term %d op %d: gather index %d out of range", t, a, x);
                    std::sort(v.begin(), v.end());
                    d.unique = (std::adjacent_find(v.begin(), v.end()) == v.end()) ? 1 : 0;
                    break;
                }
                default:
                    return fail(MC_ERR_INVALID, "term %d op %d: bad operand kind %d", t, a,
                                o.kind);
            }
        }
        if (dt.affine) {
            // a non-injective gather only as the loc itself (alpha[group] + b * x,
            // the segmented path), with a data x
            for (int k = 0; k < 5; ++k) {
                const DevOperand* d = k < 3 ? &dt.op[k] : (k == 3 ? &dt.ab : &dt.ax);
                if (d->kind == MC_OP_GATHER && !d->unique && !(k == 1 && dt.ax.kind == MC_OP_DATA))
                    return fail(MC_ERR_UNSUPPORTED, "term %d: an affine-loc term gathers through "
                                "a non-injective index only in its loc, with a data x", t);
            }
            if (dt.op[1].kind == MC_OP_NONE)
                return fail(MC_ERR_INVALID, "term %d: affine loc without a loc operand", t);
        }
        // the non-injective gather, if any, orders the term
        int primary = -1;
        for (int a = 0; a < 3; ++a) {
            if (dt.op[a].kind == MC_OP_GATHER && !dt.op[a].unique) {
                if (primary >= 0)
                    return fail(MC_ERR_UNSUPPORTED,
                                "term %d gathers through two non-injective index arrays", t);
                primary = a;
            }
        }
        dt.primary = primary;
        if (primary >= 0) {
            const int64_t ip = dt.op[primary].pool;
            bool sorted = true;
            for (int64_t i = 1; i < n && sorted; ++i) sorted = ipool[ip + i - 1] <= ipool[ip + i];
            if (!sorted) {
                std::vector<int64_t> perm(n);
                std::iota(perm.begin(), perm.end(), 0);
                std::stable_sort(perm.begin(), perm.end(), [&](int64_t x, int64_t y) {
                    return ipool[ip + x] < ipool[ip + y];
                });
                for (int a = 0; a < 4; ++a) {
                    if (a == 3 && !dt.affine) break;
                    DevOperand& d = a < 3 ? dt.op[a] : dt.ax;  // (an affine x is data)
                    if (d.kind == MC_OP_DATA) {
                        const int64_t base = (int64_t)dpool.size();
                        for (int64_t i = 0; i < n; ++i) dpool.push_back(dpool[d.pool + perm[i]]);
                        d.pool = base;
                    } else if (d.kind == MC_OP_GATHER) {
                        const int64_t base = (int64_t)ipool.size();
                        for (int64_t i = 0; i < n; ++i) ipool.push_back(ipool[d.pool + perm[i]]);
                        d.pool = base;
                    } else if (d.kind == MC_OP_PVEC) {
                        const int64_t base = (int64_t)ipool.size();
                        for (int64_t i = 0; i < n; ++i) ipool.push_back((int32_t)perm[i]);
                        d.kind = MC_OP_GATHER;
                        d.pool = base;
                        d.unique = 1;
                    }
                }
            }
        }
        // constant-shape normalisers (every layout reads them: the sliced
        // planners copy them from the validated terms)
        dt.clogs = (dt.op[2].kind == MC_OP_CONST) ? (float)std::log((double)dt.op[2].cval) : 0.0f;
        dt.clg = 0.0f;
        if ((dt.dist == MC_DIST_GAMMA && dt.op[1].kind == MC_OP_CONST) ||
            (dt.dist == MC_DIST_BETA && dt.op[1].kind == MC_OP_CONST &&
             dt.op[2].kind == MC_OP_CONST))
            dt.clg = lgamma_norm(dt.dist, dt.op[1].cval, dt.op[2].cval);
        raws.push_back(dt);
        // pass planning: accumulating vector operands with overlapping parameter
        // ranges go to different sweeps
        int64_t lo[3], hi[3];
        for (int a = 0; a < 3; ++a) {
            const DevOperand& d = dt.op[a];
            lo[a] = hi[a] = -1;
            if (d.kind == MC_OP_PVEC) {
                lo[a] = d.poff;
                hi[a] = d.poff + n - 1;
            } else if (d.kind == MC_OP_GATHER) {
                int32_t mn = ipool[d.pool], mx = ipool[d.pool];
                for (int64_t i = 1; i < n; ++i) {
                    mn = std::min(mn, ipool[d.pool + i]);
                    mx = std::max(mx, ipool[d.pool + i]);
                }
                lo[a] = d.poff + mn;
                hi[a] = d.poff + mx;
            }
        }
        uint32_t masks[3] = {PASS_LP, 0, 0};
        int npass = 1;
        for (int a = 0; a < 3; ++a) {
            const uint32_t bit = 1u << a;
            if (dt.op[a].kind == MC_OP_PSCALAR) {
                masks[0] |= bit;
                continue;
            }
            if (!is_acc_vec(dt.op[a].kind)) continue;
            int placed = -1;
            for (int ps = 0; ps < npass && placed < 0; ++ps) {
                bool clash = false;
                for (int b = 0; b < a; ++b)
                    if ((masks[ps] & (1u << b)) && is_acc_vec(dt.op[b].kind) &&
                        !(hi[a] < lo[b] || hi[b] < lo[a]))
                        clash = true;
                if (!clash) placed = ps;
            }
            if (placed < 0) placed = npass++;
            masks[placed] |= bit;
        }
        if (dt.affine) {
            // the slope's and x's cotangents accumulate in the loc's sweep:
            // x must not overlap another accumulating operand of the term
            const bool acc = dt.ab.kind == MC_OP_PSCALAR || is_acc_vec(dt.ax.kind);
            bool has_loc = false;
            for (int ps = 0; ps < npass; ++ps) has_loc |= (masks[ps] & PASS_LOC) != 0;
            if (acc && !has_loc) masks[0] |= PASS_LOC;
            if (is_acc_vec(dt.ax.kind)) {
                int64_t xl, xh;
                if (dt.ax.kind == MC_OP_PVEC) {
                    xl = dt.ax.poff;
                    xh = dt.ax.poff + n - 1;
                } else {
                    int32_t mn = ipool[dt.ax.pool], mx = ipool[dt.ax.pool];
                    for (int64_t i = 1; i < n; ++i) {
                        mn = std::min(mn, ipool[dt.ax.pool + i]);
                        mx = std::max(mx, ipool[dt.ax.pool + i]);
                    }
                    xl = dt.ax.poff + mn;
                    xh = dt.ax.poff + mx;
                }
                for (int a = 0; a < 3; ++a)
                    if (is_acc_vec(dt.op[a].kind) && !(xh < lo[a] || hi[a] < xl))
                        return fail(MC_ERR_UNSUPPORTED, "term %d: the affine x overlaps operand "
                                    "%d's parameters", t, a);
            }
        }
        dt.npass = npass;
        dt.pass_masks = masks[0] | (masks[1] << 4) | (masks[2] << 8);
        dt.wave_task = -1;
        dt.prim_poff = primary >= 0 ? dt.op[primary].poff : 0;
        if (primary >= 0) {
            const int rc = build_segments(dt, dpool, ipool, 64 * wpc);
            if (rc) return rc;
        }
        dts.push_back(dt);
    }

    // broadcast-parameter cotangent slots and their fixed-order finalize list
    int32_t nslot = 0;
    std::vector<std::pair<int32_t, int32_t>> uses;  // (param, slot)
    for (DevTerm& dt : dts) {
        for (int a = 0; a < 3; ++a)
            if (dt.op[a].kind == MC_OP_PSCALAR) {
                dt.op[a].slot = nslot;
                uses.push_back({dt.op[a].poff, nslot});
                ++nslot;
            }
        if (dt.affine && dt.ab.kind == MC_OP_PSCALAR) {
            dt.ab.slot = nslot;
            uses.push_back({dt.ab.poff, nslot});
            ++nslot;
        }
        if (dt.dist == MC_DIST_EXPR)
            for (int k = 0; k < dt.expr_n; ++k) {
                DevExprNode& d = gnodes[dt.expr_base + k];
                if (d.op != MC_EX_LEAF || d.leaf.kind != MC_OP_PSCALAR) continue;
                d.leaf.slot = nslot;
                uses.push_back({d.leaf.poff, nslot});
                ++nslot;
            }
    }
    std::stable_sort(uses.begin(), uses.end(),
                     [](const std::pair<int32_t, int32_t>& x,
                        const std::pair<int32_t, int32_t>& y) { return x.first < y.first; });
    std::vector<int32_t> fin_hdr, fin_ids;
    for (size_t i = 0; i < uses.size();) {
        size_t j = i;
        while (j < uses.size() && uses[j].first == uses[i].first) ++j;
        fin_hdr.push_back(uses[i].first);
        fin_hdr.push_back((int32_t)fin_ids.size());
        fin_hdr.push_back((int32_t)(j - i));
        for (size_t k = i; k < j; ++k) fin_ids.push_back(uses[k].second);
        i = j;
    }
    const int64_t sfin_base = (int64_t)ipool.size();
    ipool.push_back((int32_t)(fin_hdr.size() / 3));
    ipool.insert(ipool.end(), fin_hdr.begin(), fin_hdr.end());
    ipool.insert(ipool.end(), fin_ids.begin(), fin_ids.end());
    // small terms whose only cotangents are broadcast parameters run as wave
    // tasks: one wave each, round robin, concurrently with the other waves
    {
        int next = 0;
        for (DevTerm& dt : dts) {
            bool vec_param = false;
            for (int a = 0; a < 3; ++a)
                if (dt.op[a].kind == MC_OP_PVEC || dt.op[a].kind == MC_OP_GATHER) vec_param = true;
            if (dt.affine && (dt.ax.kind == MC_OP_PVEC || dt.ax.kind == MC_OP_GATHER))
                vec_param = true;
            if (dt.dist == MC_DIST_EXPR)
                for (int k = 0; k < dt.expr_n; ++k)
                    if (gnodes[dt.expr_base + k].op == MC_EX_LEAF &&
                        is_acc_vec(gnodes[dt.expr_base + k].leaf.kind))
                        vec_param = true;
            if (dt.primary < 0 && dt.npass == 1 && dt.n <= 64 && !vec_param)
                dt.wave_task = (next++) % wpc;
        }
    }
    // evaluate all-wave terms first and the wave tasks last: a wave task only
    // writes its own cotangent slots, so its position is free, and at the end
    // it overlaps the other waves' share of the last all-wave term
    std::stable_partition(dts.begin(), dts.end(),
                          [](const DevTerm& dt) { return dt.wave_task < 0; });
    // barriers between terms whose gradient writes overlap (vector operands)
    {
        std::vector<std::pair<int64_t, int64_t>> open_ranges;
        for (DevTerm& dt : dts) {
            std::vector<std::pair<int64_t, int64_t>> mine;
            if (dt.dist == MC_DIST_EXPR)
                for (int k = 0; k < dt.expr_n; ++k) {
                    const DevExprNode& d = gnodes[dt.expr_base + k];
                    if (d.op != MC_EX_LEAF) continue;
                    if (d.leaf.kind == MC_OP_PVEC)
                        mine.push_back({d.leaf.poff, d.leaf.poff + dt.n - 1});
                    else if (d.leaf.kind == MC_OP_GATHER)
                        mine.push_back({0, (int64_t)n_params - 1});
                }
            for (int a = 0; a < 4; ++a) {
                if (a == 3 && !dt.affine) break;
                const DevOperand& d = a < 3 ? dt.op[a] : dt.ax;
                if (d.kind == MC_OP_PVEC) {
                    mine.push_back({d.poff, d.poff + dt.n - 1});
                } else if (d.kind == MC_OP_GATHER) {
                    // conservative: the whole parameter vector
                    mine.push_back({0, (int64_t)n_params - 1});
                }
            }
            bool clash = false;
            for (auto& r : mine)
                for (auto& o : open_ranges)
                    if (!(r.second < o.first || o.second < r.first)) clash = true;
            dt.sync_before = clash ? 1 : 0;
            if (clash) open_ranges.clear();
            open_ranges.insert(open_ranges.end(), mine.begin(), mine.end());
        }
    }

    // expression leaves address the pools with 32-bit offsets (eval.h reads
    // them into lanes): every offset, tiled copies included, lies below the
    // pools' final sizes, so bounding those bounds them all
    if (!gnodes.empty() && (dpool.size() > (size_t)INT32_MAX || ipool.size() > (size_t)INT32_MAX))
        return fail(MC_ERR_UNSUPPORTED,
                    "expression terms: the data / index pools (%zu / %zu elements) exceed the "
                    "2^31 elements their 32-bit leaf offsets address", dpool.size(), ipool.size());
    mc_program* p = new mc_program();
    p->D = n_params;
    p->nslots = nslot + 1;
    p->sfin_base = sfin_base;
    p->lp_const = lp_const;
    p->max_n = max_n;
    p->wpc = wpc;
    p->terms = dts;
    p->raw = raws;
    p->nodes = gnodes;
    p->ex = !gnodes.empty();
    p->h_data = dpool;
    p->h_index = ipool;
    if (g_program_host_only) {  // test hook: the host tables only (no device)
        *out = p;
        return MC_OK;
    }
    hipError_t e = hipSuccess;
    if (!dts.empty()) {
        e = hipMalloc(&p->d_terms, dts.size() * sizeof(DevTerm));
        if (e == hipSuccess)
            e = hipMemcpy(p->d_terms, dts.data(), dts.size() * sizeof(DevTerm),
                          hipMemcpyHostToDevice);
    }
    if (e == hipSuccess && !gnodes.empty()) {
        e = hipMalloc(&p->d_nodes, gnodes.size() * sizeof(DevExprNode));
        if (e == hipSuccess)
            e = hipMemcpy(p->d_nodes, gnodes.data(), gnodes.size() * sizeof(DevExprNode),
                          hipMemcpyHostToDevice);
    }
    if (e == hipSuccess && !dpool.empty()) {
        e = hipMalloc(&p->d_data, dpool.size() * sizeof(float));
        if (e == hipSuccess)
            e = hipMemcpy(p->d_data, dpool.data(), dpool.size() * sizeof(float),
                          hipMemcpyHostToDevice);
    }
    if (e == hipSuccess && !ipool.empty()) {
        e = hipMalloc(&p->d_index, ipool.size() * sizeof(int32_t));
        if (e == hipSuccess)
            e = hipMemcpy(p->d_index, ipool.data(), ipool.size() * sizeof(int32_t),
                          hipMemcpyHostToDevice);
    }
    if (e != hipSuccess) {
        mc_program_destroy(p);
        return fail(e == hipErrorOutOfMemory ? MC_ERR_NOMEM : MC_ERR_HIP,
                    "program upload failed: %s", hipGetErrorString(e));
    }
    {
        const int rc = mc_program_set_slices(p, 0);
        if (rc != MC_OK) {
            mc_program_destroy(p);
            return rc;
        }
    }
    *out = p;
    return MC_OK;
}

// Test hook without a device: the slice and lane plans of a host-only program
// (mc_debug_program_host_only) with S slices, host tables only (no upload),
// so the lane-resident expression source can be generated and compiled on a
// machine without a GPU (mc_debug_expr_jit_source / _compile with a
// "mc::k_hmc_lr<...>" kernel).  Returns the planner's status; MC_OK with
// lr.has_expr set when the program's expression terms took the lane layout.
extern "C" int mc_debug_lane_plan_host(mc_program* p, int32_t S) {
    if (!p) return fail(MC_ERR_INVALID, "program is NULL");
    if (S < 1 || S > kLrSlices) return fail(MC_ERR_INVALID, "S must be in [1, %d]", kLrSlices);
    free_lanes(p->lr);
    SlicePlan P;
    SlPartition part;
    int rc = plan_slices(p, S, P, &part);
    if (rc != MC_OK) return rc;
    rc = plan_lanes(p, P, part, p->lr);
    if (rc != MC_OK) return fail(rc, "lane-resident kernel: %s", p->lr.why.c_str());
    return MC_OK;
}

// Test hook (mc_debug_program_host_only): programs built after it is set keep
// their host tables only — no device upload, no slice plan — for host-side
// checks without a GPU (the expression JIT's code generation and compilation,
// mc_debug_expr_jit_compile).  Such a program must not be launched.
extern "C" int mc_debug_program_host_only(int on) {
    g_program_host_only = on != 0;
    return MC_OK;
}

extern "C" int mc_program_destroy(mc_program* p) {
    if (!p) return MC_OK;
    jit_free(p);
    free_slices(p->sl);
    free_lanes(p->lr);
    if (p->d_terms) (void)hipFree(p->d_terms);
    if (p->d_nodes) (void)hipFree(p->d_nodes);
    if (p->d_data) (void)hipFree(p->d_data);
    if (p->d_index) (void)hipFree(p->d_index);
    delete p;
    return MC_OK;
}

extern "C" int32_t mc_program_num_params(const mc_program* p) { return p ? p->D : -1; }
extern "C" int32_t mc_program_waves_per_chain(const mc_program* p) { return p ? p->wpc : -1; }


// ---------------------------------------------------------------------------
// batched log density + gradient
// ---------------------------------------------------------------------------
template <int WPC, bool EX>
__global__ void __launch_bounds__(WPC >= 4 ? 64 * WPC : 256)
k_logp(DevCtx P, int64_t n_points, const float* q, float* logp, float* grad, int lds_floats) {
    constexpr int CPB = (WPC >= 4) ? 1 : 4 / WPC;
    constexpr int T = 64 * WPC;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int lc = threadIdx.x / T;
    const int64_t c = (int64_t)blockIdx.x * CPB + lc;
    if (c >= n_points) return;
    Group<WPC> G;
    SegScratch S;
    G.tid = threadIdx.x % T;
    carve_group<WPC>(smem + (int64_t)lc * lds_floats, G, S);
    const float lp = eval_lp_grad<WPC, false, EX>(P, q + c * P.D, grad + c * P.D, G, S);
    if (G.tid == 0) logp[c] = lp;
}

template <int WPC, bool EX>
static int launch_logp(const mc_program* p, int64_t n, const float* q, float* lp, float* g,
                       hipStream_t st) {
    const int lds_floats = scratch_of(p);
    const size_t lds = (size_t)cpb_of(WPC) * lds_floats * 4;
    const int64_t grid = (n + cpb_of(WPC) - 1) / cpb_of(WPC);
    MC_HIP_TRY(allow_lds(k_logp<WPC, EX>, lds));
    hipLaunchKernelGGL((k_logp<WPC, EX>), dim3((unsigned)grid), dim3(block_of(WPC)), lds, st, ctx_of(p),
                       n, q, lp, g, lds_floats);
    MC_HIP_TRY(hipGetLastError());
    return MC_OK;
}

extern "C" int mc_logp_grad(const mc_program* p, int64_t n_points, const float* q, float* logp,
                            float* grad, void* stream) {
    if (!p) return fail(MC_ERR_INVALID, "program is NULL");
    if (n_points < 0) return fail(MC_ERR_INVALID, "n_points < 0");
    if (n_points == 0) return MC_OK;
    if (!q || !logp || !grad) return fail(MC_ERR_INVALID, "NULL buffer");
    hipStream_t st = (hipStream_t)stream;
    switch (p->wpc) {
        case 1: return p->ex ? launch_logp<1, true>(p, n_points, q, logp, grad, st)
                             : launch_logp<1, false>(p, n_points, q, logp, grad, st);
        case 4: return p->ex ? launch_logp<4, true>(p, n_points, q, logp, grad, st)
                             : launch_logp<4, false>(p, n_points, q, logp, grad, st);
        default: return p->ex ? launch_logp<8, true>(p, n_points, q, logp, grad, st)
                              : launch_logp<8, false>(p, n_points, q, logp, grad, st);
    }
}

// ---------------------------------------------------------------------------
// elementwise Distribution.log_prob
// ---------------------------------------------------------------------------
__global__ void k_dist(int dist, float c0, int64_t n, const float* v, int vb, const float* m,
                       int mb, const float* s, int sb, float* out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const float vv = v[vb ? 0 : i];
        const float ss = s[sb ? 0 : i];
        const float mm = m[mb ? 0 : i];
        const float logs = logf(ss);
        const float lg = lgamma_norm(dist, mm, ss);
        out[i] = elem_eval(dist, c0, vv, mm, ss, logs, lg).lp;
    }
}

extern "C" int mc_dist_log_prob(int32_t dist, int64_t n, const float* v, int32_t vb,
                                const float* m, int32_t mb, const float* s, int32_t sb,
                                float* out, void* stream) {
    if (dist < MC_DIST_NORMAL || dist > MC_DIST_BETA)
        return fail(MC_ERR_INVALID, "unknown distribution %d", dist);
    if (n < 0) return fail(MC_ERR_INVALID, "n < 0");
    if (n == 0) return MC_OK;
    const bool need_m = dist == MC_DIST_NORMAL || dist == MC_DIST_GAMMA || dist == MC_DIST_BETA;
    if (!v || !s || !out || (need_m && !m)) return fail(MC_ERR_INVALID, "NULL operand");
    if (!need_m) mb = 1;  // the unused middle operand is read as element 0 of value
    const float c0 = dist_c0(dist);
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_dist, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, dist,
                       c0, n, v, vb, m ? m : v, mb, s, sb, out);
    MC_HIP_TRY(hipGetLastError());
    return MC_OK;
}

// ---------------------------------------------------------------------------
// state
// ---------------------------------------------------------------------------
static int64_t align256(int64_t x) { return (x + 255) / 256 * 256; }

extern "C" int mc_state_offsets(const mc_program* p, int64_t C, int64_t* q_off, int64_t* g_off) {
    if (!p || C < 0) return fail(MC_ERR_INVALID, "bad arguments");
    const int64_t s = align256(C * (int64_t)sizeof(mc_chain_scalars));
    const int64_t qb = align256(C * p->D * 4);
    if (q_off) *q_off = s;
    if (g_off) *g_off = s + qb;
    return MC_OK;
}

extern "C" int64_t mc_state_bytes(const mc_program* p, int64_t C) {
    if (!p || C < 0) return -1;
    return align256(C * (int64_t)sizeof(mc_chain_scalars)) + 2 * align256(C * p->D * 4);
}

template <int WPC, bool EX>
__global__ void __launch_bounds__(WPC >= 4 ? 64 * WPC : 256)
k_init(DevCtx P, int64_t C, const float* q0, double eps0, float mu, mc_chain_scalars* scal,
       float* st_q, float* st_g, int lds_floats) {
    constexpr int CPB = (WPC >= 4) ? 1 : 4 / WPC;
    constexpr int T = 64 * WPC;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int lc = threadIdx.x / T;
    const int64_t c = (int64_t)blockIdx.x * CPB + lc;
    if (c >= C) return;
    Group<WPC> G;
    SegScratch S;
    G.tid = threadIdx.x % T;
    carve_group<WPC>(smem + (int64_t)lc * lds_floats, G, S);
    const int D = P.D;
    for (int j = G.tid; j < D; j += T) st_q[c * D + j] = q0[c * D + j];
    const float lp = eval_lp_grad<WPC, false, EX>(P, q0 + c * D, st_g + c * D, G, S);
    if (G.tid == 0) {
        mc_chain_scalars sc = {};
        sc.step_size = eps0;
        sc.step_size_bar = 1.0;
        sc.h_bar = 0.0;
        sc.mu = mu;
        sc.logp = lp;
        sc.n_grad = 1;
        scal[c] = sc;
    }
}

template <int WPC, bool EX>
static int launch_init(const mc_program* p, int64_t C, const float* q0, double eps0,
                       void* state, hipStream_t st) {
    int64_t qo, go;
    mc_state_offsets(p, C, &qo, &go);
    char* b = (char*)state;
    const int lds_floats = scratch_of(p);
    const size_t lds = (size_t)cpb_of(WPC) * lds_floats * 4;
    const int64_t grid = (C + cpb_of(WPC) - 1) / cpb_of(WPC);
    const float mu = mc_logf_ref((float)(10.0 * eps0));  // nuts.py:63 mx.log(10 * step_size)
    MC_HIP_TRY(allow_lds(k_init<WPC, EX>, lds));
    hipLaunchKernelGGL((k_init<WPC, EX>), dim3((unsigned)grid), dim3(block_of(WPC)), lds, st,
                       ctx_of(p), C, q0, eps0, mu, (mc_chain_scalars*)b, (float*)(b + qo),
                       (float*)(b + go), lds_floats);
    MC_HIP_TRY(hipGetLastError());
    return MC_OK;
}

extern "C" int mc_state_init(const mc_program* p, int64_t C, const float* q0, double eps0,
                             void* state, void* stream) {
    if (!p || C < 0 || (C > 0 && (!q0 || !state))) return fail(MC_ERR_INVALID, "bad arguments");
    if (C == 0) return MC_OK;
    hipStream_t st = (hipStream_t)stream;
    switch (p->wpc) {
        case 1: return p->ex ? launch_init<1, true>(p, C, q0, eps0, state, st)
                             : launch_init<1, false>(p, C, q0, eps0, state, st);
        case 4: return p->ex ? launch_init<4, true>(p, C, q0, eps0, state, st)
                             : launch_init<4, false>(p, C, q0, eps0, state, st);
        default: return p->ex ? launch_init<8, true>(p, C, q0, eps0, state, st)
                              : launch_init<8, false>(p, C, q0, eps0, state, st);
    }
}




// ---------------------------------------------------------------------------
// RNG fill (test hook and Distribution.sample)
// ---------------------------------------------------------------------------
__global__ void k_rng(uint64_t seed, uint32_t chain, uint32_t iter, uint32_t tag, uint32_t sub,
                      uint32_t index0, int64_t n, int mode, void* out) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
         e += (int64_t)gridDim.x * blockDim.x) {
        const mc_u32x4 r = mc_draw(seed, chain, iter, tag, sub, index0 + (uint32_t)e);
        if (mode == 0) {
            uint32_t* o = (uint32_t*)out + 4 * e;
            o[0] = r.x;
            o[1] = r.y;
            o[2] = r.z;
            o[3] = r.w;
        } else if (mode == 1) {
            float* o = (float*)out + 4 * e;
            o[0] = mc_u01_f32(r.x);
            o[1] = mc_u01_f32(r.y);
            o[2] = mc_u01_f32(r.z);
            o[3] = mc_u01_f32(r.w);
        } else {
            float* o = (float*)out + 4 * e;
            mc_box_muller(r.x, r.y, &o[0], &o[1]);
            mc_box_muller(r.z, r.w, &o[2], &o[3]);
        }
    }
}

extern "C" int mc_rng_fill(uint64_t seed, uint32_t chain, uint32_t iter, uint32_t tag,
                           uint32_t sub, uint32_t index0, int64_t n, int32_t mode, void* out,
                           void* stream) {
    if (n < 0 || (n > 0 && !out) || mode < 0 || mode > 2)
        return fail(MC_ERR_INVALID, "bad arguments");
    if (n == 0) return MC_OK;
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_rng, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, seed,
                       chain, iter, tag, sub, index0, n, mode, out);
    MC_HIP_TRY(hipGetLastError());
    return MC_OK;
}


// ---------------------------------------------------------------------------
// diagnostics (diag.h)
// ---------------------------------------------------------------------------
static int check_csd(int64_t C, int64_t S, int64_t D, const void* x) {
    if (C < 1 || S < 1 || D < 1) return fail(MC_ERR_INVALID, "C, S and D must be >= 1");
    if (!x) return fail(MC_ERR_INVALID, "samples is NULL");
    return MC_OK;
}

extern "C" int mc_series_stats(int64_t C, int64_t S, int64_t D, const float* samples,
                               int32_t max_lag, double* stats, void* stream) {
    if (int rc = check_csd(C, S, D, samples)) return rc;
    if (!stats) return fail(MC_ERR_INVALID, "stats is NULL");
    if (max_lag < 1) return fail(MC_ERR_INVALID, "max_lag must be >= 1");
    const int32_t lmax = (int32_t)std::min<int64_t>(S / 2, max_lag);
    const int64_t blocks = (C * D + 255) / 256;
    hipLaunchKernelGGL(k_series_stats, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                       samples, C, S, D, lmax, stats);
    MC_HIP_TRY(hipGetLastError());
    return MC_OK;
}

extern "C" int mc_stats_reduce(int64_t C, int64_t S, int64_t D, const double* stats,
                               const double* center, int64_t m_total, double* out, void* stream) {
    if (int rc = check_csd(C, S, D, stats)) return rc;
    if (!out) return fail(MC_ERR_INVALID, "out is NULL");
    if (center && (S < 4 || m_total < 2))
        return fail(MC_ERR_INVALID, "split R-hat needs S >= 4 draws and >= 2 half chains");
    hipLaunchKernelGGL(k_stats_reduce, dim3((unsigned)((D + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, stats, C, S, D, center ? 1 : 0, center, m_total, out);
    MC_HIP_TRY(hipGetLastError());
    return MC_OK;
}

extern "C" int mc_rhat(int64_t D, int64_t m_total, int64_t S, const double* spread, double* rhat,
                       void* stream) {
    if (D < 1 || !spread || !rhat) return fail(MC_ERR_INVALID, "bad mc_rhat arguments");
    if (S < 4 || m_total < 2)
        return fail(MC_ERR_INVALID, "split R-hat needs S >= 4 draws and >= 2 half chains");
    hipLaunchKernelGGL(k_rhat, dim3((unsigned)((D + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, spread, D, m_total, S / 2, rhat);
    MC_HIP_TRY(hipGetLastError());
    return MC_OK;
}

extern "C" int mc_pool_moments(int64_t C, int64_t S, int64_t D, const double* stats, int64_t off,
                               int64_t len, double* out, void* stream) {
    if (int rc = check_csd(C, S, D, stats)) return rc;
    if (off < 0 || len < 1 || off + len > D || !out)
        return fail(MC_ERR_INVALID, "element range [%lld, %lld) outside [0, %lld)", (long long)off,
                    (long long)(off + len), (long long)D);
    hipLaunchKernelGGL(k_pool_moments, dim3(1), dim3(256), 0, (hipStream_t)stream, stats, C, S, D,
                       off, len, out);
    MC_HIP_TRY(hipGetLastError());
    return MC_OK;
}

extern "C" int64_t mc_select_workspace_bytes(int32_t nk) {
    if (nk < 1 || nk > kSelMaxTargets) return -1;
    return (int64_t)nk * (int64_t)(sizeof(SelState) + 256 * sizeof(unsigned long long)) + 16;
}

extern "C" int mc_select(int64_t C, int64_t S, int64_t D, const float* samples, int64_t off,
                         int64_t len, int32_t nk, const int64_t* k, float* out, void* ws,
                         int64_t ws_bytes, void* stream) {
    if (int rc = check_csd(C, S, D, samples)) return rc;
    if (off < 0 || len < 1 || off + len > D)
        return fail(MC_ERR_INVALID, "element range outside [0, D)");
    if (nk < 1 || nk > kSelMaxTargets || !k || !out)
        return fail(MC_ERR_INVALID, "nk must be in [1, %d] with k and out set", kSelMaxTargets);
    if (!ws || ws_bytes < mc_select_workspace_bytes(nk))
        return fail(MC_ERR_INVALID, "workspace too small (need %lld bytes)",
                    (long long)mc_select_workspace_bytes(nk));
    const int64_t rows = C * S, n = rows * len;
    SelTargets tg{};
    tg.nk = nk;
    for (int i = 0; i < nk; ++i) {
        if (k[i] < 0 || k[i] >= n)
            return fail(MC_ERR_INVALID, "rank %lld outside [0, %lld)", (long long)k[i], (long long)n);
        tg.k[i] = k[i];
    }
    hipStream_t st = (hipStream_t)stream;
    SelState* stt = (SelState*)ws;
    unsigned long long* hist = (unsigned long long*)(stt + nk);
    uint32_t* nanf = (uint32_t*)(hist + nk * 256);
    hipLaunchKernelGGL(k_sel_init, dim3(1), dim3(256), 0, st, tg, stt, hist, nanf);
    const unsigned blocks = (unsigned)std::min<int64_t>((n + 1023) / 1024, 2048);
    for (int shift = 24; shift >= 0; shift -= 8) {
        hipLaunchKernelGGL(k_sel_hist, dim3(blocks), dim3(256), 0, st, samples, rows, D, off, len,
                           nk, shift, stt, hist, nanf);
        hipLaunchKernelGGL(k_sel_pick, dim3(1), dim3(64), 0, st, nk, shift, stt, hist, nanf,
                           shift == 0 ? out : nullptr);
    }
    MC_HIP_TRY(hipGetLastError());
    return MC_OK;
}

// Host evaluations of the samplers' Box-Muller and uniform log (philox.h:
// the same code the kernels run), for the CPU tests against libm / the oracle.
extern "C" int mc_box_muller_host(const uint32_t* words, int64_t n, float* out) {
    if (n < 0 || (n > 0 && (!words || !out))) return fail(MC_ERR_INVALID, "bad arguments");
    for (int64_t i = 0; i < n; ++i) mc_box_muller(words[2 * i], words[2 * i + 1], &out[2 * i], &out[2 * i + 1]);
    return MC_OK;
}
extern "C" int mc_logf_unit_host(const float* x, int64_t n, float* out) {
    if (n < 0 || (n > 0 && (!x || !out))) return fail(MC_ERR_INVALID, "bad arguments");
    for (int64_t i = 0; i < n; ++i) out[i] = mc_logf_unit(x[i]);
    return MC_OK;
}

extern "C" const char* mc_last_error(void) { return g_last_error.c_str(); }
extern "C" int32_t mc_abi_version(void) { return MC_ABI_VERSION; }
