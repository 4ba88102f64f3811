// run_nuts.hip — NUTS launches (k_nuts_lr, k_nuts) and mc_nuts_run.
#include "run_nuts_sl.h"
#include "jit.h"


// LDS floats per chain group of k_nuts: group scratch, pending words and,
// with the LDS arena, the trajectory arena
static int64_t nuts_lds_floats(const mc_program* p, int32_t max_depth, bool lds_arena) {
    return scratch_of(p) + kNutsLdsWords +
           (lds_arena ? nuts_arena_vectors(max_depth) * (int64_t)dpad_of(p->D) : 0);
}
// The arena goes to LDS when a workgroup's share fits 150 KB (one workgroup
// per CU: NUTS runs few chains — 64 per GPU in config 5 — so occupancy is not
// what bounds it; the L2 round trips of a global arena are)
static constexpr int64_t kNutsLdsBudget = 150 * 1024;
static bool nuts_use_lds(const mc_program* p, int32_t max_depth) {
    return cpb_of(p->wpc) * nuts_lds_floats(p, max_depth, true) * 4 <= kNutsLdsBudget;
}

extern "C" int64_t mc_nuts_workspace_bytes(const mc_program* p, int64_t C, int32_t max_depth) {
    if (!p || C < 0 || max_depth < 0 || max_depth > kMaxTreeDepth) return -1;
    const int64_t tape =
        nuts_use_lds(p, max_depth) ? 0 : C * nuts_arena_vectors(max_depth) * (int64_t)dpad_of(p->D) * 4;
    // (an expression program's sliced launch may fall back to the tape: jit.hip)
    if (use_nuts_sliced(p, max_depth))
        return std::max(nuts_sl_workspace_bytes(p, C, max_depth), p->lr.fast ? 0 : tape);
    return tape;
}

template <int WPC, bool LDS, bool EX>
static int launch_nuts(const mc_program* p, const mc_run_config* cfg, void* state,
                       float* samples, const mc_trace* tr, float* ws, hipStream_t st) {
    int64_t qo, go;
    mc_state_offsets(p, cfg->num_chains, &qo, &go);
    char* b = (char*)state;
    RunArgs A;
    std::memset(&A, 0, sizeof(A));
    A.cfg = *cfg;
    A.dpad = dpad_of(p->D);
    A.scratch_floats = scratch_of(p);
    A.lds_floats = (int32_t)nuts_lds_floats(p, cfg->max_tree_depth, LDS);
    size_t lds = (size_t)cpb_of(WPC) * A.lds_floats * 4;
    // the data pool after the chain groups when it fits as well
    const size_t dbytes = (p->h_data.size() + 3) / 4 * 16;
    A.data_lds = 0;
    if (LDS && lds + dbytes <= (size_t)kNutsLdsBudget) {
        A.data_lds = (int32_t)p->h_data.size();
        lds += dbytes;
    }
    const int64_t grid = (cfg->num_chains + cpb_of(WPC) - 1) / cpb_of(WPC);
    // the program's expression terms compiled (jit.hip), with at most the
    // default 64 KB of dynamic LDS (module kernels launch without the
    // attribute allow_lds sets)
    if (EX && lds <= 64 * 1024) {
        DevCtx ctx = ctx_of(p);
        mc_chain_scalars* scal = (mc_chain_scalars*)b;
        float *sq = (float*)(b + qo), *sg = (float*)(b + go);
        TraceDev td = trace_of(tr);
        void* args[] = {&ctx, &A, &scal, &sq, &sg, &samples, &td, &ws};
        bool used = false;
        const int rc = jit_launch(p, "mc::k_nuts<" + std::to_string(WPC) + ", " +
                                         (LDS ? "true" : "false") + ", true>",
                                  (unsigned)grid, block_of(WPC), lds, st, args, &used);
        if (rc != MC_OK || used) return rc;
    }
    MC_HIP_TRY(allow_lds(k_nuts<WPC, LDS, EX>, lds));
    hipLaunchKernelGGL((k_nuts<WPC, LDS, EX>), dim3((unsigned)grid), dim3(block_of(WPC)), lds, st,
                       ctx_of(p), A, (mc_chain_scalars*)b, (float*)(b + qo), (float*)(b + go),
                       samples, trace_of(tr), ws);
    MC_HIP_TRY(hipGetLastError());
    return MC_OK;
}

// The lane-resident NUTS kernel (nuts_lanes.h) for programs planned as one
// lane-resident slice (the layout k_hmc_lr runs with X1), unless
// MC_NUTS_LANES=0 in the environment (A/B timing against k_nuts) or the
// arena does not fit the LDS budget.
static bool nuts_lanes_enabled() {
    static int on = -1;
    if (on < 0) {
        const char* e = std::getenv("MC_NUTS_LANES");
        on = (e && e[0] == '0') ? 0 : 1;
    }
    return on == 1;
}
static size_t nuts_lr_lds_bytes(const mc_program* p, int max_depth) {
    return (size_t)p->lr.sdata_floats * 4 + p->lr.sterms.size() * sizeof(LrSterm) +
           (size_t)nuts_lr_arena_floats(p->lr.rs, max_depth) * 4;
}
static bool use_nuts_lanes(const mc_program* p, int max_depth) {
    return nuts_lanes_enabled() && p->sl.S < 2 && p->lr.ok && p->lr.S == 1 && !p->lr.has_xf &&
           p->slice_kernel != 1 && nuts_lr_lds_bytes(p, max_depth) <= (size_t)kSlLdsBudget;
}
// no broadcast parameter, no scalar term and one slice term with at most one
// element per (lane, slot): a data-scale term or a direct term with constant
// loc and scale (k_nuts_lr<..., 2>: the gradient from per-slot registers)
static bool lanes_register_only(const mc_program* p) {
    const LanePlan& L = p->lr;
    if (!L.ok || L.S != 1 || L.Dsh != 0 || !L.sterms.empty() || L.blocks[2] != 1) return false;
    const LrTerm& T = L.terms[0];
    const bool ds = T.sig == LS_DSCALE && T.kind[1 - T.pp] != SK_SHARED;
    const bool dir = T.sig == LS_PP_C_C && T.pp == 0;
    if (!ds && !dir) return false;
    const int32_t* lens = (const int32_t*)&L.data[(size_t)L.blocks[0] + T.len_off];
    for (int i = 0; i < T.nslot * 64; ++i)
        if (lens[i] > 1) return false;
    return true;
}

extern "C" int32_t mc_program_nuts_lanes(const mc_program* p, int32_t max_tree_depth) {
    if (!p) return -1;
    if (use_nuts_sliced(p, max_tree_depth)) return 3;
    if (!use_nuts_lanes(p, max_tree_depth)) return 0;
    return lanes_register_only(p) ? 2 : 1;
}

// every slice term of the one-slice lane plan has a specialised form and
// every scalar term is an own prior (k_nuts_lr<..., SPEC>)
static bool lanes_specialised(const mc_program* p) {
    const LanePlan& L = p->lr;
    if (L.n_generic != 0 || L.S != 1) return false;
    const int nact = (int)L.blocks[2];
    for (int t = 0; t < nact; ++t)
        if (L.terms[t].sig == LS_GENERIC) return false;
    return true;
}

extern "C" int mc_debug_nuts_sliced(int on) {
    g_nuts_sliced = on < 0 ? -1 : (on ? 1 : 0);
    return MC_OK;
}

// k_nuts_lr's draw wave for the register-only variant: MC_NUTS_DRAW_WAVE=0 in
// the environment keeps one wave per chain (A/B)
static bool nuts_draw_wave_enabled() {
    static const int on = [] {
        const char* e = std::getenv("MC_NUTS_DRAW_WAVE");
        return (e && e[0] == '0') ? 0 : 1;
    }();
    return on == 1;
}

static int g_nuts_variant = -1;  // mc_debug_nuts_variant
extern "C" int mc_debug_nuts_variant(int variant) {
    g_nuts_variant = (variant < -1 || variant > 1) ? -1 : variant;
    return MC_OK;
}

template <int RS, int NSH>
static int launch_nuts_lr(const mc_program* p, const mc_run_config* cfg, void* state,
                          float* samples, const mc_trace* tr, hipStream_t st) {
    int64_t qo, go;
    mc_state_offsets(p, cfg->num_chains, &qo, &go);
    char* b = (char*)state;
    RunArgs A;
    std::memset(&A, 0, sizeof(A));
    A.cfg = *cfg;
    size_t lds = nuts_lr_lds_bytes(p, cfg->max_tree_depth);
    // the draw wave (nuts_lanes.h PW) when its buffers fit
    const size_t lds_pw = lds + (size_t)nuts_lr_draw_words(cfg->max_tree_depth) * 4;
    const bool pw = nuts_draw_wave_enabled() && cfg->max_tree_depth <= 12 &&
                    lds_pw <= (size_t)kSlLdsBudget;
    auto kern = lanes_specialised(p) ? (pw ? k_nuts_lr<RS, NSH, 1, true> : k_nuts_lr<RS, NSH, 1>)
                                     : (pw ? k_nuts_lr<RS, NSH, 0, true> : k_nuts_lr<RS, NSH, 0>);
    if constexpr (NSH == 3)
        if (lanes_register_only(p) && g_nuts_variant < 0)
            kern = pw ? k_nuts_lr<RS, NSH, 2, true> : k_nuts_lr<RS, NSH, 2>;
    if (g_nuts_variant == 0) kern = pw ? k_nuts_lr<RS, NSH, 0, true> : k_nuts_lr<RS, NSH, 0>;
    if (pw) lds = lds_pw;
    const int threads = pw ? 128 : 64;
    MC_HIP_TRY(allow_lds(kern, lds));
    hipLaunchKernelGGL(kern, dim3((unsigned)cfg->num_chains), dim3(threads), lds, st, lrctx_of(p), A,
                       (mc_chain_scalars*)b, (float*)(b + qo), (float*)(b + go), samples,
                       trace_of(tr));
    MC_HIP_TRY(hipGetLastError());
    return MC_OK;
}

extern "C" int mc_nuts_run(const mc_program* p, const mc_run_config* cfg, void* state,
                           float* samples, const mc_trace* tr, void* ws, int64_t ws_bytes,
                           void* stream) {
    int rc = check_cfg(p, cfg, state);
    if (rc) return rc;
    if (cfg->max_tree_depth < 0 || cfg->max_tree_depth > kMaxTreeDepth)
        return fail(MC_ERR_UNSUPPORTED, "max_tree_depth must be in [0, %d]", kMaxTreeDepth);
    if (cfg->num_chains == 0 || cfg->iter_count == 0) return MC_OK;
    const int64_t need = mc_nuts_workspace_bytes(p, cfg->num_chains, cfg->max_tree_depth);
    if (need > 0 && (ws == nullptr || ws_bytes < need))
        return fail(MC_ERR_INVALID, "workspace too small: need %lld bytes", (long long)need);
    hipStream_t st = (hipStream_t)stream;
    if (use_nuts_sliced(p, cfg->max_tree_depth)) {
        // (tags continue on this workspace: no ws_forget, nuts_sliced.h)
        if (device_cus() <= 0) return fail(MC_ERR_HIP, "no HIP device");
        constexpr int HIER = LF_SW | LF_SWS | LF_DIR | LF_DM | LF_DS;
        const int rc_sl = (p->lr.fast && p->lr.form == HIER && lanes_forms_enabled())
                              ? nuts_sl_hier(p, cfg, state, samples, tr, ws, st)
                              : nuts_sl_rt(p, cfg, state, samples, tr, ws, st);
        if (rc_sl != kLanesNoJit) return rc_sl;
        // (expression terms without their compiled kernel: the tape below)
    }
    if (ws) ws_forget(ws);  // another kernel's data: a later sliced launch clears it
    if (use_nuts_lanes(p, cfg->max_tree_depth)) {
        const bool n4 = p->lr.Dsh > 3;
        switch (p->lr.rs) {
            case 1: return n4 ? launch_nuts_lr<1, 4>(p, cfg, state, samples, tr, st)
                              : launch_nuts_lr<1, 3>(p, cfg, state, samples, tr, st);
            case 2: return n4 ? launch_nuts_lr<2, 4>(p, cfg, state, samples, tr, st)
                              : launch_nuts_lr<2, 3>(p, cfg, state, samples, tr, st);
            default: return n4 ? launch_nuts_lr<4, 4>(p, cfg, state, samples, tr, st)
                               : launch_nuts_lr<4, 3>(p, cfg, state, samples, tr, st);
        }
    }
    float* w = (float*)ws;
    const bool lds = nuts_use_lds(p, cfg->max_tree_depth);
    return dispatch_tape(p, lds, [&](auto W, auto L, auto E) {
        return launch_nuts<decltype(W)::value, decltype(L)::value, decltype(E)::value>(
            p, cfg, state, samples, tr, w, st);
    });
}

#ifdef MC_STAMPS
MC_STAMPS_EXPORT(mc_debug_stamps_nuts, mc_debug_stamps_nuts_wg)
#endif
