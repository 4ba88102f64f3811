// run_mh.hip — Metropolis-Hastings launches (k_mh) and mc_mh_run.
#include "host.h"
#include "jit.h"
#include "run_mh_sl.h"

// ---- Metropolis-Hastings (metropolis.py:6-101) --------------------------------
static int64_t mh_lds_floats(const mc_program* p, bool lds_arena) {
    return scratch_of(p) + (lds_arena ? 2 * (int64_t)dpad_of(p->D) : 0);
}
static bool mh_use_lds(const mc_program* p) {
    return cpb_of(p->wpc) * mh_lds_floats(p, true) * 4 <= kLdsArenaBudget;
}

extern "C" int mc_debug_mh_sliced(int on) {
    g_mh_sliced = on < 0 ? -1 : (on ? 1 : 0);
    return MC_OK;
}

extern "C" int32_t mc_program_mh_sliced(const mc_program* p) {
    if (!p) return -1;
    return use_mh_sliced(p) ? 1 : 0;
}

extern "C" int64_t mc_mh_workspace_bytes(const mc_program* p, int64_t C) {
    if (!p || C < 0) return -1;
    const int64_t tape = mh_use_lds(p) ? 0 : C * 2 * (int64_t)dpad_of(p->D) * 4;
    // (an expression program's sliced launch may fall back to the tape: jit.hip)
    if (use_mh_sliced(p)) return std::max(mh_sl_workspace_bytes(p, C), p->lr.fast ? 0 : tape);
    return tape;
}

template <int WPC, bool LDS, bool EX>
static int launch_mh(const mc_program* p, const mc_run_config* cfg, float scale, void* state,
                     float* samples, const mc_trace* tr, float* ws, hipStream_t st) {
    int64_t qo, go;
    mc_state_offsets(p, cfg->num_chains, &qo, &go);
    char* b = (char*)state;
    RunArgs A;
    std::memset(&A, 0, sizeof(A));
    A.cfg = *cfg;
    A.dpad = dpad_of(p->D);
    A.lds_floats = (int32_t)mh_lds_floats(p, LDS);
    A.scratch_floats = scratch_of(p);
    const size_t lds = (size_t)cpb_of(WPC) * A.lds_floats * 4;
    const int64_t grid = (cfg->num_chains + cpb_of(WPC) - 1) / cpb_of(WPC);
    if constexpr (EX) {  // the program's expression terms compiled (jit.hip)
        DevCtx ctx = ctx_of(p);
        mc_chain_scalars* scal = (mc_chain_scalars*)b;
        float* sq = (float*)(b + qo);
        TraceDev td = trace_of(tr);
        void* args[] = {&ctx, &A, &scale, &scal, &sq, &samples, &td, &ws};
        bool used = false;
        const int rc = jit_launch(p, "mc::k_mh<" + std::to_string(WPC) + ", " +
                                         (LDS ? "true" : "false") + ", true>",
                                  (unsigned)grid, block_of(WPC), lds, st, args, &used);
        if (rc != MC_OK || used) return rc;
    }
    MC_HIP_TRY(allow_lds(k_mh<WPC, LDS, EX>, lds));
    hipLaunchKernelGGL((k_mh<WPC, LDS, EX>), dim3((unsigned)grid), dim3(block_of(WPC)), lds, st,
                       ctx_of(p), A, scale, (mc_chain_scalars*)b, (float*)(b + qo), samples,
                       trace_of(tr), ws);
    MC_HIP_TRY(hipGetLastError());
    return MC_OK;
}

extern "C" int mc_mh_run(const mc_program* p, const mc_run_config* cfg, double proposal_scale,
                         void* state, float* samples, const mc_trace* tr, void* ws,
                         int64_t ws_bytes, void* stream) {
    int rc = check_cfg(p, cfg, state);
    if (rc) return rc;
    if (!std::isfinite(proposal_scale)) return fail(MC_ERR_INVALID, "proposal_scale not finite");
    if (cfg->num_chains == 0 || cfg->iter_count == 0) return MC_OK;
    if (use_mh_sliced(p)) {
        const int64_t need = mh_sl_workspace_bytes(p, cfg->num_chains);
        if (ws == nullptr || ws_bytes < need)
            return fail(MC_ERR_INVALID, "workspace too small: need %lld bytes", (long long)need);
        if (device_cus() <= 0) return fail(MC_ERR_HIP, "no HIP device");
        const int rc_sl = mh_sliced_run(p, cfg, (float)proposal_scale, state, samples, tr, ws,
                                        (hipStream_t)stream);
        if (rc_sl != kLanesNoJit) return rc_sl;
        // (expression terms without their compiled kernel: the tape below)
    }
    const bool lds = mh_use_lds(p);
    const int64_t need = mc_mh_workspace_bytes(p, cfg->num_chains);
    if (!lds && (ws == nullptr || ws_bytes < need))
        return fail(MC_ERR_INVALID, "workspace too small: need %lld bytes", (long long)need);
    ws_forget(ws);  // another kernel's data: a later sliced launch clears it
    hipStream_t st = (hipStream_t)stream;
    float* w = (float*)ws;
    const float sc = (float)proposal_scale;  // f32(proposal_scale): MLX's weak scalar
    return dispatch_tape(p, lds, [&](auto W, auto L, auto E) {
        return launch_mh<decltype(W)::value, decltype(L)::value, decltype(E)::value>(
            p, cfg, sc, state, samples, tr, w, st);
    });
}
