// run_mh_sl.hip — the sliced Metropolis-Hastings launch (k_mh_sl, mh_sliced.h)
// for programs sliced onto the fast-form lane layout.
#include "run_mh_sl.h"

template <int RS, int NSH, int OCC, int FORM>
static int launch_mh_sl(const mc_program* p, const mc_run_config* cfg, float scale, void* state,
                        float* samples, const mc_trace* tr, void* ws, hipStream_t st) {
    auto kern = k_mh_sl<RS, NSH, kNslWaves, OCC, FORM>;
    // the compile-time form also with L2-resident records (host.h xcd_round_robin)
    auto kern_xl = kern;
    if constexpr (FORM >= 0) kern_xl = k_mh_sl<RS, NSH, kNslWaves, OCC, FORM, true>;
    int64_t qo, go;
    mc_state_offsets(p, cfg->num_chains, &qo, &go);
    char* b = (char*)state;
    RunArgs A;
    std::memset(&A, 0, sizeof(A));
    A.cfg = *cfg;
    const LrCtx ctx = lrctx_of(p);
    const size_t lds = (size_t)p->lr.sdata_floats * 4 + p->lr.sterms.size() * sizeof(LrSterm);
    MC_HIP_TRY(allow_lds(kern, lds));
    if (kern_xl != kern) MC_HIP_TRY(allow_lds(kern_xl, lds));
    const int64_t C = cfg->num_chains;
    const int64_t groups = (C + kNslWaves - 1) / kNslWaves;
    const int S = p->lr.S;
    const int64_t cap = resident_capacity(kern, 64 * kNslWaves, lds);
    if (cap < S)
        return fail(MC_ERR_UNSUPPORTED,
                    "sliced MH: a chain block's %d workgroups must be co-resident, the device "
                    "holds %lld of this kernel", S, (long long)cap);
    const int64_t gpl = std::min(groups, cap / S);
    const int64_t lines = mh_sl_line_bytes(p, C);
    int* status = (int*)ws;
    unsigned long long* xch = (unsigned long long*)((char*)ws + kSlStatusBytes);
    A.fault = g_exchange_fault;
    const uint64_t per_launch = (uint64_t)cfg->iter_count + 1;  // one exchange per iteration
    const int64_t nlaunch = (groups + gpl - 1) / gpl;
    uint32_t base = 0;
    if (ws_reserve(ws, per_launch * (uint64_t)nlaunch, (uint64_t)(kSlStatusBytes + lines), &base))
        MC_HIP_TRY(hipMemsetAsync(ws, 0, kSlStatusBytes + lines, st));
    ws_mark_status(ws);
    for (int64_t g0 = 0; g0 < groups; g0 += gpl) {
        const int64_t ng = std::min(gpl, groups - g0);
        const bool xl = kern_xl != kern && xcd_round_robin(ng * S, S);
        const hipError_t e = launch_exchange(xl ? kern_xl : kern, ng * S, 64 * kNslWaves, lds, st,
                                             ctx, A, scale,
                                             g0 * kNslWaves, ng, (mc_chain_scalars*)b,
                                             (float*)(b + qo), samples, trace_of(tr), xch, status,
                                             base);
        MC_HIP_TRY(e);
        base += (uint32_t)per_launch;
    }
    return MC_OK;
}

// The run-time form compiled with the program's expression terms (jit.hip);
// kLanesNoJit when the JIT is off or the compilation failed.
template <int RS, int NSH>
static int launch_mh_sl_jit(const mc_program* p, const mc_run_config* cfg, float scale,
                            void* state, float* samples, const mc_trace* tr, void* ws,
                            hipStream_t st) {
    const std::string name = "mc::k_mh_sl<" + std::to_string(RS) + ", " + std::to_string(NSH) +
                             ", " + std::to_string(kNslWaves) + ", 2, -1";
    hipFunction_t f = nullptr, fxl = nullptr;
    int rc = jit_function(p, name + ", false>", &f);
    if (rc != MC_OK) return rc;
    if (f == nullptr) return kLanesNoJit;
    int64_t qo, go;
    mc_state_offsets(p, cfg->num_chains, &qo, &go);
    char* b = (char*)state;
    RunArgs A;
    std::memset(&A, 0, sizeof(A));
    A.cfg = *cfg;
    LrCtx ctx = lrctx_of(p);
    const size_t lds = (size_t)p->lr.sdata_floats * 4 + p->lr.sterms.size() * sizeof(LrSterm);
    const int64_t C = cfg->num_chains;
    const int64_t groups = (C + kNslWaves - 1) / kNslWaves;
    const int S = p->lr.S;
    int n = 0;
    if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&n, f, 64 * kNslWaves, lds) !=
        hipSuccess)
        n = 0;
    const int64_t cap = (int64_t)n * device_cus();
    if (cap < S)
        return fail(MC_ERR_UNSUPPORTED,
                    "sliced MH (expression JIT): a chain block's %d workgroups must be "
                    "co-resident, the device holds %lld of this kernel", S, (long long)cap);
    const int64_t gpl = std::min(groups, cap / S);
    const int64_t lines = mh_sl_line_bytes(p, C);
    int* status = (int*)ws;
    unsigned long long* xch = (unsigned long long*)((char*)ws + kSlStatusBytes);
    A.fault = g_exchange_fault;
    const uint64_t per_launch = (uint64_t)cfg->iter_count + 1;
    const int64_t nlaunch = (groups + gpl - 1) / gpl;
    uint32_t base = 0;
    if (ws_reserve(ws, per_launch * (uint64_t)nlaunch, (uint64_t)(kSlStatusBytes + lines), &base))
        MC_HIP_TRY(hipMemsetAsync(ws, 0, kSlStatusBytes + lines, st));
    ws_mark_status(ws);
    mc_chain_scalars* scal = (mc_chain_scalars*)b;
    float* sq = (float*)(b + qo);
    TraceDev td = trace_of(tr);
    for (int64_t g0 = 0; g0 < groups; g0 += gpl) {
        int64_t ng = std::min(gpl, groups - g0);
        int64_t cb = g0 * kNslWaves;
        hipFunction_t k = f;
        if (xcd_round_robin(ng * S, S)) {
            if (fxl == nullptr) {
                rc = jit_function(p, name + ", true>", &fxl);
                if (rc != MC_OK) return rc;
            }
            if (fxl != nullptr) k = fxl;
        }
        void* args[] = {&ctx, &A, &scale, &cb, &ng, &scal, &sq, &samples, &td, &xch, &status,
                        &base};
        MC_HIP_TRY(hipModuleLaunchKernel(k, (unsigned)(ng * S), 1, 1, 64 * kNslWaves, 1, 1,
                                         (unsigned)lds, st, args, nullptr));
        base += (uint32_t)per_launch;
    }
    return MC_OK;
}

int mh_sliced_run(const mc_program* p, const mc_run_config* cfg, float scale, void* state,
                  float* samples, const mc_trace* tr, void* ws, hipStream_t st) {
    if (!p->lr.fast) {  // expression terms (LanePlan::nuts_expr): the JIT-compiled form
        const bool n4x = p->lr.Dsh > 3;
        switch (p->lr.rs) {
            case 1: return n4x ? launch_mh_sl_jit<1, 4>(p, cfg, scale, state, samples, tr, ws, st)
                               : launch_mh_sl_jit<1, 3>(p, cfg, scale, state, samples, tr, ws, st);
            case 2: return n4x ? launch_mh_sl_jit<2, 4>(p, cfg, scale, state, samples, tr, ws, st)
                               : launch_mh_sl_jit<2, 3>(p, cfg, scale, state, samples, tr, ws, st);
            default: return n4x ? launch_mh_sl_jit<4, 4>(p, cfg, scale, state, samples, tr, ws, st)
                                : launch_mh_sl_jit<4, 3>(p, cfg, scale, state, samples, tr, ws, st);
        }
    }
    constexpr int HIER = LF_SW | LF_SWS | LF_DIR | LF_DM | LF_DS;
    const bool hier = p->lr.form == HIER && lanes_forms_enabled();
    const bool o4 = nuts_sl_occ(p) == 4;
    const bool n4 = p->lr.Dsh > 3;
#define MC_MH_SL(RS_)                                                                          \
    if (hier) return o4 ? launch_mh_sl<RS_, 3, 4, HIER>(p, cfg, scale, state, samples, tr, ws, st) \
                        : launch_mh_sl<RS_, 3, 2, HIER>(p, cfg, scale, state, samples, tr, ws, st); \
    return n4 ? launch_mh_sl<RS_, 4, 2, -1>(p, cfg, scale, state, samples, tr, ws, st)             \
              : launch_mh_sl<RS_, 3, 2, -1>(p, cfg, scale, state, samples, tr, ws, st)
    switch (p->lr.rs) {
        case 1: MC_MH_SL(1);
        case 2: MC_MH_SL(2);
        default: MC_MH_SL(4);
    }
#undef MC_MH_SL
}
