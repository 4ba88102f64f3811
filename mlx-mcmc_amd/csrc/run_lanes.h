// run_lanes.h — the lane-resident HMC launch (k_hmc_lf / k_hmc_lr), included by
// run_lanes_rs{1,2,4}.hip: one translation unit per register-slot count, so
// the instantiations compile in parallel.
#pragma once
#include "host.h"
#include "jit.h"


// workgroups of a JIT-compiled kernel the device holds at once
inline int64_t resident_capacity_fn(hipFunction_t f, int block, size_t lds) {
    int n = 0;
    if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&n, f, block, lds) != hipSuccess)
        return -1;
    return (int64_t)n * device_cus();
}

template <int RS, int NSH, int NW, bool X1>
inline int launch_hmc_lr_jit(const mc_program* p, const mc_run_config* cfg, void* state,
                             float* samples, const mc_trace* tr, void* ws, hipStream_t st) {
    const std::string name = "mc::k_hmc_lr<" + std::to_string(RS) + ", " + std::to_string(NSH) +
                             ", " + std::to_string(NW) + ", " + (X1 ? "true" : "false");
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
    constexpr int NB = 2 * NW;
    const int64_t groups = (C + NB - 1) / NB;
    const int64_t gpl = lr_groups_per_launch(p, C);
    const int64_t used = sl_workspace_bytes(p, C);
    int* status = (int*)ws;
    unsigned long long* xch = (unsigned long long*)((char*)ws + kSlStatusBytes);
    const uint64_t per_launch = (uint64_t)cfg->iter_count * cfg->num_leapfrog_steps + 1;
    const int64_t nlaunch = (groups + gpl - 1) / gpl;
    if (!X1) {
        const int64_t cap = resident_capacity_fn(f, 64 * NW, lds);
        if (cap < std::min(gpl, groups) * p->lr.S)
            return fail(MC_ERR_UNSUPPORTED,
                        "lane-resident HMC (expression JIT): %lld workgroups must be co-resident, "
                        "the device holds %lld of this kernel",
                        (long long)(std::min(gpl, groups) * p->lr.S), (long long)cap);
        A.fault = g_exchange_fault;
    }
    uint32_t base = 0;
    if (ws_reserve(ws, per_launch * (uint64_t)nlaunch, (uint64_t)used, &base))
        MC_HIP_TRY(hipMemsetAsync(ws, 0, used, st));
    ws_mark_status(ws);
    mc_chain_scalars* scal = (mc_chain_scalars*)b;
    float *sq = (float*)(b + qo), *sg = (float*)(b + go);
    TraceDev td = trace_of(tr);
    for (int64_t g0 = 0; g0 < groups; g0 += gpl) {
        int64_t ng = std::min(gpl, groups - g0);
        const int64_t grid = ng * p->lr.S;
        int64_t cb = g0 * NB;
        hipFunction_t k = f;
        if (!X1 && xcd_round_robin(grid, p->lr.S)) {
            if (fxl == nullptr) {
                rc = jit_function(p, name + ", true>", &fxl);
                if (rc != MC_OK) return rc;
            }
            if (fxl != nullptr) k = fxl;
        }
        void* args[] = {&ctx, &A, &cb, &ng, &scal, &sq, &sg, &samples, &td, &xch, &status, &base};
        MC_HIP_TRY(hipModuleLaunchKernel(k, (unsigned)grid, 1, 1, 64 * NW, 1, 1, (unsigned)lds, st,
                                         args, nullptr));
        base += (uint32_t)per_launch;
    }
    return MC_OK;
}

template <int RS, int NSH, int NW, bool X1>
inline int launch_hmc_lr(const mc_program* p, const mc_run_config* cfg, void* state,
                         float* samples, const mc_trace* tr, void* ws, hipStream_t st) {
    if (p->lr.has_expr) return launch_hmc_lr_jit<RS, NSH, NW, X1>(p, cfg, state, samples, tr, ws, st);
    const bool fast = p->lr.fast && lanes_fast_enabled();
    auto kern = fast ? k_hmc_lf<RS, NSH, NW, X1, -1> : k_hmc_lr<RS, NSH, NW, X1>;
    // the same with L2-resident records (host.h xcd_round_robin): the generic
    // kernel and the compile-time forms (the run-time form keeps sc1 records)
    auto kern_xl = (fast || X1) ? kern : k_hmc_lr<RS, NSH, NW, X1, true>;
    const bool forms = lanes_forms_enabled();
    if constexpr (NSH == 3) {  // the compile-time forms (one instantiation each)
        constexpr int HIER = LF_SW | LF_SWS | LF_DIR | LF_DM | LF_DS;
        if (fast && forms && p->lr.form == HIER) {
            kern = k_hmc_lf<RS, lf_nroles(HIER), NW, X1, HIER>;
            kern_xl = X1 ? kern : k_hmc_lf<RS, lf_nroles(HIER), NW, X1, HIER, true>;
        }
        if (fast && forms && p->lr.form == LF_DIR) {
            kern = k_hmc_lf<RS, lf_nroles(LF_DIR), NW, X1, LF_DIR>;
            kern_xl = X1 ? kern : k_hmc_lf<RS, lf_nroles(LF_DIR), NW, X1, LF_DIR, true>;
        }
    }
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
    constexpr int NB = 2 * NW;
    const int64_t groups = (C + NB - 1) / NB;
    const int64_t gpl = lr_groups_per_launch(p, C);
    const int64_t used = sl_workspace_bytes(p, C);
    int* status = (int*)ws;
    unsigned long long* xch = (unsigned long long*)((char*)ws + kSlStatusBytes);
    const uint64_t per_launch = (uint64_t)cfg->iter_count * cfg->num_leapfrog_steps + 1;
    const int64_t nlaunch = (groups + gpl - 1) / gpl;
    if (!X1) {
        const int64_t cap = resident_capacity(kern, 64 * NW, lds);
        if (cap < std::min(gpl, groups) * p->lr.S)
            return fail(MC_ERR_UNSUPPORTED,
                        "lane-resident HMC: %lld workgroups must be co-resident, the device holds "
                        "%lld of this kernel", (long long)(std::min(gpl, groups) * p->lr.S),
                        (long long)cap);
        A.fault = g_exchange_fault;
    }
    uint32_t base = 0;
    if (ws_reserve(ws, per_launch * (uint64_t)nlaunch, (uint64_t)used, &base))
        MC_HIP_TRY(hipMemsetAsync(ws, 0, used, st));  // status word and granule lines
    ws_mark_status(ws);
    for (int64_t g0 = 0; g0 < groups; g0 += gpl) {
        const int64_t ng = std::min(gpl, groups - g0);
        const int64_t grid = ng * p->lr.S;
        if (X1) {
            hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(64 * NW), lds, st, ctx, A,
                               g0 * NB, ng, (mc_chain_scalars*)b, (float*)(b + qo),
                               (float*)(b + go), samples, trace_of(tr), xch, status, base);
            MC_HIP_TRY(hipGetLastError());
        } else {
            const bool xl = kern_xl != kern && xcd_round_robin(grid, p->lr.S);
            const hipError_t e = launch_exchange(
                xl ? kern_xl : kern, grid, 64 * NW, lds, st, ctx, A, g0 * NB, ng,
                (mc_chain_scalars*)b, (float*)(b + qo), (float*)(b + go), samples, trace_of(tr),
                xch, status, base);
            MC_HIP_TRY(e);
        }
        base += (uint32_t)per_launch;
    }
    return MC_OK;
}


// NSH (3 or 4 shared parameters) x waves per workgroup (one slice: 1 wave and
// no exchange; <= 8 slices: 4; else 8)
template <int RS>
inline int hmc_lanes_dispatch(const mc_program* p, const mc_run_config* cfg, void* state,
                              float* samples, const mc_trace* tr, void* ws, hipStream_t st) {
    const bool n4 = p->lr.Dsh > 3, w4 = lr_nw(p) == 4, x1 = p->lr.S == 1;
#define MC_LR(NSH_)                                                                        \
    return x1 ? launch_hmc_lr<RS, NSH_, 1, true>(p, cfg, state, samples, tr, ws, st)       \
         : w4 ? launch_hmc_lr<RS, NSH_, 4, false>(p, cfg, state, samples, tr, ws, st)      \
              : launch_hmc_lr<RS, NSH_, 8, false>(p, cfg, state, samples, tr, ws, st)
    if (n4) MC_LR(4);
    MC_LR(3);
#undef MC_LR
}
