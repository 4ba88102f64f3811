// run_nuts_sl.h — the sliced NUTS launch (k_nuts_sl, nuts_sliced.h), included
// by run_nuts_sl.hip (the compile-time hierarchical form) and
// run_nuts_sl_rt.hip (the run-time form): two translation units so the
// instantiations compile in parallel.
#pragma once
#include "host.h"
#include "jit.h"

// chains (waves) per workgroup of k_nuts_sl
constexpr int kNslWaves = 8;

// LDS bytes of a k_nuts_sl workgroup: the slice block and scalar terms, then
// per wave the first-leaf arena and the shared parameters' arena rows
inline size_t nuts_sl_lds_bytes(const mc_program* p, int max_depth) {
    return (size_t)p->lr.sdata_floats * 4 + p->lr.sterms.size() * sizeof(LrSterm) +
           (size_t)kNslWaves *
               ((size_t)nuts_sl_first_floats(p->lr.rs, max_depth) +
                (size_t)nuts_sl_shared_rows(max_depth) * 4) * 4;
}

// waves per SIMD the kernel is compiled for: with more than 8 slices two
// workgroups share a CU (4 waves per SIMD, <= 128 VGPRs), so 256 chains of 16
// slices run at once (4096 waves); with <= 8 one workgroup per CU (2 waves
// per SIMD).  Large shape, 256 chains, 16 slices: 21.7 M leaf-steps/s at 4
// waves per SIMD, 14.3 M at 2 (two launches of 128 chains); 8 slices at 2:
// 18.5 M.  MC_NUTS_SL_OCC=2|4 overrides.
inline int nuts_sl_occ(const mc_program* p) {
    if (const char* e = std::getenv("MC_NUTS_SL_OCC")) {
        const int v = std::atoi(e);
        if (v == 2 || v == 4) return v;
    }
    return p->lr.S > 8 ? 4 : 2;
}

// exchange lines (both parities) for every chain block of C chains, then the
// XCD check's slots (16 granules per slice of a block)
inline int64_t nuts_sl_line_bytes(const mc_program* p, int64_t C) {
    const int64_t groups = (C + kNslWaves - 1) / kNslWaves;
    return 2 * groups * kNslWaves * (int64_t)p->lr.S * kNslLine * 8 +
           groups * (int64_t)p->lr.S * 16 * 8;
}

template <int RS, int NSH, int OCC, int FORM>
inline int launch_nuts_sl(const mc_program* p, const mc_run_config* cfg, void* state,
                          float* samples, const mc_trace* tr, void* ws, hipStream_t st) {
    auto kern = k_nuts_sl<RS, NSH, kNslWaves, OCC, FORM>;
    // the compile-time form also with L2-resident records (host.h xcd_round_robin)
    auto kern_xl = kern;
    if constexpr (FORM >= 0) kern_xl = k_nuts_sl<RS, NSH, kNslWaves, OCC, FORM, true>;
    int64_t qo, go;
    mc_state_offsets(p, cfg->num_chains, &qo, &go);
    char* b = (char*)state;
    RunArgs A;
    std::memset(&A, 0, sizeof(A));
    A.cfg = *cfg;
    const LrCtx ctx = lrctx_of(p);
    const int maxj = cfg->max_tree_depth;
    const size_t lds = nuts_sl_lds_bytes(p, maxj);
    MC_HIP_TRY(allow_lds(kern, lds));
    if (kern_xl != kern) MC_HIP_TRY(allow_lds(kern_xl, lds));
    const int64_t C = cfg->num_chains;
    const int64_t groups = (C + kNslWaves - 1) / kNslWaves;
    const int S = p->lr.S;
    const int64_t cap = resident_capacity(kern, 64 * kNslWaves, lds);
    if (cap < S)
        return fail(MC_ERR_UNSUPPORTED,
                    "sliced NUTS: a chain block's %d workgroups must be co-resident, the device "
                    "holds %lld of this kernel", S, (long long)cap);
    const int64_t gpl = std::min(groups, cap / S);
    const int64_t lines = nuts_sl_line_bytes(p, C);
    int* status = (int*)ws;
    unsigned long long* xch = (unsigned long long*)((char*)ws + kSlStatusBytes);
    float* pool = (float*)((char*)ws + kSlStatusBytes + lines);
    A.fault = g_exchange_fault;
    // tags: one per leaf, at most iter_count * 2^maxj leaves per chain
    const uint64_t per_launch = (uint64_t)cfg->iter_count * (1ull << maxj) + 1;
    const int64_t nlaunch = (groups + gpl - 1) / gpl;
    uint32_t base = 0;
    if (ws_reserve(ws, per_launch * (uint64_t)nlaunch, (uint64_t)(kSlStatusBytes + lines), &base))
        MC_HIP_TRY(hipMemsetAsync(ws, 0, kSlStatusBytes + lines, st));
    ws_mark_status(ws);
    for (int64_t g0 = 0; g0 < groups; g0 += gpl) {
        const int64_t ng = std::min(gpl, groups - g0);
        const bool xl = kern_xl != kern && xcd_round_robin(ng * S, S);
        const hipError_t e = launch_exchange(
            xl ? kern_xl : kern, ng * S, 64 * kNslWaves, lds, st, ctx, A, g0 * kNslWaves, ng,
            (mc_chain_scalars*)b, (float*)(b + qo), (float*)(b + go), samples, trace_of(tr), xch,
            pool, status, base);
        MC_HIP_TRY(e);
        base += (uint32_t)per_launch;
    }
    return MC_OK;
}

// The run-time form compiled with the program's expression terms (jit.hip):
// kLanesNoJit when the JIT is off or the compilation failed (the caller runs
// the program on the tape).
template <int RS, int NSH, int OCC>
inline int launch_nuts_sl_jit(const mc_program* p, const mc_run_config* cfg, void* state,
                              float* samples, const mc_trace* tr, void* ws, hipStream_t st) {
    const std::string name = "mc::k_nuts_sl<" + std::to_string(RS) + ", " + std::to_string(NSH) +
                             ", " + std::to_string(kNslWaves) + ", " + std::to_string(OCC) + ", -1";
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
    const int maxj = cfg->max_tree_depth;
    const size_t lds = nuts_sl_lds_bytes(p, maxj);
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
                    "sliced NUTS (expression JIT): a chain block's %d workgroups must be "
                    "co-resident, the device holds %lld of this kernel", S, (long long)cap);
    const int64_t gpl = std::min(groups, cap / S);
    const int64_t lines = nuts_sl_line_bytes(p, C);
    int* status = (int*)ws;
    unsigned long long* xch = (unsigned long long*)((char*)ws + kSlStatusBytes);
    float* pool = (float*)((char*)ws + kSlStatusBytes + lines);
    A.fault = g_exchange_fault;
    const uint64_t per_launch = (uint64_t)cfg->iter_count * (1ull << maxj) + 1;
    const int64_t nlaunch = (groups + gpl - 1) / gpl;
    uint32_t base = 0;
    if (ws_reserve(ws, per_launch * (uint64_t)nlaunch, (uint64_t)(kSlStatusBytes + lines), &base))
        MC_HIP_TRY(hipMemsetAsync(ws, 0, kSlStatusBytes + lines, st));
    ws_mark_status(ws);
    mc_chain_scalars* scal = (mc_chain_scalars*)b;
    float *sq = (float*)(b + qo), *sg = (float*)(b + go);
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
        void* args[] = {&ctx, &A, &cb, &ng, &scal, &sq, &sg, &samples, &td, &xch, &pool, &status,
                        &base};
        MC_HIP_TRY(hipModuleLaunchKernel(k, (unsigned)(ng * S), 1, 1, 64 * kNslWaves, 1, 1,
                                         (unsigned)lds, st, args, nullptr));
        base += (uint32_t)per_launch;
    }
    return MC_OK;
}

// the compile-time hierarchical form (run_nuts_sl.hip) and the run-time form
// (run_nuts_sl_rt.hip)
int nuts_sl_hier(const mc_program* p, const mc_run_config* cfg, void* state, float* samples,
                 const mc_trace* tr, void* ws, hipStream_t st);
int nuts_sl_rt(const mc_program* p, const mc_run_config* cfg, void* state, float* samples,
               const mc_trace* tr, void* ws, hipStream_t st);

// The sliced NUTS kernel runs programs the automatic plan slices (S >= 2)
// onto the fast-form lane layout (k_hmc_lf's programs), unless
// MC_NUTS_SLICED=0 in the environment or mc_debug_nuts_variant(0) (A/B and
// tests: k_nuts on the tape), the slice kernel is forced to the interpreter,
// max_tree_depth is outside [1, kNslMaxDepth] or the LDS arenas do not fit.
inline int g_nuts_sliced = -1;  // mc_debug_nuts_sliced; -1: MC_NUTS_SLICED
inline bool nuts_sliced_enabled() {
    if (g_nuts_sliced < 0) {
        const char* e = std::getenv("MC_NUTS_SLICED");
        g_nuts_sliced = (e && e[0] == '0') ? 0 : 1;
    }
    return g_nuts_sliced == 1;
}
// A program with expression terms (LanePlan::nuts_expr) runs the JIT-compiled
// run-time form (their element code exists only compiled per program): not
// while the JIT is off or after its compilation failed (the tape runs it).
inline bool use_nuts_sliced(const mc_program* p, int max_depth) {
    const bool expr = p->lr.nuts_expr && jit_enabled() && jit_error(p).empty();
    return nuts_sliced_enabled() && p->sl.S >= 2 && p->lr.ok && (p->lr.fast || expr) &&
           lanes_fast_enabled() && p->lr.S >= 2 && p->lr.S <= kLrSlices &&
           p->slice_kernel != 1 && max_depth >= 1 && max_depth <= kNslMaxDepth &&
           nuts_sl_lds_bytes(p, max_depth) <= (size_t)kSlLdsBudget;
}
// status word, exchange lines, then the candidate pool of every chain
inline int64_t nuts_sl_workspace_bytes(const mc_program* p, int64_t C, int max_depth) {
    const int64_t groups = (C + kNslWaves - 1) / kNslWaves;
    return kSlStatusBytes + nuts_sl_line_bytes(p, C) +
           groups * kNslWaves * (int64_t)p->lr.S * nuts_sl_pool_floats(p->lr.rs, max_depth) * 4;
}
