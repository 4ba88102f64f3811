// run_hmc.hip — HMC launches (k_hmc_lf, k_hmc_lr, k_hmc_sl, k_hmc) and mc_hmc_run.
#include "host.h"
#include "jit.h"

extern "C" int mc_workspace_release(const void* ws) {
    if (ws) ws_forget(ws);
    return MC_OK;
}

extern "C" int mc_debug_exchange_fault(int on) {
    g_exchange_fault = on ? 1 : 0;
    return MC_OK;
}

// Exchange groups (blocks, counted by slice 0) launched on the workspace
// since it was last cleared that were found on one XCD (L2-resident
// publishes) / not (sliced.h xcd_agree): the status area's words 8 and 9.
extern "C" int mc_debug_workspace_xcd(const void* ws, int32_t* local, int32_t* remote) {
    if (!ws) return fail(MC_ERR_INVALID, "workspace is NULL");
    int32_t w[2] = {0, 0};
    MC_HIP_TRY(hipMemcpy(w, (const int32_t*)ws + 8, sizeof(w), hipMemcpyDeviceToHost));
    if (local) *local = w[0];
    if (remote) *remote = w[1];
    return MC_OK;
}

// host.h: the device deals workgroups round-robin over its XCDs (probe)
static __global__ void k_xcc_probe(uint32_t* out) {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    if (threadIdx.x == 0) out[blockIdx.x] = x;
}
bool xcd_round_robin(int64_t grid, int S) {
    if (g_xcd_local < 0) {
        const char* e = std::getenv("MC_XCD_LOCAL");
        g_xcd_local = (e && e[0] == '0') ? 0 : 1;
    }
    if (g_xcd_local == 0 || S < 2 || grid % 8 != 0 || (grid / 8) % S != 0) return false;
    static std::mutex mu;
    static std::map<std::pair<int, int64_t>, bool> cache;
    int dev = 0;
    (void)hipGetDevice(&dev);
    const auto key = std::make_pair(dev, grid);
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    bool ok = false;
    uint32_t* d = nullptr;
    if (hipMalloc(&d, grid * sizeof(uint32_t)) == hipSuccess) {
        std::vector<uint32_t> h((size_t)grid, 0xFFFFFFFFu);
        hipLaunchKernelGGL(k_xcc_probe, dim3((unsigned)grid), dim3(64), 0, 0, d);
        if (hipGetLastError() == hipSuccess &&
            hipMemcpy(h.data(), d, grid * sizeof(uint32_t), hipMemcpyDeviceToHost) == hipSuccess) {
            ok = true;
            for (int64_t b = 8; b < grid && ok; ++b) ok = h[b] == h[b % 8];
        }
        (void)hipFree(d);
    }
    (void)hipGetLastError();
    cache[key] = ok;
    return ok;
}

extern "C" int mc_debug_xcd_local(int on) {
    g_xcd_local = on < 0 ? -1 : (on ? 1 : 0);
    return MC_OK;
}

extern "C" int mc_debug_lanes_fast(int on) {
    g_lanes_fast = on ? 1 : 0;
    return MC_OK;
}

extern "C" int mc_debug_lanes_forms(int on) {
    g_lanes_forms = on ? 1 : 0;
    return MC_OK;
}

template <int NB>
static int launch_hmc_sl(const mc_program* p, const mc_run_config* cfg, void* state,
                         float* samples, const mc_trace* tr, void* ws, hipStream_t st) {
    if (!interp_ok(p))
        return fail(MC_ERR_UNSUPPORTED, "the term interpreter does not run transformed operands "
                    "or affine locs");
    int64_t qo, go;
    mc_state_offsets(p, cfg->num_chains, &qo, &go);
    char* b = (char*)state;
    RunArgs A;
    std::memset(&A, 0, sizeof(A));
    A.cfg = *cfg;
    const SlCtx ctx = slctx_of(p);
    const size_t lds = (size_t)SlLayout<NB>(ctx).total * 4;
    MC_HIP_TRY(allow_lds(k_hmc_sl<NB>, lds));
    const int64_t C = cfg->num_chains;
    const int64_t groups = (C + NB - 1) / NB;
    const int64_t gpl = sl_groups_per_launch(p, C);
    const int64_t used = sl_workspace_bytes(p, C);
    int* status = (int*)ws;
    unsigned long long* xch = (unsigned long long*)((char*)ws + kSlStatusBytes);
    const int64_t cap = resident_capacity(k_hmc_sl<NB>, kSlLanes * NB / 2, lds);
    if (cap < std::min(gpl, groups) * p->sl.S)
        return fail(MC_ERR_UNSUPPORTED,
                    "sliced HMC: %lld workgroups must be co-resident, the device holds %lld of "
                    "this kernel", (long long)(std::min(gpl, groups) * p->sl.S), (long long)cap);
    A.fault = g_exchange_fault;
    ws_forget(ws);  // its tags restart at 1: the lane-resident kernel must clear again
    ws_mark_status(ws);
    for (int64_t g0 = 0; g0 < groups; g0 += gpl) {
        const int64_t ng = std::min(gpl, groups - g0);
        // the exchange tags restart at 1 in every launch: clear the granules
        // (and, first, the status word) ahead of it
        MC_HIP_TRY(hipMemsetAsync(g0 == 0 ? ws : (void*)xch, 0,
                                  g0 == 0 ? used : used - kSlStatusBytes, st));
        const int64_t grid = ng * p->sl.S;
        const hipError_t e = launch_exchange(k_hmc_sl<NB>, grid, kSlLanes * NB / 2, lds, st, ctx,
                                             A, g0 * NB, ng, (mc_chain_scalars*)b,
                                             (float*)(b + qo), (float*)(b + go), samples,
                                             trace_of(tr), xch, status);
        MC_HIP_TRY(e);
    }
    return MC_OK;
}

extern "C" int mc_workspace_status(const mc_program* p, const void* ws, int64_t bytes,
                                   void* stream) {
    if (!p) return fail(MC_ERR_INVALID, "program is NULL");
    if (!ws || !ws_has_status(ws)) return MC_OK;  // the last launch on ws had no exchange
    if (bytes < kSlStatusBytes) return fail(MC_ERR_INVALID, "bad workspace");
    int v = 0;
    MC_HIP_TRY(hipMemcpyAsync(&v, ws, sizeof(int), hipMemcpyDeviceToHost, (hipStream_t)stream));
    MC_HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    if (v != 0) {
        ws_forget(ws);  // the next launch clears the status word and the granules
        if (v == 2) {
            // the placement probe was wrong for this device: later launches in
            // this process use the agent-scope exchange (as MC_XCD_LOCAL=0);
            // the launch that failed skipped work and has to be redone
            g_xcd_local = 0;
            return fail(MC_ERR_UNSUPPORTED,
                        "sliced launch: an exchange group's workgroups were not on one XCD, which "
                        "its L2-resident records need (the device's workgroup placement differs "
                        "from its probe); the L2-resident exchange is now off in this process: "
                        "redo the launch from the chains' state before it");
        }
        return fail(MC_ERR_TIMEOUT, "sliced HMC: a cross-workgroup exchange timed out");
    }
    return MC_OK;
}

extern "C" int64_t mc_hmc_workspace_bytes(const mc_program* p, int64_t C) {
    if (!p || C < 0) return -1;
    // (a lanes1 program runs L = 0 configurations on the unsliced kernel, and
    // so does a sliced program with transformed operands, which the term
    // interpreter does not take: mc_hmc_run)
    const int64_t x = (lanes1(p) || sliced(p)) ? sl_workspace_bytes(p, C) : 0;
    if (sliced(p) && interp_ok(p)) return x;
    if (hmc_use_lds(p)) return x;
    return std::max(x, C * 5 * (int64_t)dpad_of(p->D) * 4);
}

template <int WPC, bool LDS, bool EX>
static int launch_hmc(const mc_program* p, const mc_run_config* cfg, void* state,
                      float* samples, const mc_trace* tr, float* ws, hipStream_t st) {
    int64_t qo, go;
    mc_state_offsets(p, cfg->num_chains, &qo, &go);
    char* b = (char*)state;
    RunArgs A;
    std::memset(&A, 0, sizeof(A));
    A.cfg = *cfg;
    A.dpad = dpad_of(p->D);
    A.lds_floats = (int32_t)hmc_lds_floats(p, LDS);
    A.scratch_floats = scratch_of(p);
    const size_t lds = (size_t)cpb_of(WPC) * A.lds_floats * 4;
    const int64_t grid = (cfg->num_chains + cpb_of(WPC) - 1) / cpb_of(WPC);
    if constexpr (EX) {  // the program's expression terms compiled (jit.hip)
        DevCtx ctx = ctx_of(p);
        mc_chain_scalars* scal = (mc_chain_scalars*)b;
        float *sq = (float*)(b + qo), *sg = (float*)(b + go);
        TraceDev td = trace_of(tr);
        void* args[] = {&ctx, &A, &scal, &sq, &sg, &samples, &td, &ws};
        bool used = false;
        const int rc = jit_launch(p, "mc::k_hmc<" + std::to_string(WPC) + ", " +
                                         (LDS ? "true" : "false") + ", true>",
                                  (unsigned)grid, block_of(WPC), lds, st, args, &used);
        if (rc != MC_OK || used) return rc;
    }
    MC_HIP_TRY(allow_lds(k_hmc<WPC, LDS, EX>, lds));
    hipLaunchKernelGGL((k_hmc<WPC, LDS, EX>), dim3((unsigned)grid), dim3(block_of(WPC)), lds, st,
                       ctx_of(p), A, (mc_chain_scalars*)b, (float*)(b + qo), (float*)(b + go),
                       samples, trace_of(tr), ws);
    MC_HIP_TRY(hipGetLastError());
    return MC_OK;
}

extern "C" int mc_hmc_run(const mc_program* p, const mc_run_config* cfg, void* state,
                          float* samples, const mc_trace* tr, void* ws, int64_t ws_bytes,
                          void* stream) {
    int rc = check_cfg(p, cfg, state);
    if (rc) return rc;
    if (cfg->num_leapfrog_steps < 0) return fail(MC_ERR_INVALID, "num_leapfrog_steps < 0");
    if (cfg->num_chains == 0 || cfg->iter_count == 0) return MC_OK;
    // L = 0 with transformed operands: the interpreter (k_hmc_sl) declines
    // them, so such a run takes the chain-per-workgroup tape (as lanes1 does)
    const bool sl_tape = sliced(p) && !use_lanes(p, cfg) && !interp_ok(p);
    if ((sliced(p) && !sl_tape) || (lanes1(p) && use_lanes(p, cfg))) {
        const int64_t need = sl_workspace_bytes(p, cfg->num_chains);
        if (ws == nullptr || ws_bytes < need)
            return fail(MC_ERR_INVALID, "workspace too small: need %lld bytes", (long long)need);
        if (device_cus() <= 0) return fail(MC_ERR_HIP, "no HIP device");
        int rc = kLanesNoJit;
        if (use_lanes(p, cfg)) {
            hipStream_t st = (hipStream_t)stream;
            switch (p->lr.rs) {  // (one translation unit per slot count: run_lanes_rs*.hip)
                case 1: rc = hmc_lanes_rs1(p, cfg, state, samples, tr, ws, st); break;
                case 2: rc = hmc_lanes_rs2(p, cfg, state, samples, tr, ws, st); break;
                default: rc = hmc_lanes_rs4(p, cfg, state, samples, tr, ws, st); break;
            }
            // an expression program without its JIT-compiled lane kernel (the
            // JIT off or failed): the tape below
            if (rc != kLanesNoJit) return rc;
        } else {
            return sl_nb_for(p, cfg->num_chains) == 16
                       ? launch_hmc_sl<16>(p, cfg, state, samples, tr, ws, (hipStream_t)stream)
                       : launch_hmc_sl<8>(p, cfg, state, samples, tr, ws, (hipStream_t)stream);
        }
    }
    ws_forget(ws);
    const bool lds = hmc_use_lds(p);
    const int64_t need = mc_hmc_workspace_bytes(p, cfg->num_chains);
    if (!lds && (ws == nullptr || ws_bytes < need))
        return fail(MC_ERR_INVALID, "workspace too small: need %lld bytes", (long long)need);
    hipStream_t st = (hipStream_t)stream;
    float* w = (float*)ws;
    return dispatch_tape(p, lds, [&](auto W, auto L, auto E) {
        return launch_hmc<decltype(W)::value, decltype(L)::value, decltype(E)::value>(
            p, cfg, state, samples, tr, w, st);
    });
}

#ifdef MC_STAMPS
MC_STAMPS_EXPORT(mc_debug_stamps, mc_debug_stamps_wg)
#endif
