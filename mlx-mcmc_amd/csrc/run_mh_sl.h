// run_mh_sl.h — the sliced Metropolis-Hastings kernel's host side (k_mh_sl,
// mh_sliced.h): eligibility, workspace, dispatch (run_mh_sl.hip).
#pragma once
#include "run_nuts_sl.h"
#include "mh_sliced.h"

// exchange lines (both parities) for every chain block of C chains
inline int64_t mh_sl_line_bytes(const mc_program* p, int64_t C) {
    const int64_t groups = (C + kNslWaves - 1) / kNslWaves;
    return 2 * groups * kNslWaves * (int64_t)p->lr.S * kMslLine * 8;
}
// Sliced fast-form programs run k_mh_sl unless MC_MH_SLICED=0 in the
// environment or mc_debug_mh_sliced(0) (A/B and tests: k_mh on the tape),
// or the slice kernel is forced to the interpreter.
inline int g_mh_sliced = -1;
inline bool mh_sliced_enabled() {
    if (g_mh_sliced < 0) {
        const char* e = std::getenv("MC_MH_SLICED");
        g_mh_sliced = (e && e[0] == '0') ? 0 : 1;
    }
    return g_mh_sliced == 1;
}
// (a program with expression terms, LanePlan::nuts_expr: the JIT-compiled
// run-time form, not while the JIT is off or after its compilation failed)
inline bool use_mh_sliced(const mc_program* p) {
    const bool expr = p->lr.nuts_expr && jit_enabled() && jit_error(p).empty();
    return mh_sliced_enabled() && p->sl.S >= 2 && p->lr.ok && (p->lr.fast || expr) &&
           lanes_fast_enabled() &&
           p->lr.S >= 2 && p->lr.S <= kLrSlices && p->slice_kernel != 1 &&
           (size_t)p->lr.sdata_floats * 4 + p->lr.sterms.size() * sizeof(LrSterm) <=
               (size_t)kSlLdsBudget;
}
inline int64_t mh_sl_workspace_bytes(const mc_program* p, int64_t C) {
    return kSlStatusBytes + mh_sl_line_bytes(p, C);
}
int mh_sliced_run(const mc_program* p, const mc_run_config* cfg, float scale, void* state,
                  float* samples, const mc_trace* tr, void* ws, hipStream_t st);
