// run_nuts_sl_rt.hip — sliced NUTS, run-time form (k_nuts_sl<..., FORM = -1>):
// fast-form programs whose slices differ in their terms or share roles.
#include "run_nuts_sl.h"

int nuts_sl_rt(const mc_program* p, const mc_run_config* cfg, void* state, float* samples,
               const mc_trace* tr, void* ws, hipStream_t st) {
    const bool n4 = p->lr.Dsh > 3;
    if (!p->lr.fast) {  // expression terms (LanePlan::nuts_expr): the JIT-compiled form
        // (2 waves per SIMD: at 16 slices 4 — every chain block of 256 chains
        // resident in one launch — measured no faster on the N = 100 K GLMs,
        // logistic 4.30 vs 4.25 M leaf-steps/s, two-predictor 8.97 vs 8.18;
        // MC_NUTS_SL_OCC=4 selects it)
        const char* oe = std::getenv("MC_NUTS_SL_OCC");
        const bool o4 = oe && std::atoi(oe) == 4;
#define MC_NSLJ(R)                                                                              \
        return o4 ? (n4 ? launch_nuts_sl_jit<R, 4, 4>(p, cfg, state, samples, tr, ws, st)       \
                        : launch_nuts_sl_jit<R, 3, 4>(p, cfg, state, samples, tr, ws, st))      \
                  : (n4 ? launch_nuts_sl_jit<R, 4, 2>(p, cfg, state, samples, tr, ws, st)       \
                        : launch_nuts_sl_jit<R, 3, 2>(p, cfg, state, samples, tr, ws, st))
        switch (p->lr.rs) {
            case 1: MC_NSLJ(1);
            case 2: MC_NSLJ(2);
            default: MC_NSLJ(4);
        }
#undef MC_NSLJ
    }
    switch (p->lr.rs) {
        case 1: return n4 ? launch_nuts_sl<1, 4, 2, -1>(p, cfg, state, samples, tr, ws, st)
                          : launch_nuts_sl<1, 3, 2, -1>(p, cfg, state, samples, tr, ws, st);
        case 2: return n4 ? launch_nuts_sl<2, 4, 2, -1>(p, cfg, state, samples, tr, ws, st)
                          : launch_nuts_sl<2, 3, 2, -1>(p, cfg, state, samples, tr, ws, st);
        default: return n4 ? launch_nuts_sl<4, 4, 2, -1>(p, cfg, state, samples, tr, ws, st)
                           : launch_nuts_sl<4, 3, 2, -1>(p, cfg, state, samples, tr, ws, st);
    }
}
