// run_nuts_sl_rt.hip — sliced NUTS, run-time form (k_nuts_sl<..., FORM = -1>):
// fast-form programs whose slices differ in their terms or share roles.
#include "run_nuts_sl.h"

int nuts_sl_rt(const mc_program* p, const mc_run_config* cfg, void* state, float* samples,
               const mc_trace* tr, void* ws, hipStream_t st) {
    const bool n4 = p->lr.Dsh > 3;
    if (!p->lr.fast) {  // expression terms (LanePlan::nuts_expr): the JIT-compiled form
        // (4 waves per SIMD with more than 8 slices, as the hierarchical form:
        // every chain block of 256 chains resident in one launch)
        const bool o4 = nuts_sl_occ(p) == 4;
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
