// run_nuts_sl.hip — sliced NUTS, the compile-time hierarchical form
// (k_nuts_sl<..., FORM = LF_SW | LF_SWS | LF_DIR | LF_DM | LF_DS>: BASELINE
// configs[2]/[3]'s model, the README "Large" row) and its dispatch.
#include "run_nuts_sl.h"

int nuts_sl_hier(const mc_program* p, const mc_run_config* cfg, void* state, float* samples,
                 const mc_trace* tr, void* ws, hipStream_t st) {
    constexpr int HIER = LF_SW | LF_SWS | LF_DIR | LF_DM | LF_DS;
    constexpr int NSH = lf_nroles(HIER);
    const bool o4 = nuts_sl_occ(p) == 4;
    switch (p->lr.rs) {
        case 1: return o4 ? launch_nuts_sl<1, NSH, 4, HIER>(p, cfg, state, samples, tr, ws, st)
                          : launch_nuts_sl<1, NSH, 2, HIER>(p, cfg, state, samples, tr, ws, st);
        case 2: return o4 ? launch_nuts_sl<2, NSH, 4, HIER>(p, cfg, state, samples, tr, ws, st)
                          : launch_nuts_sl<2, NSH, 2, HIER>(p, cfg, state, samples, tr, ws, st);
        default: return launch_nuts_sl<4, NSH, 2, HIER>(p, cfg, state, samples, tr, ws, st);
    }
}

#ifdef MC_STAMPS
MC_STAMPS_EXPORT(mc_debug_stamps_nuts_sl, mc_debug_stamps_nuts_sl_wg)
#endif
