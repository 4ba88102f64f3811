// run_lanes_rs4.hip — lane-resident HMC launches with 4 register slots per lane.
#include "run_lanes.h"

int hmc_lanes_rs4(const mc_program* p, const mc_run_config* cfg, void* state, float* samples,
                  const mc_trace* tr, void* ws, hipStream_t st) {
    return hmc_lanes_dispatch<4>(p, cfg, state, samples, tr, ws, st);
}

#ifdef MC_STAMPS
#if 4 == 1
MC_STAMPS_EXPORT(mc_debug_stamps_lanes, mc_debug_stamps_lanes_wg)
#endif
#endif
