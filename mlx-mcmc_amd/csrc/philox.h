// philox.h — counter-based RNG shared by host and device code.
//
// Replaces the reference's keyed MLX RNG (mx.random.key / split / normal /
// uniform at mlx_mcmc/kernels/hmc.py:116-118,145-146 and nuts.py:182,204-205,
// 223-225,234-235,253-254,271).  MLX's own stream cannot be reproduced (its
// source is not available here), so the engine defines its draws as a pure
// function of (seed, global chain id, iteration, tag, index):
//
//   Philox4x32-10 (Salmon, Moraes, Dror, Shaw, "Parallel random numbers: as
//   easy as 1, 2, 3", SC'11), key = (seed lo32, seed hi32),
//   counter = (chain, iteration, tag << 24 | sub, index).
//
// Transforms (identical in oracle/philox.py):
//   uniform f32 in (0,1):   ((w >> 9) + 0.5) * 2^-23          (exact in f32)
//   uniform f64 in (0,1):   (w + 0.5) * 2^-32                  (exact in f64)
//   normal pair:            double Box-Muller on two f64 uniforms, each
//                           result rounded once to f32 (device: sincospi).
// Doing Box-Muller and every log/exp that feeds a decision in double and
// rounding once makes the GPU and the CPU oracle agree bit-for-bit except when
// a double result lies within ~1 ulp(f64) of an f32 rounding boundary
// (probability ~1e-8 per value).
#pragma once
#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__)
#define MC_HD __host__ __device__ inline
#else
#define MC_HD inline
#endif

struct mc_u32x4 {
    uint32_t x, y, z, w;
};

MC_HD mc_u32x4 mc_philox4x32_10(mc_u32x4 c, uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)M0 * c.x;
        const uint64_t p1 = (uint64_t)M1 * c.z;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        mc_u32x4 n;
        n.x = hi1 ^ c.y ^ k0;
        n.y = lo1;
        n.z = hi0 ^ c.w ^ k1;
        n.w = lo0;
        c = n;
        k0 += W0;
        k1 += W1;
    }
    return c;
}

MC_HD mc_u32x4 mc_draw(uint64_t seed, uint32_t chain, uint32_t iter, uint32_t tag,
                       uint32_t sub, uint32_t index) {
    mc_u32x4 c;
    c.x = chain;
    c.y = iter;
    c.z = (tag << 24) | (sub & 0x00FFFFFFu);
    c.w = index;
    return mc_philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
}

MC_HD float mc_u01_f32(uint32_t w) {
    return ((float)(w >> 9) + 0.5f) * 1.1920928955078125e-07f;  // 2^-23
}

MC_HD double mc_u01_f64(uint32_t w) {
    return ((double)w + 0.5) * 2.3283064365386962890625e-10;  // 2^-32
}

// Device only.  cos / sin of 2 pi u2 through sincospi(2 u2) (2 u2 is exact):
// one call, no Payne-Hanek reduction; the f64 values agree with the oracle's
// numpy cos / sin(2 pi u2) to ~1 ulp(f64), so the f32 results are identical
// except within ~1 ulp(f64) of an f32 rounding boundary.
__device__ inline void mc_box_muller(uint32_t a, uint32_t b, float* z0, float* z1) {
    const double u1 = mc_u01_f64(a);
    const double u2 = mc_u01_f64(b);
    const double r = sqrt(-2.0 * log(u1));
    double s, c;
    sincospi(2.0 * u2, &s, &c);
    *z0 = (float)(r * c);
    *z1 = (float)(r * s);
}

// f32 log / exp "as IEEE would round them": evaluated in double, rounded once.
MC_HD float mc_logf_ref(float x) { return (float)log((double)x); }
MC_HD float mc_expf_ref(float x) { return (float)exp((double)x); }
