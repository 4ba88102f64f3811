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
//   normal pair:            Box-Muller in f32 from IEEE operations only
//                           (mc_box_muller below): bit-identical on host,
//                           device and in the NumPy oracle;
//   log of an accept / slice uniform: mc_logf_unit (the same f32 log).
// Other f32 log / exp values that feed a decision (dual averaging) are
// evaluated in double and rounded once (mc_logf_ref / mc_expf_ref): GPU and
// oracle agree except when a double result lies within ~1 ulp(f64) of an f32
// rounding boundary (probability ~1e-8 per value).
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

// Box-Muller in single precision from IEEE operations only (+, -, *, /,
// correctly rounded sqrt; built with -ffp-contract=off), so that host, device
// and the NumPy oracle (oracle/philox.py: the same operations in float32)
// produce the same bits:
//   u = (float(w) + 0.5) 2^-32  (w rounded to f32 once, then exact steps);
//   mc_logf_unit(u), u in (0, 1]: FreeBSD msun e_logf.c's reduction and
//     minimax polynomial (k ln2 + log(1 + f), f in [sqrt(2)/2 - 1, sqrt(2) - 1));
//   mc_sincospif_unit(x), x in [0, 2]: quadrant n = rint(2x), r = x - n/2
//     (exact), Taylor polynomials of sin / cos on pi r, |pi r| <= pi/4.
// Each normal is within a few ulp(f32) of the exact transform of its
// uniforms (tests/test_golden.py).  A double-precision transform costs ~3x
// the VALU: 3.6 % of the bench kernel's time on MI355X (three normals per
// lane and iteration, profiles/r3/ab).
MC_HD float mc_logf_unit(float x) {
    const float ln2_hi = 0x1.62e300p-1f, ln2_lo = 0x1.2fefa2p-17f;  // (exact f32 values)
    const float Lg1 = 0x1.555554p-1f, Lg2 = 0x1.999c26p-2f, Lg3 = 0x1.23d3dcp-2f,
                Lg4 = 0x1.f13c4cp-3f;
    int k;
    float m = frexpf(x, &k);                 // x = m 2^k, m in [0.5, 1)
    if (m < 0x1.6a09e6p-1f) {               // m in [sqrt(2)/2, sqrt(2))
        m = m * 2.0f;
        k -= 1;
    }
    const float f = m - 1.0f;                // exact
    const float s = f / (2.0f + f);
    const float dk = (float)k;
    const float z = s * s, w = z * z;
    const float t1 = w * (Lg2 + w * Lg4);
    const float t2 = z * (Lg1 + w * Lg3);
    const float R = t2 + t1;
    const float hfsq = 0.5f * f * f;
    return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
}
MC_HD void mc_sincospif_unit(float x, float* sp, float* cp) {
    const float S1 = -0x1.555556p-3f, S2 = 0x1.111112p-7f, S3 = -0x1.a01a02p-13f,
                S4 = 0x1.71de3ap-19f;  // f32(-1/3!), f32(1/5!), ...
    const float C1 = 0x1.555556p-5f, C2 = -0x1.6c16c2p-10f, C3 = 0x1.a01a02p-16f,
                C4 = -0x1.27e4fcp-22f;  // f32(1/4!), f32(-1/6!), ...
    const float n = rintf(2.0f * x);         // quadrant 0..4
    const float r = x - 0.5f * n;            // exact, |r| <= 1/4
    const float t = r * 0x1.921fb6p+1f;     // f32(pi)
    const float z = t * t;
    const float sn = t + (t * z) * (S1 + z * (S2 + z * (S3 + z * S4)));
    const float cs = (1.0f - 0.5f * z) + (z * z) * (C1 + z * (C2 + z * (C3 + z * C4)));
    const int q = ((int)n) & 3;
    *sp = q == 0 ? sn : (q == 1 ? cs : (q == 2 ? -sn : -cs));
    *cp = q == 0 ? cs : (q == 1 ? -sn : (q == 2 ? -cs : sn));
}
MC_HD float mc_u01_boxf(uint32_t w) { return ((float)w + 0.5f) * 0x1p-32f; }

// The normal pair of two Philox words.
MC_HD void mc_box_muller(uint32_t a, uint32_t b, float* z0, float* z1) {
    const float u1 = mc_u01_boxf(a);
    const float u2 = mc_u01_boxf(b);
    const float r = sqrtf(-2.0f * mc_logf_unit(u1));
    float s, c;
    mc_sincospif_unit(2.0f * u2, &s, &c);
    *z0 = r * c;
    *z1 = r * s;
}

// The same pair from the precomputed log of the first uniform (l1 =
// mc_logf_unit(mc_u01_boxf(a))) and the second word: bit-identical to
// mc_box_muller(a, b) (k_hmc_lf's lane RNG plan computes the log once and
// shares it with an accept draw).
MC_HD void mc_box_muller_log(float l1, uint32_t b, float* z0, float* z1) {
    const float u2 = mc_u01_boxf(b);
    const float r = sqrtf(-2.0f * l1);
    float s, c;
    mc_sincospif_unit(2.0f * u2, &s, &c);
    *z0 = r * c;
    *z1 = r * s;
}

// f32 log / exp "as IEEE would round them": evaluated in double, rounded once.
MC_HD float mc_logf_ref(float x) { return (float)log((double)x); }
// The log of an accept / slice uniform in (0, 1]: mc_logf_unit.
MC_HD float mc_logf_u01(float u) { return mc_logf_unit(u); }
MC_HD float mc_expf_ref(float x) { return (float)exp((double)x); }
