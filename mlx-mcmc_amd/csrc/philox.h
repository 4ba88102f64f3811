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

// Box-Muller's double log and sincospi, restricted to the arguments the
// uniforms produce (the device math library's general versions handle every
// special case and cost ~90 / ~60 VALU; these ~40 each, and the samplers draw
// 3 normals and 2 accept logs per lane and iteration):
//   mc_log_unit(x), x in [2^-40, 1]: fdlibm's e_log.c reduction and minimax
//     polynomial (k ln2 + log(1 + f), f in [sqrt(2)/2 - 1, sqrt(2) - 1),
//     < 1 ulp);
//   mc_sincospi_unit(x), x in [0, 2): sin / cos(pi x) from the quadrant
//     n = rint(2x) (exact: x has <= 33 significant bits) and fdlibm's
//     __kernel_sin / __kernel_cos on pi (x - n / 2), |.| <= pi / 4 (< 1 ulp).
// Both use only IEEE +, -, *, / (built with -ffp-contract=off: no FMA), so
// host and device agree bit for bit; tests/test_golden.py checks them
// against libm.
MC_HD double mc_log_unit(double x) {
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
                 Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
                 Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                 Lg7 = 1.479819860511658591e-01;
    int k;
    double m = frexp(x, &k);                 // x = m 2^k, m in [0.5, 1)
    if (m < 0.70710678118654752440) {        // m in [sqrt(2)/2, sqrt(2))
        m = m * 2.0;
        k -= 1;
    }
    const double f = m - 1.0;                // exact
    const double s = f / (2.0 + f);
    const double dk = (double)k;
    const double z = s * s, w = z * z;
    const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    const double R = t2 + t1;
    const double hfsq = 0.5 * f * f;
    return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
}
MC_HD void mc_sincospi_unit(double x, double* sp, double* cp) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const double n = rint(2.0 * x);          // quadrant 0..4
    const double r = x - 0.5 * n;            // exact, |r| <= 1/4
    const double t = r * 3.14159265358979311600e+00;
    const double z = t * t;
    const double v = z * t;
    const double sr = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    const double sn = t + v * (S1 + z * sr);
    const double cr = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    const double hz = 0.5 * z;
    const double w = 1.0 - hz;
    const double cs = w + (((1.0 - w) - hz) + z * cr);
    const int q = ((int)n) & 3;
    *sp = q == 0 ? sn : (q == 1 ? cs : (q == 2 ? -sn : -cs));
    *cp = q == 0 ? cs : (q == 1 ? -sn : (q == 2 ? -cs : sn));
}

// Device only.  cos / sin of 2 pi u2 through sincospi(2 u2) (2 u2 is exact):
// one call, no Payne-Hanek reduction; the f64 values agree with the oracle's
// numpy cos / sin(2 pi u2) to ~1 ulp(f64), so the f32 results are identical
// except within ~1 ulp(f64) of an f32 rounding boundary.
MC_HD void mc_box_muller(uint32_t a, uint32_t b, float* z0, float* z1) {
    const double u1 = mc_u01_f64(a);
    const double u2 = mc_u01_f64(b);
    const double r = sqrt(-2.0 * mc_log_unit(u1));
    double s, c;
    mc_sincospi_unit(2.0 * u2, &s, &c);
    *z0 = (float)(r * c);
    *z1 = (float)(r * s);
}

// f32 log / exp "as IEEE would round them": evaluated in double, rounded once.
MC_HD float mc_logf_ref(float x) { return (float)log((double)x); }
// The same for a uniform in (0, 1] (accept / slice draws): mc_log_unit.
MC_HD float mc_logf_u01(float u) { return (float)mc_log_unit((double)u); }
MC_HD float mc_expf_ref(float x) { return (float)exp((double)x); }
