// diag.h — device-side sample diagnostics.
//
// Sample buffers are [C, S, D] f32 (chain, draw, flattened element), the
// layout mc_hmc_run / mc_nuts_run write.  A *series* is x[c, :, d].
//
//   k_series_stats   one thread per series: the reference ESS rule
//                    (examples/06_nuts_comparison.py:22-41) plus the moments
//                    split R-hat and MCMC.summary need.  HBM-bound: pass 1
//                    reads the series once (mean, half means); pass 2 reads it
//                    once per block of 8 lags (lag 0 = variance), normally one
//                    block because the reference stops at the first rho < 0.05.
//                    Consecutive threads take consecutive d of one chain, so
//                    every draw s is one coalesced row read.
//   k_stats_reduce   one thread per element: sums over chains in chain order
//                    (deterministic, no atomics).  Two modes so that the R-hat
//                    spread is computed about the *global* grand mean: mode 0
//                    sums the half-chain means (and ESS), the caller all-reduces
//                    that [2, D] block over ranks, mode 1 sums squared
//                    deviations from it and the half-chain variances.
//   k_rhat           split R-hat (Gelman et al., BDA3 eq. 11.4) from the two
//                    reduced rows.
//   k_pool_moments   one workgroup per parameter: pooled mean / std (ddof 0)
//                    of every value of a parameter over all chains and draws
//                    (mcmc.py:205-206) from the per-series moments (Chan's
//                    combination, fixed-order tree).
//   k_sel_hist/pick  exact order statistics of a parameter's pooled values
//                    (median / percentiles, mcmc.py:207-209): MSB-first radix
//                    select on order-preserving u32 keys, 4 passes of 8 bits,
//                    per-block LDS histograms merged with u64 atomics (counts are
//                    order-independent, so the result is deterministic).
#pragma once

enum { ST_ESS = 0, ST_MEAN, ST_M2, ST_HMEAN0, ST_HMEAN1, ST_HM2_0, ST_HM2_1, ST_COUNT };

constexpr int kLagBlock = 8;
constexpr int kSelMaxTargets = 8;

__global__ __launch_bounds__(256) void k_series_stats(const float* __restrict__ x, int64_t C,
                                                      int64_t S, int64_t D, int32_t lmax,
                                                      double* __restrict__ st) {
    const int64_t nser = C * D;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nser) return;
    const int64_t c = t / D, d = t - c * D;
    const float* __restrict__ p = x + c * S * D + d;
    const int64_t h = S / 2;

    // pass 1: means (examples/06:25 np.mean), half-chain means
    double s_all = 0.0, s0 = 0.0, s1 = 0.0;
#pragma unroll 4
    for (int64_t s = 0; s < S; ++s) {
        const double v = (double)p[s * D];
        s_all += v;
        if (s < h) s0 += v;
        if (s >= S - h) s1 += v;
    }
    const double mean = s_all / (double)S;
    const double m0 = h > 0 ? s0 / (double)h : 0.0;
    const double m1 = h > 0 ? s1 / (double)h : 0.0;

    // pass 2: autocovariance sums, kLagBlock lags per read of the series.
    // acc[j] = sum_{s < S-lag} (x_s - mean)(x_{s+lag} - mean), lag = l0 + j;
    // the ring w holds x_{s+l0+j} - mean (0 past the end: adds exact zeros).
    double m2 = 0.0, hm0 = 0.0, hm1 = 0.0, var = 0.0, acf_sum = 0.0;
    bool done = false;
    for (int64_t l0 = 0; !done; l0 += kLagBlock) {
        double acc[kLagBlock], w[kLagBlock];
#pragma unroll
        for (int j = 0; j < kLagBlock; ++j) {
            acc[j] = 0.0;
            w[j] = (l0 + j < S) ? (double)p[(l0 + j) * D] - mean : 0.0;
        }
        for (int64_t s = 0; s + l0 < S; ++s) {
            const double raw = (double)p[s * D];
            const double v = raw - mean;
#pragma unroll
            for (int j = 0; j < kLagBlock; ++j) acc[j] += v * w[j];
            if (l0 == 0) {
                if (s < h) { const double e = raw - m0; hm0 += e * e; }
                if (s >= S - h) { const double e = raw - m1; hm1 += e * e; }
            }
#pragma unroll
            for (int j = 0; j + 1 < kLagBlock; ++j) w[j] = w[j + 1];
            const int64_t nx = s + l0 + kLagBlock;
            w[kLagBlock - 1] = nx < S ? (double)p[nx * D] - mean : 0.0;
        }
        // the reference's loop (examples/06:31-36) over this block's lags
        for (int j = 0; j < kLagBlock && !done; ++j) {
            const int64_t lag = l0 + j;
            if (lag == 0) {
                m2 = acc[0];
                var = acc[0] / (double)S;                       // np.var, ddof 0
                if (var == 0.0) done = true;                    // examples/06:28-29
                continue;
            }
            if (lag >= lmax) { done = true; break; }
            const double cr = (acc[j] / (double)(S - lag)) / var;
            acf_sum += cr;
            if (cr < 0.05) done = true;
        }
        if (l0 + kLagBlock >= lmax) done = true;          // every lag < lmax was in this block
    }
    const double ess = var == 0.0 ? (double)S : (double)S / (1.0 + 2.0 * acf_sum);
    st[ST_ESS * nser + t] = ess;
    st[ST_MEAN * nser + t] = mean;
    st[ST_M2 * nser + t] = m2;
    st[ST_HMEAN0 * nser + t] = m0;
    st[ST_HMEAN1 * nser + t] = m1;
    st[ST_HM2_0 * nser + t] = hm0;
    st[ST_HM2_1 * nser + t] = hm1;
}

// mode 0: out[0][d] = sum_c (hmean0 + hmean1), out[1][d] = sum_c ess
// mode 1: out[0][d] = sum_c (hmean_h - g)^2 with g = center[d] / m_total,
//         out[1][d] = sum_c (hm2_0 + hm2_1) / (h - 1)
__global__ __launch_bounds__(256) void k_stats_reduce(const double* __restrict__ st, int64_t C,
                                                      int64_t S, int64_t D, int32_t mode,
                                                      const double* __restrict__ center,
                                                      int64_t m_total, double* __restrict__ out) {
    const int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= D) return;
    const int64_t nser = C * D;
    double a = 0.0, b = 0.0;
    if (mode == 0) {
        for (int64_t c = 0; c < C; ++c) {
            const int64_t t = c * D + d;
            a += st[ST_HMEAN0 * nser + t];
            a += st[ST_HMEAN1 * nser + t];
            b += st[ST_ESS * nser + t];
        }
    } else {
        const double g = center[d] / (double)m_total;
        const double hm1 = (double)(S / 2) - 1.0;
        for (int64_t c = 0; c < C; ++c) {
            const int64_t t = c * D + d;
            const double e0 = st[ST_HMEAN0 * nser + t] - g, e1 = st[ST_HMEAN1 * nser + t] - g;
            a += e0 * e0;
            a += e1 * e1;
            b += st[ST_HM2_0 * nser + t] / hm1;
            b += st[ST_HM2_1 * nser + t] / hm1;
        }
    }
    out[d] = a;
    out[D + d] = b;
}

// BDA3 11.4 on m half-chains of n draws: W = mean within variance,
// B/n = spread / (m - 1), var+ = (n-1)/n W + B/n, R = sqrt(var+ / W).
__global__ __launch_bounds__(256) void k_rhat(const double* __restrict__ spread, int64_t D,
                                              int64_t m, int64_t n, double* __restrict__ rhat) {
    const int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= D) return;
    const double W = spread[D + d] / (double)m;
    const double Bn = spread[d] / (double)(m - 1);
    const double vp = ((double)(n - 1) / (double)n) * W + Bn;
    rhat[d] = sqrt(vp / W);
}

__device__ inline double block_sum256(double v, double* sh) {
    sh[threadIdx.x] = v;
    __syncthreads();
#pragma unroll
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
        __syncthreads();
    }
    const double r = sh[0];
    __syncthreads();
    return r;
}

// Pooled mean / std over C * S * len values from the per-series moments:
// M = sum mean_cd / (C len); M2 = sum [m2_cd + S (mean_cd - M)^2].
__global__ __launch_bounds__(256) void k_pool_moments(const double* __restrict__ st, int64_t C,
                                                      int64_t S, int64_t D, int64_t off,
                                                      int64_t len, double* __restrict__ out) {
    __shared__ double sh[256];
    const int64_t nser = C * D, n = C * len;
    double a = 0.0;
    for (int64_t i = threadIdx.x; i < n; i += 256) {
        const int64_t c = i / len, e = i - c * len;
        a += st[ST_MEAN * nser + c * D + off + e];
    }
    const double M = block_sum256(a, sh) / (double)n;
    double b = 0.0;
    for (int64_t i = threadIdx.x; i < n; i += 256) {
        const int64_t c = i / len, e = i - c * len;
        const int64_t t = c * D + off + e;
        const double dm = st[ST_MEAN * nser + t] - M;
        b += st[ST_M2 * nser + t] + (double)S * (dm * dm);
    }
    const double M2 = block_sum256(b, sh);
    if (threadIdx.x == 0) {
        out[0] = M;
        out[1] = sqrt(M2 / ((double)n * (double)S));
    }
}

// ---------------------------------------------------------------- select --
struct SelTargets {
    int64_t k[kSelMaxTargets];
    int32_t nk;
};

struct SelState {                 // per target, in the workspace
    uint32_t prefix;
    uint32_t pad;
    int64_t rank;                 // remaining rank within the current prefix
};

__device__ __forceinline__ uint32_t f32_key(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key_f32(uint32_t k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// workspace: [SelState x nk][u64 hist nk x 256][u32 nan flag]
__global__ void k_sel_init(SelTargets tg, SelState* __restrict__ stt,
                           unsigned long long* __restrict__ hist, uint32_t* __restrict__ nanf) {
    const int i = threadIdx.x;
    if (i < tg.nk) { stt[i].prefix = 0; stt[i].pad = 0; stt[i].rank = tg.k[i]; }
    for (int j = i; j < tg.nk * 256; j += blockDim.x) hist[j] = 0ull;
    if (i == 0) *nanf = 0u;
}

__global__ __launch_bounds__(256) void k_sel_hist(const float* __restrict__ x, int64_t rows,
                                                  int64_t D, int64_t off, int64_t len, int32_t nk,
                                                  int32_t shift, const SelState* __restrict__ stt,
                                                  unsigned long long* __restrict__ hist,
                                                  uint32_t* __restrict__ nanf) {
    __shared__ uint32_t lh[kSelMaxTargets * 256];
    __shared__ uint32_t pre[kSelMaxTargets];
    for (int j = threadIdx.x; j < nk * 256; j += 256) lh[j] = 0u;
    if ((int)threadIdx.x < nk) pre[threadIdx.x] = stt[threadIdx.x].prefix;
    __syncthreads();
    const int64_t n = rows * len;
    const uint32_t hi_mask = shift >= 24 ? 0u : (0xffffffffu << (shift + 8));
    bool saw_nan = false;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * 256) {
        const int64_t r = i / len, e = i - r * len;
        const float f = x[r * D + off + e];
        saw_nan |= (f != f);
        const uint32_t k = f32_key(f);
        const uint32_t dig = (k >> shift) & 255u;
        for (int t = 0; t < nk; ++t)
            if (((k ^ pre[t]) & hi_mask) == 0u) atomicAdd(&lh[t * 256 + dig], 1u);
    }
    if (saw_nan) atomicOr(nanf, 1u);
    __syncthreads();
    for (int j = threadIdx.x; j < nk * 256; j += 256)
        if (lh[j]) atomicAdd(&hist[j], (unsigned long long)lh[j]);
}

// One wave per target: find the digit whose cumulative count covers rank,
// extend the prefix, clear the histogram for the next pass; after the last
// pass write the value (NaN if the pool holds a NaN, like np.percentile).
__global__ void k_sel_pick(int32_t nk, int32_t shift, SelState* __restrict__ stt,
                           unsigned long long* __restrict__ hist,
                           const uint32_t* __restrict__ nanf, float* __restrict__ out) {
    const int t = threadIdx.x;
    if (t >= nk) return;
    unsigned long long* hh = hist + t * 256;
    int64_t rank = stt[t].rank;
    uint32_t dig = 255u;
    unsigned long long cum = 0ull;
    for (int b = 0; b < 256; ++b) {
        const unsigned long long c = hh[b];
        if ((unsigned long long)rank < cum + c) { dig = (uint32_t)b; break; }
        cum += c;
    }
    for (int b = 0; b < 256; ++b) hh[b] = 0ull;
    stt[t].rank = rank - (int64_t)cum;
    stt[t].prefix |= dig << shift;
    if (shift == 0 && out) out[t] = *nanf ? __uint_as_float(0x7fc00000u) : key_f32(stt[t].prefix);
}
