// Microbenchmark: issue throughput of packed vs scalar FP32 VALU on gfx950,
// and the dependent-chain latency of each (cycles per wave-instruction per
// SIMD, from s_memtime; one and two waves per SIMD).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ void __launch_bounds__(256) k(float* out, int iters, long long* cyc) {
    float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
          a6 = a0 + 6, a7 = a0 + 7;
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7};
    const float x = out[threadIdx.x] + 1.0f;
    const f2 xx = {x, x};
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            if (MODE == 0) {  // 8 independent scalar adds
                a0 += x; a1 += x; a2 += x; a3 += x; a4 += x; a5 += x; a6 += x; a7 += x;
            } else if (MODE == 1) {  // 4 independent packed adds (= 8 lane-ops)
                p0 += xx; p1 += xx; p2 += xx; p3 += xx;
            } else if (MODE == 2) {  // 1 dependent scalar chain
                a0 += x;
            } else if (MODE == 3) {  // 1 dependent packed chain
                p0 += xx;
            } else if (MODE == 4) {  // 4 independent packed fma
                p0 = __builtin_elementwise_fma(xx, xx, p0);
                p1 = __builtin_elementwise_fma(xx, xx, p1);
                p2 = __builtin_elementwise_fma(xx, xx, p2);
                p3 = __builtin_elementwise_fma(xx, xx, p3);
            } else if (MODE == 5) {  // 8 independent scalar fma
                a0 = fmaf(x, x, a0); a1 = fmaf(x, x, a1); a2 = fmaf(x, x, a2); a3 = fmaf(x, x, a3);
                a4 = fmaf(x, x, a4); a5 = fmaf(x, x, a5); a6 = fmaf(x, x, a6); a7 = fmaf(x, x, a7);
            }
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] =
        a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + p0.x + p0.y + p1.x + p1.y + p2.x + p2.y + p3.x + p3.y;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE>
void run(const char* name, int wpsimd, float* d, long long* c, int ninstr_per_u) {
    const int iters = 4096;
    // one workgroup per CU: 4 waves (1 per SIMD) or 8 (2 per SIMD)
    int threads = 64 * 4 * wpsimd;
    hipLaunchKernelGGL(k<MODE>, dim3(256), dim3(threads > 256 ? 256 : threads), 0, 0, d, iters, c);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    // wpsimd = 2: two workgroups of 256 per CU (grid 512)
    hipLaunchKernelGGL(k<MODE>, dim3(256 * wpsimd), dim3(256), 0, 0, d, iters, c);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    long long h[1]; hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost);
    double per = (double)h[0] / (iters * 16.0 * ninstr_per_u);
    printf("%-28s waves/SIMD %d: %.2f cycles per wave-instruction (memtime), %.3f ms\n", name, wpsimd, per, ms);
}

int main() {
    float* d; long long* c;
    hipMalloc(&d, 1 << 24); hipMemset(d, 0, 1 << 24);
    hipMalloc(&c, 8 * 4096);
    for (int w = 1; w <= 2; ++w) {
        run<0>("scalar add x8 indep", w, d, c, 8);
        run<1>("packed add x4 indep", w, d, c, 4);
        run<5>("scalar fma x8 indep", w, d, c, 8);
        run<4>("packed fma x4 indep", w, d, c, 4);
        run<2>("scalar add dep chain", w, d, c, 1);
        run<3>("packed add dep chain", w, d, c, 1);
    }
    return 0;
}
