// Microbenchmark: cycles per wave of one Philox4x32-10 draw and of one
// Box-Muller pair (csrc/philox.h), one wave per SIMD (s_memtime).
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../mlx-mcmc_amd/csrc/philox.h"

template <int MODE>
__global__ void __launch_bounds__(256) k(float* out, int iters, long long* cyc) {
    uint32_t acc = threadIdx.x;
    float facc = 0.0f;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        if (MODE == 0) {  // one Philox block per lane
            const mc_u32x4 r = mc_draw(12345ull, threadIdx.x, i, 3, 0, acc & 7);
            acc ^= r.x ^ r.y ^ r.z ^ r.w;
        } else if (MODE == 1) {  // one Box-Muller pair per lane
            float z0, z1;
            mc_box_muller(acc * 2654435761u + i, acc ^ (uint32_t)i, &z0, &z1);
            facc += z0 + z1;
            acc += __float_as_uint(z0);
        } else {  // one f32 log of a uniform
            const float l = mc_logf_u01(mc_u01_f32(acc + i));
            facc += l;
            acc += __float_as_uint(l);
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = facc + (float)acc;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE>
void run(const char* name, float* d, long long* c) {
    const int iters = 2048;
    hipLaunchKernelGGL(k<MODE>, dim3(256), dim3(256), 0, 0, d, iters, c);
    hipDeviceSynchronize();
    hipLaunchKernelGGL(k<MODE>, dim3(256), dim3(256), 0, 0, d, iters, c);
    hipDeviceSynchronize();
    long long h[1];
    hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost);
    printf("%-28s %.1f cycles per wave-call (memtime, one wave per SIMD)\n", name,
           (double)h[0] / iters);
}

int main() {
    float* d;
    long long* c;
    hipMalloc(&d, 1 << 24);
    hipMemset(d, 0, 1 << 24);
    hipMalloc(&c, 8 * 4096);
    run<0>("philox4x32-10 block", d, c);
    run<1>("box-muller pair (IEEE f32)", d, c);
    run<2>("logf of a uniform (IEEE)", d, c);
    return 0;
}
