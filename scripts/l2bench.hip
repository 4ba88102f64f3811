// l2bench.hip — how fast can 256 workgroups each stream the SAME ~432 KB
// (L2-resident) array?  Variants: lockstep start, rotated start per block,
// distinct arrays per block.  Build: hipcc -O3 --offload-arch=gfx950 l2bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void __launch_bounds__(512) stream(const float4* __restrict__ buf, int n4, int reps,
                                             int mode, float* out) {
    const int tid = threadIdx.x;
    float acc = 0.f;
    const int nb = n4 / 512;  // float4 rows of 512 per block-sweep
    const int rot = (mode == 1) ? (blockIdx.x * 7) % nb : 0;
    const float4* b = (mode == 2) ? buf + (size_t)blockIdx.x * n4 : buf;
    for (int r = 0; r < reps; ++r) {
        for (int i0 = 0; i0 < nb; i0 += 8) {
            float4 x[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                int i = i0 + k;
                if (i < nb) {
                    int j = i + rot;
                    if (j >= nb) j -= nb;
                    x[k] = b[(size_t)j * 512 + tid];
                } else {
                    x[k] = make_float4(0, 0, 0, 0);
                }
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) acc += x[k].x + x[k].y + x[k].z + x[k].w;
        }
    }
    if (acc == 12345.f) out[0] = acc;
}

int main() {
    const int n4 = 108 * 1024 / 4 * 4;  // ~432 KB of float4 (multiple of 512)
    const int n4r = (n4 / 512) * 512;
    const int blocks = 256, reps = 20;
    float4* buf;
    float* out;
    hipMalloc(&buf, (size_t)n4r * 16 * blocks);
    hipMemset(buf, 0, (size_t)n4r * 16 * blocks);
    hipMalloc(&out, 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const char* names[3] = {"same array, lockstep", "same array, rotated start", "distinct arrays"};
    for (int mode = 0; mode < 3; ++mode) {
        for (int it = 0; it < 2; ++it) {
            hipEventRecord(a);
            hipLaunchKernelGGL(stream, dim3(blocks), dim3(512), 0, 0, buf, n4r, reps, mode, out);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            double bytes = (double)n4r * 16 * reps * blocks;
            if (it == 1)
                printf("%-28s %8.3f ms  %7.2f TB/s  %6.1f B/clk/CU @2.4GHz\n", names[mode], ms,
                       bytes / ms / 1e9, bytes / (ms * 1e-3) / 256 / 2.4e9);
        }
    }
    return 0;
}
