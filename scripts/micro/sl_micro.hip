// Microbenchmark of the sliced evaluator's building blocks (one 512-thread
// workgroup per CU, 256 workgroups): cycles per call measured with s_memtime.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__device__ __forceinline__ unsigned long long now() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

template <int NB>
__device__ __forceinline__ float reduce_chains(const float (&x)[NB], int lane) {
    float v[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) v[i] = x[i];
#pragma unroll
    for (int k = 0, m = NB; m > 1; ++k, m >>= 1) {
        const bool hi = (lane >> k) & 1;
#pragma unroll
        for (int i = 0; i < m / 2; ++i) {
            const float keep = hi ? v[2 * i + 1] : v[2 * i];
            const float send = hi ? v[2 * i] : v[2 * i + 1];
            v[i] = keep + __shfl_xor(send, 1 << k);
        }
    }
    float t = v[0];
#pragma unroll
    for (int msk = NB; msk < 64; msk <<= 1) t = t + __shfl_xor(t, msk);
    return t;
}

template <int NB>
__global__ void __launch_bounds__(512) k_micro(int mode, int reps, int len, float* out,
                                               unsigned long long* cyc) {
    extern __shared__ float sm[];
    const int tid = threadIdx.x, lane = tid & 63;
    for (int i = tid; i < 16384; i += 512) sm[i] = 0.001f * (i % 97);
    __syncthreads();
    float acc = 0.0f;
    float th[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) th[b] = sm[b * 7 + lane];
    const unsigned long long t0 = now();
    for (int r = 0; r < reps; ++r) {
        if (mode == 0) {  // transpose-reduce of NB values
            float x[NB];
#pragma unroll
            for (int b = 0; b < NB; ++b) x[b] = th[b] + (float)r;
            acc += reduce_chains<NB>(x, lane);
        } else if (mode == 1) {  // moments over len elements, NB chains, data from LDS
            float s1[NB], s2[NB];
#pragma unroll
            for (int b = 0; b < NB; ++b) s1[b] = s2[b] = 0.0f;
            const float* xv = sm + 4 * lane + (r & 7) * 16;
            for (int u4 = 0; u4 < len / 4; ++u4) {
                const float4 a = *(const float4*)(xv + u4 * 256);
                const float e[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int b = 0; b < NB; ++b) {
                        const float d = e[j] - th[b];
                        s1[b] += d;
                        s2[b] = fmaf(d, d, s2[b]);
                    }
            }
#pragma unroll
            for (int b = 0; b < NB; ++b) acc += s1[b] * s2[b];
        } else if (mode == 2) {  // barrier
            __syncthreads();
            acc += sm[(tid + r) & 1023];
        } else if (mode == 3) {  // dependent LDS read chain
            int idx = tid & 1023;
            idx = __float_as_int(sm[idx]) & 1023;
            acc += (float)idx;
        } else if (mode == 4) {  // wave_sum x NB via DPP-free shfl butterfly (old deposit)
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                float x = th[b] + r;
                for (int m = 1; m < 64; m <<= 1) x += __shfl_xor(x, m);
                acc += x;
            }
        }
    }
    const unsigned long long t1 = now();
    out[blockIdx.x * 512 + tid] = acc;
    if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    float* out;
    unsigned long long* cyc;
    hipMalloc(&out, 256 * 512 * 4);
    hipMalloc(&cyc, 256 * 8);
    std::vector<unsigned long long> h(256);
    const char* names[] = {"reduce_chains<16>", "moments 16ch x len", "barrier", "dep LDS read",
                           "16 shfl wave sums"};
    hipFuncSetAttribute((const void*)k_micro<16>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
    for (int mode = 0; mode < 5; ++mode) {
        for (int len : {4, 12, 32}) {
            if (mode != 1 && len != 12) continue;
            const int reps = 200;
            hipLaunchKernelGGL(k_micro<16>, dim3(256), dim3(512), 65536, 0, mode, reps, len, out, cyc);
            hipDeviceSynchronize();
            hipLaunchKernelGGL(k_micro<16>, dim3(256), dim3(512), 65536, 0, mode, reps, len, out, cyc);
            hipDeviceSynchronize();
            hipMemcpy(h.data(), cyc, 256 * 8, hipMemcpyDeviceToHost);
            double m = 0;
            for (auto v : h) m += v;
            m /= 256;
            printf("%-22s len=%2d : %8.1f cycles per call (wave 0)\n", names[mode], len, m / reps);
        }
    }
    return 0;
}
