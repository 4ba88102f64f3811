// Microbenchmark of the sliced kernel's exchange: groups of S workgroups
// (512 threads, one per CU) repeatedly publish NI*NB tagged granules each and
// poll all S*NI*NB of their group.  Cycles per exchange, by polling variant:
//   mode 0: every thread polls its granules (s_sleep 1 between polls)
//   mode 1: as 0 with s_sleep 8
//   mode 2: wave 0 polls everything, others wait at the barrier
//   mode 3: per-slice arrival counter (atomic add after vmcnt(0)), one lane polls it,
//           then payload read with sc1 loads
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned int gu32;

__device__ __forceinline__ unsigned long long now() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

__global__ void __launch_bounds__(512) k_xch(int S, int items, int reps, int mode, int work,
                                             unsigned long long* g, unsigned* cnt, float* out,
                                             unsigned long long* cyc) {
    __shared__ float xin[4096];
    __shared__ int done;
    const int tid = threadIdx.x;
    const int w = blockIdx.x, nwg = gridDim.x;
    const int x = w & 7, r = w >> 3;
    const int gpx = (nwg / 8) / S;
    const int grp = x * gpx + r / S, slice = r % S;
    const int ngroups = nwg / S;
    float acc = 0.0f;
    unsigned long long tpoll = 0;
    const unsigned long long t0 = now();
    for (int e = 1; e <= reps; ++e) {
        unsigned long long* xg = g + ((size_t)(e & 1) * ngroups + grp) * S * items;
        for (int i = tid; i < items; i += 512)
            __hip_atomic_store((gu64*)(xg + slice * items + i),
                               ((unsigned long long)e << 32) | __float_as_uint(acc + i),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        {   // work between publishing and polling
            float v = (float)tid;
            for (int i = 0; i < work; ++i) v = v * 0.999f + 1.0f;
            acc += v;
        }
        const unsigned long long tp0 = now();
        if (mode == 4) {
            // parallel polling of this thread's granules (as in the kernel)
            float v[4];
            unsigned need = 0;
            for (int p = 0; p < 4; ++p) { v[p] = 0.f; if (p * 512 + tid < S * items) need |= 1u << p; }
            while (need) {
                unsigned long long y[4];
#pragma unroll
                for (int p = 0; p < 4; ++p)
                    if ((need >> p) & 1u)
                        y[p] = __hip_atomic_load((gu64*)(xg + p * 512 + tid), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
                for (int p = 0; p < 4; ++p)
                    if (((need >> p) & 1u) && (unsigned)(y[p] >> 32) == (unsigned)e) {
                        v[p] = __uint_as_float((unsigned)y[p]);
                        need &= ~(1u << p);
                    }
                if (need) __builtin_amdgcn_s_sleep(1);
            }
            for (int p = 0; p < 4; ++p) if (p * 512 + tid < S * items) xin[(p * 512 + tid) & 4095] = v[p];
        } else if (mode == 3) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0)
                __hip_atomic_fetch_add((gu32*)(cnt + grp), 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            if (tid == 0) {
                while (__hip_atomic_load((gu32*)(cnt + grp), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT) < (unsigned)(e * S))
                    __builtin_amdgcn_s_sleep(1);
            }
            __syncthreads();
            for (int i = tid; i < S * items; i += 512) {
                const unsigned long long y =
                    __hip_atomic_load((gu64*)(xg + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                xin[i & 4095] = __uint_as_float((unsigned)y);
            }
        } else if (mode == 2) {
            if (tid < 64) {
                for (int i = tid; i < S * items; i += 64) {
                    unsigned long long y;
                    do {
                        y = __hip_atomic_load((gu64*)(xg + i), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
                        if ((unsigned)(y >> 32) == (unsigned)e) break;
                        __builtin_amdgcn_s_sleep(1);
                    } while (true);
                    xin[i & 4095] = __uint_as_float((unsigned)y);
                }
            }
        } else {
            for (int i = tid; i < S * items; i += 512) {
                unsigned long long y;
                do {
                    y = __hip_atomic_load((gu64*)(xg + i), __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
                    if ((unsigned)(y >> 32) == (unsigned)e) break;
                    if (mode == 1) __builtin_amdgcn_s_sleep(8);
                    else __builtin_amdgcn_s_sleep(1);
                } while (true);
                xin[i & 4095] = __uint_as_float((unsigned)y);
            }
        }
        tpoll += now() - tp0;
        __syncthreads();
        acc += xin[(tid * 7) & 4095];
        __syncthreads();
    }
    const unsigned long long t1 = now();
    out[w * 512 + tid] = acc;
    if (tid == 0) { cyc[w] = t1 - t0; cyc[256 + w] = tpoll; }
}

int main() {
    const int NWG = 256, reps = 400;
    unsigned long long *g, *cyc;
    unsigned* cnt;
    float* out;
    hipMalloc(&g, 2 * 4096 * 256 * 8);
    hipMalloc(&cnt, 4096 * 4);
    hipMalloc(&out, NWG * 512 * 4);
    hipMalloc(&cyc, 2 * NWG * 8);
    std::vector<unsigned long long> h(2 * NWG);
    const char* names[] = {"all threads poll, sleep1", "all threads poll, sleep8",
                           "wave 0 polls", "arrival counter + payload", "parallel poll"};
    for (int S : {16}) {
        for (int mode : {0, 4}) {
            for (int work : {0, 50, 150, 400}) {
                const int items = 96;
                for (int rep = 0; rep < 2; ++rep) {
                    hipMemset(g, 0, 2 * 4096 * 256 * 8);
                    hipMemset(cnt, 0, 4096 * 4);
                    hipLaunchKernelGGL(k_xch, dim3(NWG), dim3(512), 0, 0, S, items, reps, mode,
                                       work, g, cnt, out, cyc);
                    hipDeviceSynchronize();
                }
                hipMemcpy(h.data(), cyc, 2 * NWG * 8, hipMemcpyDeviceToHost);
                double m = 0, mp = 0;
                for (int i = 0; i < NWG; ++i) { m += h[i]; mp += h[NWG + i]; }
                m /= NWG; mp /= NWG;
                printf("S=%2d work=%4d %-28s %8.0f cycles per exchange, poll phase %7.0f\n", S,
                       work, names[mode], m / reps, mp / reps);
            }
        }
    }
    return 0;
}
