// Probe: semantics of v_permlane32_swap / v_permlane16_swap on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* out) {
    const int i = threadIdx.x;
    int a = 1000 + i, b = 2000 + i;
    auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    out[i] = r[0];
    out[64 + i] = r[1];
    auto q = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    out[128 + i] = q[0];
    out[192 + i] = q[1];
}
int main() {
    int* d;
    hipMalloc(&d, 256 * 4);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    int h[256];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    const char* nm[4] = {"p32 r0", "p32 r1", "p16 r0", "p16 r1"};
    for (int t = 0; t < 4; ++t) {
        printf("%s:", nm[t]);
        for (int i = 0; i < 64; i += 8) printf(" [%d]=%d", i, h[t * 64 + i]);
        printf("\n");
    }
    return 0;
}
