// How long does one s_memrealtime take (timestamp overhead of the phase-timing build)?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void k(uint64_t* out) {
    uint64_t t[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) t[i] = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0)
        for (int i = 0; i < 9; ++i) out[blockIdx.x * 9 + i] = t[i];
}
int main() {
    uint64_t* d;
    hipMalloc(&d, 64 * 9 * 8);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k, dim3(32), dim3(256), 0, 0, d);
    hipDeviceSynchronize();
    uint64_t h[64 * 9];
    hipMemcpy(h, d, sizeof(uint64_t) * 32 * 9, hipMemcpyDeviceToHost);
    for (int b = 0; b < 4; ++b) {
        printf("wg %d:", b);
        for (int i = 1; i < 9; ++i) printf(" %llu", (unsigned long long)(h[b * 9 + i] - h[b * 9 + i - 1]));
        printf("  (ticks of 10 ns)\n");
    }
    return 0;
}
