// Exhaustive check (all 2^32 fp32 bit patterns) that gfx950's v_cvt_pk_bf16_f32 (the (__bf16)
// conversion) rounds exactly as the integer round-to-nearest-even sd_device.h used before: equal
// bits for every non-NaN input, NaN for every NaN input.  Run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 scripts/microbench/bf16_round.hip -o /tmp/bf16_round && /tmp/bf16_round
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ float sw_round(float f) {
    uint32_t u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return __uint_as_float(u | 0x00400000u);
    u = (u + 0x7fffu + ((u >> 16) & 1u)) & 0xffff0000u;
    return __uint_as_float(u);
}
__device__ __forceinline__ float hw_round(float f) { return (float)(__bf16)f; }

__global__ void check(uint64_t lo, unsigned long long* bad, uint32_t* first) {
    const uint64_t i = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t u = (uint32_t)i;
    const float f = __uint_as_float(u);
    const float a = sw_round(f), b = hw_round(f);
    const bool nan_a = a != a, nan_b = b != b;
    const bool ok = nan_a ? nan_b : (__float_as_uint(a) == __float_as_uint(b));
    if (!ok) {
        const unsigned long long n = atomicAdd(bad, 1ull);
        if (n < 8) first[n] = u;
    }
}

int main() {
    unsigned long long* bad;
    uint32_t* first;
    (void)hipMalloc(&bad, 8);
    (void)hipMalloc(&first, 32);
    (void)hipMemset(bad, 0, 8);
    const uint64_t chunk = 1ull << 30;
    for (uint64_t lo = 0; lo < (1ull << 32); lo += chunk)
        hipLaunchKernelGGL(check, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, lo, bad, first);
    unsigned long long h = 0;
    uint32_t f[8] = {};
    (void)hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(f, first, 32, hipMemcpyDeviceToHost);
    printf("bf16 rounding mismatches over 2^32 inputs: %llu\n", h);
    for (int k = 0; k < 8 && k < (int)h; ++k) printf("  0x%08x\n", f[k]);
    return h != 0;
}
