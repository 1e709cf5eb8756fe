// Microbenchmark: what limits a read-only streaming reduction on MI355X?
// Variants: XOR of the raw words (pure read), + one exp per bf16 element, + online max/sum.
// Buffers: 64 MiB (Infinity-Cache resident when re-read) and 1 GiB (HBM).  hipEvent timing.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ float fexp(float x) {
    constexpr float kL = 1.44269502162933349609375f, kLlo = 1.925963033500011e-08f;
    x = x < -1000.f ? -1000.f : x;
    const float t = x * kL;
    const float err = fmaf(x, kL, -t) + x * kLlo;
    const float r = __builtin_amdgcn_exp2f(t);
    return fmaf(r, err * 0.693147180559945309f, r);
}

template <int MODE, int D>
__global__ void __launch_bounds__(256) k_read(const uint4* __restrict__ p, long n_vec, float* out) {
    float acc = 0.f, m = -INFINITY;
    unsigned x = 0;
    const long stride = (long)gridDim.x * 256;
    long i = (long)blockIdx.x * 256 + threadIdx.x;
    for (; i + (D - 1) * stride < n_vec; i += D * stride) {
        uint4 v[D];
#pragma unroll
        for (int d = 0; d < D; ++d) v[d] = p[i + d * stride];
#pragma unroll
        for (int d = 0; d < D; ++d) {
            if (MODE == 0) {
                x ^= v[d].x ^ v[d].y ^ v[d].z ^ v[d].w;
            } else {
                const unsigned w[4] = {v[d].x, v[d].y, v[d].z, v[d].w};
                float y[8];
#pragma unroll
                for (int k = 0; k < 4; ++k) { y[2 * k] = __uint_as_float(w[k] << 16); y[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u); }
                if (MODE == 1) {
#pragma unroll
                    for (int k = 0; k < 8; ++k) acc += fexp(y[k] - 4.0f);
                } else {
                    float vm = y[0];
#pragma unroll
                    for (int k = 1; k < 8; ++k) vm = fmaxf(vm, y[k]);
                    if (vm > m) { acc = m > -INFINITY ? acc * fexp(m - vm) : 0.f; m = vm; }
#pragma unroll
                    for (int k = 0; k < 8; ++k) acc += fexp(y[k] - m);
                }
            }
        }
    }
    if (acc == 12345.f || x == 0x12345u) out[blockIdx.x] = acc + m + (float)x;
}

template <int MODE, int D>
void run(const char* name, const uint4* p, long bytes, int grid, float* out) {
    const long nv = bytes / 16;
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_read<MODE, D>), dim3(grid), dim3(256), 0, 0, p, nv, out);
    const int n = 20;
    CK(hipEventRecord(a));
    for (int r = 0; r < n; ++r) hipLaunchKernelGGL((k_read<MODE, D>), dim3(grid), dim3(256), 0, 0, p, nv, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    ms /= n;
    printf("%-10s D=%d grid=%5d bytes=%5ld MiB: %8.1f us %7.0f GB/s\n", name, D, grid, bytes >> 20, ms * 1e3, bytes / ms / 1e6);
}

int main() {
    const long big = 1l << 30;
    uint4* p; float* out;
    CK(hipMalloc(&p, big)); CK(hipMalloc(&out, 1 << 20));
    CK(hipMemset(p, 0x3f, big));
    for (long bytes : {32l << 20, 64l << 20, big}) {
        for (int grid : {256, 512, 1024, 2048, 4096, 8192}) {
            run<0, 4>("xor", p, bytes, grid, out);
            run<1, 4>("exp", p, bytes, grid, out);
            run<2, 4>("online", p, bytes, grid, out);
        }
        run<0, 8>("xor", p, bytes, 512, out);
        run<0, 8>("xor", p, bytes, 1024, out);
        run<0, 8>("xor", p, bytes, 2048, out);
        run<2, 8>("online", p, bytes, 2048, out);
        run<0, 1>("xor", p, bytes, 2048, out);
        run<2, 1>("online", p, bytes, 2048, out);
    }
    return 0;
}
