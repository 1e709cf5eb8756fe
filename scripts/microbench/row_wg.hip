// Microbenchmark: how fast can FEW workgroups stream one 128256-wide bf16 row each?  The drafter
// draw reads 32 rows per launch; today it spreads each row over ~63 workgroups and pays a
// cross-workgroup exchange (store, counter, reload).  Here: W workgroups of T threads per row, a
// lazy-reference Σexp over the row, the workgroup's (m, S) reduced in LDS, no exchange.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
constexpr int kV = 128256;

template <int T, int PIPE>
__global__ void __launch_bounds__(T) k_row(const uint16_t* rows, int wpr, float2* out) {
    const int r = blockIdx.y, c = blockIdx.x;
    const uint16_t* row = rows + (long)r * kV;
    constexpr int STEP = T * 8;
    const int nst = kV / STEP;                       // full stages (the ragged end is skipped here)
    const int lo = (int)((long)nst * c / wpr), hi = (int)((long)nst * (c + 1) / wpr), n = hi - lo;
    const uint4* vb = reinterpret_cast<const uint4*>(row) + (long)lo * T + threadIdx.x;
    constexpr float L = 1.44269502162933349609375f;
    float m = -INFINITY, acc = 0.f;
    auto consume = [&](uint4 v) {
        const unsigned w[4] = {v.x, v.y, v.z, v.w};
        float y[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) { y[2 * k] = __uint_as_float(w[k] << 16); y[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u); }
        float sv = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) sv += __builtin_amdgcn_exp2f((y[k] - m) * L);
        if (!(sv < 1.8446744e19f)) {
            float vm = -INFINITY;
            for (int k = 0; k < 8; ++k) vm = fmaxf(vm, y[k]);
            if (vm > m) { acc = m > -INFINITY ? acc * __builtin_amdgcn_exp2f((m - vm) * L) : 0.f; m = vm; }
            sv = 0.f;
            for (int k = 0; k < 8; ++k) sv += __builtin_amdgcn_exp2f((y[k] - m) * L);
        }
        acc += sv;
    };
    uint4 buf[PIPE];
    // n >= 1 (the host keeps wpr <= stages per row): the clamped prefetch index never goes below 0
#pragma unroll
    for (int d = 0; d < PIPE; ++d) buf[d] = vb[(long)(d < n ? d : n - 1) * T];
    int it = 0;
    for (; it + PIPE <= n; it += PIPE) {
#pragma unroll
        for (int d = 0; d < PIPE; ++d) {
            const uint4 v = buf[d];
            const int nx = it + d + PIPE;
            buf[d] = vb[(long)(nx < n ? nx : n - 1) * T];
            consume(v);
        }
    }
#pragma unroll
    for (int d = 0; d < PIPE; ++d)
        if (it + d < n) consume(buf[d]);
    for (int o = 32; o > 0; o >>= 1) {
        const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(acc, o, 64);
        const float mn = fmaxf(m, m2);
        if (mn > -INFINITY) { acc = (m > -INFINITY ? acc * __builtin_amdgcn_exp2f((m - mn) * L) : 0.f) + (m2 > -INFINITY ? s2 * __builtin_amdgcn_exp2f((m2 - mn) * L) : 0.f); m = mn; }
    }
    __shared__ float2 lw[T / 64];
    if ((threadIdx.x & 63) == 0) lw[threadIdx.x >> 6] = make_float2(m, acc);
    __syncthreads();
    if (threadIdx.x == 0) {
        float M = -INFINITY, S = 0.f;
        for (int k = 0; k < T / 64; ++k) M = fmaxf(M, lw[k].x);
        for (int k = 0; k < T / 64; ++k) S += lw[k].y * __builtin_amdgcn_exp2f((lw[k].x - M) * L);
        out[r * wpr + c] = make_float2(M, S);
    }
}

template <int T, int PIPE>
void run(const uint16_t* rows, int nrows, int wpr, float2* out) {
    if (wpr > kV / (T * 8)) return;   // a workgroup without a full stage would index before its row
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    const dim3 grid(wpr, nrows);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_row<T, PIPE>), grid, dim3(T), 0, 0, rows, wpr, out);
    const int n = 20;
    CK(hipEventRecord(a));
    for (int i = 0; i < n; ++i) hipLaunchKernelGGL((k_row<T, PIPE>), grid, dim3(T), 0, 0, rows, wpr, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); ms /= n;
    printf("T=%4d pipe=%d wg/row=%2d grid=%5d: %7.2f us %6.0f GB/s\n", T, PIPE, wpr, wpr * nrows, ms * 1e3,
           2.0 * kV * nrows / ms / 1e6);
}

int main() {
    const int nrows = 32;
    std::vector<uint16_t> h((size_t)nrows * kV);
    std::mt19937 g(1);
    std::normal_distribution<float> nd(0.f, 3.f);
    for (auto& v : h) { float f = nd(g); unsigned u; memcpy(&u, &f, 4); v = (uint16_t)(u >> 16); }
    uint16_t* d; float2* out;
    CK(hipMalloc(&d, h.size() * 2)); CK(hipMalloc(&out, 1 << 20));
    CK(hipMemcpy(d, h.data(), h.size() * 2, hipMemcpyHostToDevice));
    for (int wpr : {1, 2, 4, 8}) {
        run<1024, 4>(d, nrows, wpr, out);
        run<1024, 8>(d, nrows, wpr, out);
        run<512, 8>(d, nrows, wpr, out);
        run<256, 8>(d, nrows, wpr, out);
    }
    return 0;
}
