// Microbenchmark: variants of the row-statistics pass on the bench layout (rows x 128256 bf16,
// N(0,3^2) data), to find what separates it from a plain streaming reduction.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>
#include <cstring>
#include "sd_device.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
using namespace sd;
constexpr int kV = 128256, kStep = 2048;

// VAR 0: branchy online (product), 1: branch-free online (rescale every vector),
// 2: fixed reference max (no online), 3: xor only (no math), 4: lazy reference m (k_stats),
// 5: lazy reference m with packed f32 math (v_pk_fma / v_pk_add)
template <int VAR, int PIPE>
__global__ void __launch_bounds__(256) k_var(const uint16_t* rows, int chunk, int n_chunks, float2* part) {
    const int r = blockIdx.y, c = blockIdx.x;
    const uint16_t* row = rows + (long)r * kV;
    const long lo = (long)c * chunk, hi = lo + chunk < kV ? lo + chunk : kV;
    const int nfull = (int)((hi - lo) / kStep), nit = (int)((hi - lo + kStep - 1) / kStep);
    float m = -INFINITY, acc = 0.f;
    unsigned xx = 0;
    auto consume = [&](const float* y) {
        if (VAR == 3) { for (int k = 0; k < 8; ++k) xx ^= __float_as_uint(y[k]); return; }
        if (VAR == 2) { for (int k = 0; k < 8; ++k) acc += sd_exp(y[k] - 16.f); return; }
        if (VAR == 4 || VAR == 5) {
            constexpr float L = 1.44269502162933349609375f;
            float sv = 0.f;
            if (VAR == 4) {
#pragma unroll
                for (int k = 0; k < 8; ++k) sv += __builtin_amdgcn_exp2f((y[k] - m) * L);
            } else {
                typedef float f2 __attribute__((ext_vector_type(2)));
                const f2 mL = {-m * L, -m * L}, LL = {L, L};
                f2 s2 = {0.f, 0.f};
#pragma unroll
                for (int k = 0; k < 8; k += 2) {
                    f2 t = f2{y[k], y[k + 1]} * LL + mL;
                    s2 += f2{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
                }
                sv = s2.x + s2.y;
            }
            if (!(sv < 1.8446744e19f)) {
                float vm = -INFINITY;
                for (int k = 0; k < 8; ++k) vm = fmaxf(vm, y[k]);
                if (vm > m) { acc = m > -INFINITY ? acc * sd_exp(m - vm) : 0.f; m = vm; }
                sv = 0.f;
                for (int k = 0; k < 8; ++k) sv += __builtin_amdgcn_exp2f((y[k] - m) * L);
            }
            acc += sv;
            return;
        }
        float vm = y[0];
#pragma unroll
        for (int k = 1; k < 8; ++k) vm = fmaxf(vm, y[k]);
        if (VAR == 0) {
            if (vm > m) { acc = m > -INFINITY ? acc * sd_exp(m - vm) : 0.f; m = vm; }
        } else {
            const float mn = fmaxf(m, vm);
            acc = m > -INFINITY ? acc * sd_exp(m - mn) : 0.f;
            m = mn;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) acc += sd_exp(y[k] - m);
    };
    if (nfull > 0) {
        const uint4* vb = reinterpret_cast<const uint4*>(row + lo) + threadIdx.x;
        uint4 buf[PIPE];
#pragma unroll
        for (int d = 0; d < PIPE; ++d) buf[d] = vb[(d < nfull ? d : nfull - 1) * 256];
        int it = 0;
        for (; it + PIPE <= nfull; it += PIPE) {
#pragma unroll
            for (int d = 0; d < PIPE; ++d) {
                const uint4 v = buf[d];
                const int nx = it + d + PIPE;
                buf[d] = vb[(nx < nfull ? nx : nfull - 1) * 256];
                float x[8];
                unpack16<SD_BF16>(v, x);
                consume(x);
            }
        }
#pragma unroll
        for (int d = 0; d < PIPE; ++d)
            if (it + d < nfull) { float x[8]; unpack16<SD_BF16>(buf[d], x); consume(x); }
    }
    for (int it = nfull; it < nit; ++it) {
        const long e0 = lo + ((long)it * 256 + threadIdx.x) * 8;
        float x[8];
        for (int k = 0; k < 8; ++k) x[k] = e0 + k < hi ? bf16_bits_to_f32(row[e0 + k]) : -INFINITY;
        consume(x);
    }
    for (int o = 32; o > 0; o >>= 1) {
        const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(acc, o, 64);
        const float mn = fmaxf(m, m2);
        if (mn > -INFINITY) { acc = (m > -INFINITY ? acc * sd_exp(m - mn) : 0.f) + (m2 > -INFINITY ? s2 * sd_exp(m2 - mn) : 0.f); m = mn; }
    }
    if ((threadIdx.x & 63) == 0) part[((long)r * n_chunks + c) * 4 + (threadIdx.x >> 6)] = make_float2(m, acc + (float)xx);
}

template <int VAR, int PIPE>
void run(const char* name, const uint16_t* rows, int nrows, int stages, float2* part) {
    const int chunk = stages * kStep, nch = (kV + chunk - 1) / chunk;
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    const dim3 grid(nch, nrows);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_var<VAR, PIPE>), grid, dim3(256), 0, 0, rows, chunk, nch, part);
    const int n = 20;
    CK(hipEventRecord(a));
    for (int i = 0; i < n; ++i) hipLaunchKernelGGL((k_var<VAR, PIPE>), grid, dim3(256), 0, 0, rows, chunk, nch, part);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); ms /= n;
    const double bytes = 2.0 * kV * nrows;
    printf("%-16s pipe=%d stages=%2d grid=%5d: %7.1f us %6.0f GB/s\n", name, PIPE, stages, nch * nrows, ms * 1e3, bytes / ms / 1e6);
}

int main() {
    const int nrows = 128;   // the bench's target rows: 32 sequences x 4
    std::vector<uint16_t> h((size_t)nrows * kV);
    std::mt19937 g(1);
    std::normal_distribution<float> nd(0.f, 3.f);
    for (auto& v : h) { float f = nd(g); unsigned u; memcpy(&u, &f, 4); v = (uint16_t)((u + 0x7fff + ((u >> 16) & 1)) >> 16); }
    uint16_t* d; float2* part;
    CK(hipMalloc(&d, h.size() * 2)); CK(hipMalloc(&part, 1 << 24));
    CK(hipMemcpy(d, h.data(), h.size() * 2, hipMemcpyHostToDevice));
    for (int st : {4, 8, 16}) {
        run<3, 4>("xor", d, nrows, st, part);
        run<4, 4>("lazy", d, nrows, st, part);
        run<5, 4>("lazy-packed", d, nrows, st, part);
        run<4, 8>("lazy", d, nrows, st, part);
        run<5, 8>("lazy-packed", d, nrows, st, part);
        run<3, 8>("xor", d, nrows, st, part);
    }
    run<2, 4>("fixed-max", d, nrows, 16, part);
    return 0;
}
