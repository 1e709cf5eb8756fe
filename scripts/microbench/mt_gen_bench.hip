// Microbenchmark of the mt19937 recurrence round (k_mt_gen's inner loop, csrc/mt_device.hip):
// S workgroups each extend a 624-word window to L words, with variants:
//   0  k_mt_gen's unrolled rounds (623 independent positions per round, 640 threads), stores
//   1  the same without the global stores (LDS + VALU + barrier only)
//   2  the plain recurrence (454 positions per round, two chained per thread, 256 threads), stores
// Prints us per launch and ns per round.  hipcc --offload-arch=gfx950 -O3 mt_gen_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

constexpr int kN = 624, kM = 397, kLag = 227, kRing = 2048, kBack = 1078, kBlk = 623;

__device__ __forceinline__ uint32_t mag(uint32_t a, uint32_t b) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}
__device__ __forceinline__ uint32_t temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int V>
__global__ void __launch_bounds__(640) k_gen(uint32_t* out, int64_t L, uint32_t* sink) {
    __shared__ uint32_t r[2 * kRing];
    const int t = threadIdx.x;
    uint32_t* o = out + (int64_t)blockIdx.x * L;
    if (t < kN) { r[t] = r[t + kRing] = 0x12345u * (t + 1) + blockIdx.x; }
    __syncthreads();
    if constexpr (V == 2) {
        uint32_t prev = t < kLag ? r[kM + t] : 0u;
        for (int q0 = kN; q0 < L; q0 += 2 * kLag) {
            if (t < kLag) {
                const int q1 = q0 + t, q2 = q1 + kLag;
                const uint32_t x1 = prev ^ mag(r[(q1 - kN) & (kRing - 1)], r[(q1 - kN + 1) & (kRing - 1)]);
                const uint32_t x2 = x1 ^ mag(r[(q2 - kN) & (kRing - 1)], r[(q2 - kN + 1) & (kRing - 1)]);
                r[q1 & (kRing - 1)] = x1;
                r[q2 & (kRing - 1)] = x2;
                if (q1 < L) o[q1] = temper(x1);
                if (q2 < L) o[q2] = temper(x2);
                prev = x2;
            }
            lds_barrier();
        }
        return;
    }
    uint32_t acc = 0;
    for (int q0 = kBack; q0 < L; q0 += kBlk) {
        if (t < kBlk) {
            const int q = q0 + t;
            const uint32_t* b = r + (q & (kRing - 1)) + kRing - kBack;
            const uint32_t x = b[397] ^ mag(b[0], b[1]) ^ mag(b[227], b[228]) ^ mag(b[454], b[455]);
            const int i = q & (kRing - 1);
            r[i] = x;
            r[i + kRing] = x;
            if constexpr (V == 1) acc ^= temper(x);
            else if (q < L) o[q] = temper(x);
        }
        lds_barrier();
    }
    if constexpr (V == 1) if (acc == 0xdeadbeefu) sink[0] = acc;
}

int main() {
    const int S = 313;
    const int64_t L = 131072;
    uint32_t *out, *sink;
    hipMalloc(&out, (size_t)S * L * 4);
    hipMalloc(&sink, 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int v = 0; v < 3; ++v) {
        auto launch = [&]() {
            if (v == 0) hipLaunchKernelGGL(k_gen<0>, dim3(S), dim3(640), 0, 0, out, L, sink);
            if (v == 1) hipLaunchKernelGGL(k_gen<1>, dim3(S), dim3(640), 0, 0, out, L, sink);
            if (v == 2) hipLaunchKernelGGL(k_gen<2>, dim3(S), dim3(256), 0, 0, out, L, sink);
        };
        for (int i = 0; i < 3; ++i) launch();
        hipDeviceSynchronize();
        hipEventRecord(a);
        const int reps = 10;
        for (int i = 0; i < reps; ++i) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double us = ms * 1e3 / reps;
        const double rounds = v == 2 ? (double)(L - kN) / (2 * kLag) : (double)(L - kBack) / kBlk;
        printf("variant %d: %.1f us per launch, %.0f ns per round (%d workgroups x %lld words)\n", v, us,
               us * 1e3 / rounds, S, (long long)L);
    }
    // one workgroup alone: the pure round latency
    for (int v : {0, 1, 2}) {
        auto launch = [&]() {
            if (v == 0) hipLaunchKernelGGL(k_gen<0>, dim3(1), dim3(640), 0, 0, out, L, sink);
            if (v == 1) hipLaunchKernelGGL(k_gen<1>, dim3(1), dim3(640), 0, 0, out, L, sink);
            if (v == 2) hipLaunchKernelGGL(k_gen<2>, dim3(1), dim3(256), 0, 0, out, L, sink);
        };
        launch();
        hipDeviceSynchronize();
        hipEventRecord(a);
        for (int i = 0; i < 5; ++i) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double us = ms * 1e3 / 5;
        const double rounds = v == 2 ? (double)(L - kN) / (2 * kLag) : (double)(L - kBack) / kBlk;
        printf("one workgroup, variant %d: %.1f us, %.0f ns per round\n", v, us, us * 1e3 / rounds);
    }
    return 0;
}
