// Microbenchmark: cost of "last arrival" signalling between workgroups on MI355X.
// 2016 workgroups (63 per sequence x 32 sequences, the k_sample grid) each store one agent-coherent
// partial and arrive on a counter; the last arrival per sequence reads the 63 partials.
// Variants (hipEvent timing over many launches):
//   0  store only (no counter)                         -> launch + store floor
//   1  one counter per sequence, 63 arrivals           (flat)
//   2  two levels: 8 group counters of 8, then 1 of 8  (hierarchical)
//   3  like 1 but the counters of all sequences on one 128 B line
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ void coh_wait() {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt(0);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}
__device__ __forceinline__ bool arrive(uint32_t* c, uint32_t total) {
    const uint32_t prev = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev + 1 != total) return false;
    __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
}

template <int MODE>
__global__ void __launch_bounds__(256) k_arrive(float* part, uint32_t* cnt, float* out, int nc) {
    __shared__ int s_last;
    const int b = blockIdx.y, c = blockIdx.x;
    if (threadIdx.x == 0) {
        __hip_atomic_store(reinterpret_cast<uint32_t*>(part + b * nc + c), __float_as_uint(1.0f + c),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool last = false;
        if (MODE == 0) {
            last = false;
        } else if (MODE == 1) {
            coh_wait();
            last = arrive(cnt + b * 32, nc);
        } else if (MODE == 3) {
            coh_wait();
            last = arrive(cnt + b, nc);
        } else {
            coh_wait();
            const int g = c / 8, ng = (nc + 7) / 8, gsz = (g == ng - 1) ? nc - 8 * g : 8;
            last = arrive(cnt + (4096 + b * 8 + g) * 32, gsz) && arrive(cnt + b * 32, ng);
        }
        s_last = last;
    }
    __syncthreads();
    if (!s_last) return;
    if (threadIdx.x < 64) {
        float s = 0.f;
        for (int k = threadIdx.x; k < nc; k += 64)
            s += __uint_as_float(__hip_atomic_load(reinterpret_cast<uint32_t*>(part + b * nc + k), __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT));
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
        if (threadIdx.x == 0) out[b] = s;
    }
}

int main() {
    const int B = 32, nc = 63;
    float *part, *out;
    uint32_t* cnt;
    CK(hipMalloc(&part, B * nc * 4));
    CK(hipMalloc(&out, B * 4));
    CK(hipMalloc(&cnt, 1 << 22));
    CK(hipMemset(cnt, 0, 1 << 22));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const float want = nc + nc * (nc - 1) / 2.0f;
    for (int mode = 0; mode < 4; ++mode) {
        auto launch = [&]() {
            const dim3 grid(nc, B);
            if (mode == 0) hipLaunchKernelGGL(k_arrive<0>, grid, dim3(256), 0, 0, part, cnt, out, nc);
            if (mode == 1) hipLaunchKernelGGL(k_arrive<1>, grid, dim3(256), 0, 0, part, cnt, out, nc);
            if (mode == 2) hipLaunchKernelGGL(k_arrive<2>, grid, dim3(256), 0, 0, part, cnt, out, nc);
            if (mode == 3) hipLaunchKernelGGL(k_arrive<3>, grid, dim3(256), 0, 0, part, cnt, out, nc);
        };
        for (int i = 0; i < 20; ++i) launch();
        CK(hipDeviceSynchronize());
        CK(hipMemset(out, 0, B * 4));
        const int iters = 200;
        CK(hipEventRecord(e0));
        for (int i = 0; i < iters; ++i) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        float h[32];
        CK(hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost));
        int ok = 1;
        for (int b = 0; b < B; ++b) ok &= (mode == 0) || (h[b] == want);
        printf("mode %d: %.2f us/launch  (tail sums %s)\n", mode, 1000.f * ms / iters, ok ? "ok" : "WRONG");
    }
    return 0;
}
