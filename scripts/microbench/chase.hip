// Dependent-load latency on MI355X: one thread per workgroup follows a pointer chain of N hops
// through a buffer of S bytes (random permutation, 256-byte spacing), hipEvent-timed.
// S = 256 KiB (L2-resident), 64 MiB (Infinity Cache), 4 GiB (HBM).  32 workgroups (like the
// per-sequence tails) and 1 workgroup.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <algorithm>
#include <random>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void k_chase(const uint64_t* __restrict__ buf, int hops, uint64_t* out) {
    if (threadIdx.x != 0) return;
    uint64_t i = (blockIdx.x * 7919ull) % 1024;
    for (int h = 0; h < hops; ++h) i = buf[i * 32];   // 256-byte stride between nodes
    out[blockIdx.x] = i;
}

int main() {
    const size_t sizes[] = {256ull << 10, 64ull << 20, 4ull << 30};
    const char* names[] = {"256KiB(L2)", "64MiB(MALL)", "4GiB(HBM)"};
    uint64_t* out;
    CK(hipMalloc(&out, 64 * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int si = 0; si < 3; ++si) {
        const size_t nodes = sizes[si] / 256;
        std::vector<uint64_t> perm(nodes);
        for (size_t k = 0; k < nodes; ++k) perm[k] = k;
        std::shuffle(perm.begin(), perm.end(), std::mt19937_64(42));
        std::vector<uint64_t> next(nodes);
        for (size_t k = 0; k < nodes; ++k) next[perm[k]] = perm[(k + 1) % nodes];
        std::vector<uint64_t> host(nodes * 32, 0);
        for (size_t k = 0; k < nodes; ++k) host[k * 32] = next[k];
        uint64_t* buf;
        CK(hipMalloc(&buf, sizes[si]));
        CK(hipMemcpy(buf, host.data(), sizes[si], hipMemcpyHostToDevice));
        for (int wgs : {1, 32}) {
            for (int hops : {1, 64}) {
                hipLaunchKernelGGL(k_chase, dim3(wgs), dim3(64), 0, 0, buf, hops, out);
                CK(hipDeviceSynchronize());
                const int iters = 50;
                CK(hipEventRecord(e0));
                for (int it = 0; it < iters; ++it) hipLaunchKernelGGL(k_chase, dim3(wgs), dim3(64), 0, 0, buf, hops, out);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                printf("%-12s wgs=%2d hops=%2d: %8.2f us/launch\n", names[si], wgs, hops, 1000.f * ms / iters);
            }
        }
        CK(hipFree(buf));
    }
    return 0;
}
