// Instruction-fetch cost of straight-line code on MI355X: kernels of N `s_nop 0` (4 bytes, one
// cycle each when the fetch keeps up), 64 / 256 workgroups of 256 threads.  "warm": the same
// kernel back to back; "cold": 8 copies of it at different code addresses launched round robin
// (8 x the code size exceeds the instruction cache from 16 KB on).  Prints us per launch; the
// issue-bound time is N cycles (N / 2.4 GHz).
//     hipcc --offload-arch=gfx950 -O3 ifetch.hip -o ifetch && ./ifetch
#include <hip/hip_runtime.h>
#include <cstdio>

template <int N, int ID>
__global__ void __launch_bounds__(256) k_line(int* out) {
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("s_nop 0");
    if (threadIdx.x == 1023) out[0] = ID;
}

template <int N>
void run(int* d, int blocks) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    void (*ks[8])(int*) = {k_line<N, 0>, k_line<N, 1>, k_line<N, 2>, k_line<N, 3>,
                           k_line<N, 4>, k_line<N, 5>, k_line<N, 6>, k_line<N, 7>};
    for (int i = 0; i < 16; ++i) hipLaunchKernelGGL(ks[i & 7], dim3(blocks), dim3(256), 0, 0, d);
    (void)hipDeviceSynchronize();
    const int reps = 64;
    float warm = 0.f, cold = 0.f;
    (void)hipEventRecord(a);
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(ks[0], dim3(blocks), dim3(256), 0, 0, d);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(&warm, a, b);
    (void)hipEventRecord(a);
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(ks[i & 7], dim3(blocks), dim3(256), 0, 0, d);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(&cold, a, b);
    printf("N=%6d (%6d B): warm %6.2f us/launch, cold %6.2f us/launch\n", N, N * 4, warm * 1e3 / reps,
           cold * 1e3 / reps);
}

int main() {
    int* d;
    (void)hipMalloc(&d, 4);
    for (int blocks : {64, 256}) {
        printf("--- %d workgroups\n", blocks);
        run<16>(d, blocks);
        run<1024>(d, blocks);
        run<2048>(d, blocks);
        run<4096>(d, blocks);
        run<8192>(d, blocks);
        run<16384>(d, blocks);
    }
    return 0;
}
