// TEST HELPER, not product code: a kernel that occupies the CUs of some XCDs for a while, so a GPU
// test can run the library's poll-mode kernels beside it (tests/test_gpu_busy.py).  Every workgroup
// reads its XCD (HW_REG_XCC_ID); on an XCD selected by xcd_mask it allocates the whole CU's LDS
// (dynamic, 160 KiB) and sleeps until `us` microseconds of wall clock (s_memrealtime, 100 MHz) have
// passed since it started; elsewhere it returns at once.  A grid of several workgroups per CU keeps
// the selected XCDs full for the whole time: a kernel launched on another stream meanwhile gets no
// slot there and runs only on the other XCDs.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void __launch_bounds__(64) k_busy(uint32_t xcd_mask, uint32_t us, uint32_t* ran) {
    extern __shared__ uint32_t lds[];
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    xcc &= 0xfu;
    if (((xcd_mask >> xcc) & 1u) == 0u) return;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)us * 100u) __builtin_amdgcn_s_sleep(127);
    lds[threadIdx.x] = xcc;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(ran, lds[0] < 8u ? 1u : 0u);   // a vector atomic: counts busy workgroups
}

extern "C" int32_t sd_test_busy(uint32_t grid, uint32_t xcd_mask, uint32_t us, uint32_t lds_bytes, void* ran,
                                void* stream) {
    if (hipFuncSetAttribute((const void*)k_busy, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes) !=
        hipSuccess)
        return -1;
    hipLaunchKernelGGL(k_busy, dim3(grid), dim3(64), lds_bytes, (hipStream_t)stream, xcd_mask, us,
                       static_cast<uint32_t*>(ran));
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
