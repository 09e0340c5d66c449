// cu_blocker.hip -- test infrastructure only (tests/test_gpu_chain.py): a kernel that holds `blocks` CUs
// (one workgroup per CU: it takes all 160 KiB of the CU's LDS) for `ms` milliseconds of s_memrealtime
// (100 MHz), so that a decode chain launched beside it on another stream cannot have all of its
// workgroups resident -- the co-residency failure the chain's bounded waits must turn into a reported
// timeout, never a hang.  Every wave ends after `ms`.
#include <hip/hip_runtime.h>

__global__ __launch_bounds__(64) void fq_test_cu_blocker_kernel(unsigned long long ticks, int *sink) {
    extern __shared__ int lds[];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    int acc = 0;
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
        __builtin_amdgcn_s_sleep(127);
        acc += lds[threadIdx.x];
    }
    if (acc == 0x7fffffff) sink[blockIdx.x] = acc;  // (never true: keeps the loop)
}

extern "C" int fq_test_cu_blocker(int blocks, int ms, int *sink, void *stream) {
    const size_t lds = 160 * 1024;
    if (hipFuncSetAttribute(reinterpret_cast<const void *>(fq_test_cu_blocker_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return 1;
    hipLaunchKernelGGL(fq_test_cu_blocker_kernel, dim3(blocks), dim3(64), lds, (hipStream_t)stream,
                       (unsigned long long)ms * 100000ull, sink);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}
