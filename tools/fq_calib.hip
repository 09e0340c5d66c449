// fq_calib.hip -- on-box peak calibration for bench.py's roofline ("calibrate
// both peaks on the box with a stream-copy kernel and an MFMA loop").  Not part of the product
// ABI (include/flexq_hip.h); built into tools/libfq_calib.so by __graft_entry__.build().
//   fqc_hbm_read : grid-stride 16 B/lane streaming read of a buffer (non-temporal), XOR-reduced
//                  into one word per block so the loads stay live -> achievable HBM read GB/s;
//   fqc_mfma_i8  : every SIMD runs 2 waves of 4 independent v_mfma_i32_16x16x64_i8 chains ->
//                  dense int8 MFMA TOPS.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_hbm_read(const v4i *__restrict__ p, long n, int *__restrict__ sink) {
    v4i acc = {0, 0, 0, 0};
    const long stride = (long)gridDim.x * blockDim.x;
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {  // 4 independent 16 B loads in flight per lane
        const v4i a = __builtin_nontemporal_load(p + i), b = __builtin_nontemporal_load(p + i + stride);
        const v4i c = __builtin_nontemporal_load(p + i + 2 * stride), d = __builtin_nontemporal_load(p + i + 3 * stride);
        acc ^= a ^ b ^ c ^ d;
    }
    for (; i < n; i += stride) acc ^= __builtin_nontemporal_load(p + i);
    const int v = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
    if (v == 0x7fffffff) sink[blockIdx.x] = v;  // practically never: keeps the loads alive
}

__global__ __launch_bounds__(512) void k_mfma_i8(int iters, int *__restrict__ sink) {
    const int lane = threadIdx.x & 63;
    v4i a = {lane, lane + 1, lane + 2, lane + 3}, b = {lane ^ 5, lane ^ 6, lane ^ 7, lane ^ 8};
    v4i c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    for (int it = 0; it < iters; it++) {
        c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(b, a, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, a, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(b, b, c3, 0, 0, 0);
    }
    const v4i s = c0 + c1 + c2 + c3;
    if ((s[0] ^ s[1] ^ s[2] ^ s[3]) == 0x7fffffff) sink[blockIdx.x] = 1;
}

extern "C" int fqc_hbm_read(const void *buf, size_t bytes, int *sink, int blocks, hipStream_t s) {
    hipLaunchKernelGGL(k_hbm_read, dim3(blocks), dim3(256), 0, s, (const v4i *)buf, (long)(bytes / 16), sink);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}

// one 512-thread block per CU (8 waves = 2 per SIMD); each wave issues 4 * iters MFMAs of
// 16 * 16 * 64 * 2 ops
extern "C" int fqc_mfma_i8(int iters, int blocks, int *sink, hipStream_t s) {
    hipLaunchKernelGGL(k_mfma_i8, dim3(blocks), dim3(512), 0, s, iters, sink);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
