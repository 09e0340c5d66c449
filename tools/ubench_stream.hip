// ubench_stream.hip -- development microbenchmark: how fast can a wave-per-contiguous-range
// stream of 3 KiB blocks run on this GPU?  Variants:
//   glds   : LDS-DMA ring (D slots per wave), hand-counted vmcnt, ds_read of the slot
//   reg    : 3 x global_load_dwordx4 per block straight to registers, unrolled by D
// Usage: ubench_stream <MiB> <waves_per_wg> <wgs> <D>     (prints GB/s per variant)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));
#define LDS_PTR(p) ((__attribute__((address_space(3))) void *)(p))

__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char *)(p);
}
__device__ __forceinline__ v4i ds_read_b128(uint32_t a) {
    v4i v;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a));
    return v;
}

template <int D>
__global__ void k_glds(const char *__restrict__ w, long nblocks, int L, int *out) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nw = blockDim.x >> 6;
    const long k = (long)blockIdx.x * nw + wid;
    long b0 = k * L;
    if (b0 > nblocks) b0 = nblocks;
    long b1 = b0 + L < nblocks ? b0 + L : nblocks;
    const int n = (int)(b1 - b0);
    char *ring = smem + wid * D * 3072;
    auto issue = [&](long b, int slot) {
        const char *src = w + b * 3072 + lane * 16;
#pragma unroll
        for (int r = 0; r < 3; r++)
            __builtin_amdgcn_global_load_lds(src + r * 1024, LDS_PTR(ring + slot * 3072 + r * 1024), 16, 0, 2);
    };
    for (int i = 0; i < (n < D ? n : D); i++) issue(b0 + i, i);
    v4i acc = {0, 0, 0, 0};
    for (int i = 0; i < n; i++) {
        const int later = (n - 1 - i) < (D - 1) ? (n - 1 - i) : (D - 1);
        switch (later) {
            case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
            case 1: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
            case 2: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
            case 3: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
            case 4: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
            case 5: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
            case 6: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
            default: asm volatile("s_waitcnt vmcnt(21)" ::: "memory"); break;
        }
        const int slot = i % D;
        const uint32_t sp = lds_addr(ring + slot * 3072 + lane * 16);
        v4i a = ds_read_b128(sp), b = ds_read_b128(sp + 1024), c = ds_read_b128(sp + 2048);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        if (i + D < n) issue(b0 + i + D, slot);
        acc ^= a ^ b ^ c;
    }
    if (acc.x == 0x12345678) out[0] = acc.y;
}

template <int D>
__global__ void k_reg(const char *__restrict__ w, long nblocks, int L, int *out) {
    const int lane = threadIdx.x & 63, nw = blockDim.x >> 6;
    const long k = (long)blockIdx.x * nw + (threadIdx.x >> 6);
    long b0 = k * L;
    if (b0 > nblocks) b0 = nblocks;
    long b1 = b0 + L < nblocks ? b0 + L : nblocks;
    v4i acc = {0, 0, 0, 0};
    long b = b0;
    for (; b + D <= b1; b += D) {
        v4i r[D][3];
#pragma unroll
        for (int j = 0; j < D; j++)
#pragma unroll
            for (int q = 0; q < 3; q++)
                r[j][q] = __builtin_nontemporal_load(reinterpret_cast<const v4i *>(w + (b + j) * 3072 + q * 1024 + lane * 16));
#pragma unroll
        for (int j = 0; j < D; j++) acc ^= r[j][0] ^ r[j][1] ^ r[j][2];
    }
    for (; b < b1; b++)
#pragma unroll
        for (int q = 0; q < 3; q++) acc ^= __builtin_nontemporal_load(reinterpret_cast<const v4i *>(w + b * 3072 + q * 1024 + lane * 16));
    if (acc.x == 0x12345678) out[0] = acc.y;
}

__global__ void k_copy(const v4i *__restrict__ a, v4i *__restrict__ b, long n) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) b[i] = a[i];
}

#define CK(x) do { if ((x) != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(x), __LINE__); exit(1); } } while (0)

template <typename F>
float timeit(F f, int reps) {
    hipEvent_t s, e;
    CK(hipEventCreate(&s));
    CK(hipEventCreate(&e));
    for (int i = 0; i < 3; i++) f(i);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(s));
    for (int i = 0; i < reps; i++) f(i);
    CK(hipEventRecord(e));
    CK(hipEventSynchronize(e));
    float ms;
    CK(hipEventElapsedTime(&ms, s, e));
    return ms * 1e3f / reps;  // us
}

int main(int argc, char **argv) {
    const long mib = argc > 1 ? atol(argv[1]) : 34;
    const int copies = 8;  // rotate buffers so the 256 MiB MALL cannot hold them
    const long bytes = mib << 20;
    const long nblocks = bytes / 3072;
    std::vector<char *> bufs(copies);
    for (auto &p : bufs) {
        CK(hipMalloc(&p, nblocks * 3072));
        CK(hipMemset(p, 1, nblocks * 3072));
    }
    int *out;
    CK(hipMalloc(&out, 64));
    const int reps = 200;
    printf("stream %ld MiB (%ld blocks of 3 KiB), %d buffers rotated\n", mib, nblocks, copies);
    for (int nw : {4, 8}) {
        for (int wpc : {1, 2, 4}) {  // WGs per CU
            const int wgs = 256 * wpc;
            const long waves = (long)wgs * nw;
            const int L = (int)((nblocks + waves - 1) / waves);
            float t4 = timeit([&](int i) { k_glds<4><<<wgs, nw * 64, nw * 4 * 3072>>>(bufs[i % copies], nblocks, L, out); }, reps);
            float t8 = (nw * 8 * 3072 <= 160 * 1024) ? timeit([&](int i) { k_glds<8><<<wgs, nw * 64, nw * 8 * 3072>>>(bufs[i % copies], nblocks, L, out); }, reps) : 0;
            float r4 = timeit([&](int i) { k_reg<4><<<wgs, nw * 64>>>(bufs[i % copies], nblocks, L, out); }, reps);
            float r8 = timeit([&](int i) { k_reg<8><<<wgs, nw * 64>>>(bufs[i % copies], nblocks, L, out); }, reps);
            printf("nw=%d wg/cu=%d L=%3d  glds D4 %7.2f us %6.0f GB/s | glds D8 %7.2f us %6.0f GB/s | reg D4 %7.2f us %6.0f GB/s | reg D8 %7.2f us %6.0f GB/s\n",
                   nw, wpc, L, t4, bytes / t4 / 1e3, t8, t8 > 0 ? bytes / t8 / 1e3 : 0, r4, bytes / r4 / 1e3, r8, bytes / r8 / 1e3);
        }
    }
    // per-CU limit: only `c` CUs stream (one 16-wave WG each, register loads, D=4)
    for (int c : {32, 64, 128, 192, 256}) {
        const long waves = (long)c * 16;
        const int L = (int)((nblocks + waves - 1) / waves);
        float r = timeit([&](int i) { k_reg<4><<<c, 1024>>>(bufs[i % copies], nblocks, L, out); }, reps);
        float r8 = timeit([&](int i) { k_reg<8><<<c, 1024>>>(bufs[i % copies], nblocks, L, out); }, reps);
        printf("cus=%3d waves/cu=16 L=%4d reg D4 %7.2f us %6.0f GB/s (%5.1f GB/s/CU) | D8 %7.2f us %6.0f GB/s\n", c, L, r,
               bytes / r / 1e3, bytes / r / 1e3 / c, r8, bytes / r8 / 1e3);
    }
    // plain copy for reference (reads + writes)
    v4i *dst;
    CK(hipMalloc(&dst, bytes));
    float tc = timeit([&](int i) { k_copy<<<4096, 256>>>((const v4i *)bufs[i % copies], dst, bytes / 16); }, reps);
    printf("copy: %7.2f us  %6.0f GB/s (read+write)\n", tc, 2.0 * bytes / tc / 1e3);
    float te = timeit([&](int i) { k_reg<4><<<1, 64>>>(bufs[0], 0, 1, out); }, reps);
    printf("empty launch: %7.2f us\n", te);
    return 0;
}
