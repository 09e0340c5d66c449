// Development micro-benchmark: cost of one quant_group16 call (fq_common.h) per wave, 8 waves per
// CU on every CU, data in registers.  Prints cycles per call (s_memtime) and us per call.
#include <cstdio>
#include <hip/hip_runtime.h>

#include "../flexq_amd/csrc/fq_common.h"

__global__ __launch_bounds__(512) void kq(const uint4 *in, uint2 *out, unsigned long long *t, int reps, int bits) {
    uint4 raw = in[(blockIdx.x * 512 + threadIdx.x) & 4095];
    uint2 acc = make_uint2(0, 0);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; r++) {
        uint2 c;
        const uint16_t s = quant_group16(raw, bits, c);
        acc.x ^= c.x + s;
        acc.y ^= c.y;
        raw.x ^= acc.x & 1;  // a dependency between calls
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 512 + threadIdx.x] = acc;
    if (threadIdx.x == 0) t[blockIdx.x] = t1 - t0;
}

int main() {
    const int grid = 256, reps = 64;
    uint4 *in;
    uint2 *out;
    unsigned long long *t;
    hipMalloc(&in, 4096 * 16);
    hipMalloc(&out, grid * 512 * 8);
    hipMalloc(&t, grid * 8);
    unsigned short h[4096 * 8];
    for (int i = 0; i < 4096 * 8; i++) h[i] = (unsigned short)(0x3000 + (i * 2654435761u >> 20) % 0x1000);
    hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
    for (int bits = 6; bits <= 8; bits += 2) {
        for (int it = 0; it < 3; it++) {
            hipEvent_t a, b;
            hipEventCreate(&a);
            hipEventCreate(&b);
            hipEventRecord(a);
            kq<<<grid, 512>>>(in, out, t, reps, bits);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            unsigned long long ht[grid];
            hipMemcpy(ht, t, sizeof(ht), hipMemcpyDeviceToHost);
            double avg = 0;
            for (int i = 0; i < grid; i++) avg += ht[i];
            avg /= grid;
            printf("bits %d: %.1f s_memtime ticks per call per wave (8 waves/CU), kernel %.2f us -> %.3f us per call\n",
                   bits, avg / reps, ms * 1e3, ms * 1e3 / reps);
        }
    }
    return 0;
}
