// ubench_valu.hip -- development microbenchmark: SIMD cycles per wave64 VALU instruction, by opcode,
// for 1 and 2 waves per SIMD (one 256- or 512-thread workgroup per CU, forced by its LDS size).
// Each iteration issues 64 independent instances of one opcode over 16 accumulator registers
// (four passes of 16, so no instruction reads a result of the last three).  Not part of the product.
// build: hipcc -O3 --offload-arch=gfx950 tools/ubench_valu.hip -o /tmp/ubv
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define REP16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

template <int OP>
__device__ __forceinline__ void body(float (&r)[16], float s, float t) {
    // every form reads r[i] and writes r[i]; s, t loop-invariant sources
#define F(i)                                                                                                  \
    if (OP == 0) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(s), "v"(t));                      \
    if (OP == 1) asm volatile("v_fma_mix_f32 %0, %0, %1, %2 op_sel_hi:[0,1,0]" : "+v"(r[i]) : "v"(s), "v"(t)); \
    if (OP == 2) asm volatile("v_cvt_f32_i32 %0, %0" : "+v"(r[i]));                                           \
    if (OP == 3) asm volatile("v_pk_mul_f16 %0, %0, %1" : "+v"(r[i]) : "v"(s));                               \
    if (OP == 4) asm volatile("v_sub_f32 %0, %0, %1" : "+v"(r[i]) : "v"(s));                                  \
    if (OP == 5) asm volatile("v_add_u32 %0, %0, %1" : "+v"(r[i]) : "v"(s));                                  \
    if (OP == 6) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(r[i]) : "v"(s));                                  \
    if (OP == 7) asm volatile("v_cvt_f32_f16 %0, %0" : "+v"(r[i]));                                           \
    if (OP == 8) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(r[i]) : "v"(s));                                  \
    if (OP == 9) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(r[i]) : "v"(s), "v"(t));                         \
    if (OP == 10) asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[0,1,0]" : "+v"(r[i]) : "v"(s), "v"(t)); \
    if (OP == 11) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(r[i]));                                          \
    if (OP == 12) asm volatile("v_pk_add_f16 %0, %0, %1" : "+v"(r[i]) : "v"(s));
    REP16(F)
#undef F
}

template <int OP>
__global__ void kern(int iters, long long *cyc, float *sink) {
    extern __shared__ char lds[];
    float r[16];
#pragma unroll
    for (int i = 0; i < 16; i++) r[i] = (float)(threadIdx.x + i) * 1e-3f;
    const float s = 1.0001f + threadIdx.x * 1e-7f, t = 1e-6f;
    __syncthreads();
    const long long t0 = clock64();
    for (int it = 0; it < iters; it++) {
        body<OP>(r, s, t);
        body<OP>(r, s, t);
        body<OP>(r, s, t);
        body<OP>(r, s, t);
    }
    const long long t1 = clock64();
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 16; i++) acc += r[i];
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 16 + threadIdx.x / 64] = t1 - t0;
    if (acc == 12345.f) sink[0] = acc + lds[0];
}

static const char *names[] = {"v_fma_f32", "v_fma_mix_f32", "v_cvt_f32_i32", "v_pk_mul_f16", "v_sub_f32",
                              "v_add_u32", "v_mul_f32", "v_cvt_f32_f16", "v_xor_b32", "v_fmac_f32",
                              "v_fma_mix_f32 (acc as C)", "v_cvt_f32_u32", "v_pk_add_f16"};

template <int OP>
static void run(int waves_per_simd) {
    const int iters = 2000, threads = 256 * waves_per_simd, nblk = 256;
    long long *cyc;
    float *sink;
    hipMalloc(&cyc, nblk * 16 * sizeof(long long));
    hipMalloc(&sink, 4);
    const size_t lds = 100 * 1024;  // one workgroup per CU
    hipLaunchKernelGGL(kern<OP>, dim3(nblk), dim3(threads), lds, 0, 10, cyc, sink);
    hipLaunchKernelGGL(kern<OP>, dim3(nblk), dim3(threads), lds, 0, iters, cyc, sink);
    hipDeviceSynchronize();
    long long h[256 * 16];
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    double sum = 0;
    const int nw = threads / 64;
    for (int b = 0; b < nblk; b++)
        for (int w = 0; w < nw; w++) sum += (double)h[b * 16 + w];
    const double per_wave = sum / (nblk * nw);
    const double insts = (double)iters * 4 * 16;  // per wave
    // cycles per instruction per SIMD: the SIMD retires waves_per_simd * insts in per_wave cycles
    printf("%-26s waves/SIMD=%d  SIMD cycles per wave64 instruction = %.2f\n", names[OP], waves_per_simd,
           per_wave / (insts * waves_per_simd));
    hipFree(cyc);
    hipFree(sink);
}

template <int OP>
static void both() {
    run<OP>(1);
    run<OP>(2);
}

int main() {
    both<0>(); both<1>(); both<2>(); both<3>(); both<4>(); both<5>(); both<6>();
    both<7>(); both<8>(); both<9>(); both<10>(); both<11>(); both<12>();
    return 0;
}
