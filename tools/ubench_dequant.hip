// ubench_dequant.hip -- development microbenchmark: the prefill inner block (int8 MFMA + the
// per-group dequant of the reference's epilogue: cvt_f32_i32 + fma_mix with the fp16 scale
// product) on registers only, to find the issue ceiling of each formulation (cycles per MFMA per
// SIMD) at 1 and 2 waves per SIMD.  Not part of the product.
// build: hipcc -O3 --offload-arch=gfx950 -fno-slp-vectorize tools/ubench_dequant.hip -o /tmp/ubd
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v2f __attribute__((ext_vector_type(2)));
typedef int v2i_ __attribute__((ext_vector_type(2)));

template <int MODE, int W>  // 0: MFMA only, 1: 16x16x64 + dequant, 2: 32x32x32 + dequant
__global__ __launch_bounds__(64 * W) void kern(int iters, long long *cyc, float *sink) {
    extern __shared__ char lds[];  // sized by the launch to force one block per CU
    const int lane = threadIdx.x & 63;
    v4i a[4][2], b[4][2];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int s = 0; s < 2; s++) {
            a[i][s] = v4i{lane * 3 + i, lane + s, lane ^ i, 7 * lane};
            b[i][s] = v4i{lane ^ 9, lane * 5 + s, i + lane, lane};
        }
    uint32_t xv[4], wv[4][2];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        xv[i] = 0x3c003c00u + lane + i;
        wv[i][0] = 0x2c002c00u + lane * i;
        wv[i][1] = 0x2c012c01u + lane * i;
    }
    float out[4][4][4];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 4; j++)
#pragma unroll
            for (int r = 0; r < 4; r++) out[i][j][r] = 0.f;
    v16i acc32[2][2];
    float (*out32)[2][16] = reinterpret_cast<float (*)[2][16]>(&out[0][0][0]);  // the same 64 registers
    long long t0 = clock64();
    for (int it = 0; it < iters; it++) {
        asm volatile("" : "+v"(a[0][0]), "+v"(b[0][0]), "+v"(xv[0]), "+v"(wv[0][0]));
        if (MODE >= 10) {  // every scale operand loop-variant (nothing hoisted out of the loop)
#pragma unroll
            for (int i = 0; i < 4; i++) asm volatile("" : "+v"(xv[i]), "+v"(wv[i][0]), "+v"(wv[i][1]));
        }
        if (MODE == 0) {
#pragma unroll
            for (int mi = 0; mi < 4; mi++)
#pragma unroll
                for (int ni = 0; ni < 4; ni++) {
                    v4i acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[ni][0], a[mi][0], v4i{0, 0, 0, 0}, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[ni][1], a[mi][1], acc, 0, 0, 0);
                    out[mi][ni][0] += __int_as_float(acc[0] ^ acc[3]);
                }
        } else if (MODE == 1 || MODE == 13) {
#pragma unroll
            for (int mi = 0; mi < 4; mi++) {
                const uint32_t x2u = __builtin_amdgcn_perm(xv[mi], xv[mi], 0x01000100u);
                const __half2 x2 = *reinterpret_cast<const __half2 *>(&x2u);
#pragma unroll
                for (int ni = 0; ni < 4; ni++) {
                    v4i acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[ni][0], a[mi][0], v4i{0, 0, 0, 0}, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[ni][1], a[mi][1], acc, 0, 0, 0);
                    const uint32_t w01 = wv[ni][0], w23 = wv[ni][1];
                    const __half2 p01 = __hmul2(*reinterpret_cast<const __half2 *>(&w01), x2);
                    const __half2 p23 = __hmul2(*reinterpret_cast<const __half2 *>(&w23), x2);
                    float *o = out[mi][ni];
                    o[0] = fmaf((float)acc[0], __low2float(p01), o[0]);
                    o[1] = fmaf((float)acc[1], __high2float(p01), o[1]);
                    o[2] = fmaf((float)acc[2], __low2float(p23), o[2]);
                    o[3] = fmaf((float)acc[3], __high2float(p23), o[3]);
                }
            }
        } else if (MODE == 10) {
            // 10: int8 MFMA seeded with the bits of 1.5 * 2^23, so the accumulator reads as the fp32
            // 12582912 + acc (exact for |acc| < 2^22); one scalar v_sub_f32 per output replaces the cvt
#pragma unroll
            for (int mi = 0; mi < 4; mi++) {
                const uint32_t x2u = __builtin_amdgcn_perm(xv[mi], xv[mi], 0x01000100u);
                const __half2 x2 = *reinterpret_cast<const __half2 *>(&x2u);
#pragma unroll
                for (int ni = 0; ni < 4; ni++) {
                    const int B = 0x4B400000;
                    v4i acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[ni][0], a[mi][0], v4i{B, B, B, B}, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[ni][1], a[mi][1], acc, 0, 0, 0);
                    const uint32_t w01 = wv[ni][0], w23 = wv[ni][1];
                    const __half2 p01 = __hmul2(*reinterpret_cast<const __half2 *>(&w01), x2);
                    const __half2 p23 = __hmul2(*reinterpret_cast<const __half2 *>(&w23), x2);
                    float *o = out[mi][ni];
                    o[0] = fmaf(__int_as_float(acc[0]) - 12582912.0f, __low2float(p01), o[0]);
                    o[1] = fmaf(__int_as_float(acc[1]) - 12582912.0f, __high2float(p01), o[1]);
                    o[2] = fmaf(__int_as_float(acc[2]) - 12582912.0f, __low2float(p23), o[2]);
                    o[3] = fmaf(__int_as_float(acc[3]) - 12582912.0f, __high2float(p23), o[3]);
                }
            }
        } else if (MODE == 11 || MODE == 12) {
            // 11: mode 10 with the bias removed by packed v_pk_add_f32 (two outputs per instruction):
            // per 16x16 block 2 pk_add + 2 pk_mul + 4 fma_mix = 4 VALU per MFMA instead of 5.
            // 12: the same, software-pipelined as mode 6 (block b's MFMAs, then block b - 1's dequant)
            const int B = 0x4B400000;
            const v2f nb = v2f{-12582912.0f, -12582912.0f};
            auto deq = [&](const v4i acc, int pm, int pn) {
                const uint32_t x2u = __builtin_amdgcn_perm(xv[pm], xv[pm], 0x01000100u);
                const __half2 x2 = *reinterpret_cast<const __half2 *>(&x2u);
                const uint32_t w01 = wv[pn][0], w23 = wv[pn][1];
                const __half2 p01 = __hmul2(*reinterpret_cast<const __half2 *>(&w01), x2);
                const __half2 p23 = __hmul2(*reinterpret_cast<const __half2 *>(&w23), x2);
                v2f f01 = __builtin_bit_cast(v2f, v2i_{acc[0], acc[1]});
                v2f f23 = __builtin_bit_cast(v2f, v2i_{acc[2], acc[3]});
                asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(f01) : "v"(nb));
                asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(f23) : "v"(nb));
                float *o = out[pm][pn];
                const uint32_t q01 = __builtin_bit_cast(uint32_t, p01), q23 = __builtin_bit_cast(uint32_t, p23);
                asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[0,1,0]" : "+v"(o[0]) : "v"(f01[0]), "v"(q01));
                asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel:[0,1,0] op_sel_hi:[0,1,0]" : "+v"(o[1]) : "v"(f01[1]), "v"(q01));
                asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[0,1,0]" : "+v"(o[2]) : "v"(f23[0]), "v"(q23));
                asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel:[0,1,0] op_sel_hi:[0,1,0]" : "+v"(o[3]) : "v"(f23[1]), "v"(q23));
            };
            if (MODE == 11) {
#pragma unroll
                for (int mi = 0; mi < 4; mi++)
#pragma unroll
                    for (int ni = 0; ni < 4; ni++) {
                        v4i acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[ni][0], a[mi][0], v4i{B, B, B, B}, 0, 0, 0);
                        acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[ni][1], a[mi][1], acc, 0, 0, 0);
                        deq(acc, mi, ni);
                    }
            } else {
                v4i accs[2];
                accs[0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[0][0], a[0][0], v4i{B, B, B, B}, 0, 0, 0);
                accs[0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[0][1], a[0][1], accs[0], 0, 0, 0);
#pragma unroll
                for (int bl = 1; bl <= 16; bl++) {
                    const int mi = bl >> 2, ni = bl & 3;
                    if (bl < 16) {
                        accs[bl & 1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[ni][0], a[mi][0], v4i{B, B, B, B}, 0, 0, 0);
                        accs[bl & 1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[ni][1], a[mi][1], accs[bl & 1], 0, 0, 0);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    deq(accs[(bl - 1) & 1], (bl - 1) >> 2, (bl - 1) & 3);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        } else if (MODE == 8 || MODE == 9) {
            // 8: the group sums on the bf16 MFMA (int8 codes and 4w weights are exact in bf16, a
            // group's sum is exact in fp32): four 16x16x32 per 16x16x128 block, no v_cvt; then the
            // fma_mix + pk_mul dequant.  9: the bf16 MFMAs alone.
#pragma unroll
            for (int mi = 0; mi < 4; mi++) {
                const uint32_t x2u = __builtin_amdgcn_perm(xv[mi], xv[mi], 0x01000100u);
                const __half2 x2 = *reinterpret_cast<const __half2 *>(&x2u);
#pragma unroll
                for (int ni = 0; ni < 4; ni++) {
                    v4f acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, b[ni][0]), __builtin_bit_cast(v8bf, a[mi][0]), v4f{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, b[ni][1]), __builtin_bit_cast(v8bf, a[mi][1]), acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, b[ni][0]), __builtin_bit_cast(v8bf, a[mi][1]), acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, b[ni][1]), __builtin_bit_cast(v8bf, a[mi][0]), acc, 0, 0, 0);
                    float *o = out[mi][ni];
                    if (MODE == 9) {
                        o[0] += acc[0] * acc[3];
                        continue;
                    }
                    const uint32_t w01 = wv[ni][0], w23 = wv[ni][1];
                    const __half2 p01 = __hmul2(*reinterpret_cast<const __half2 *>(&w01), x2);
                    const __half2 p23 = __hmul2(*reinterpret_cast<const __half2 *>(&w23), x2);
                    o[0] = fmaf(acc[0], __low2float(p01), o[0]);
                    o[1] = fmaf(acc[1], __high2float(p01), o[1]);
                    o[2] = fmaf(acc[2], __low2float(p23), o[2]);
                    o[3] = fmaf(acc[3], __high2float(p23), o[3]);
                }
            }
        } else if (MODE == 3 || MODE == 4 || MODE == 5) {  // 3: no pk_mul, 4: no cvt, 5: neither
#pragma unroll
            for (int mi = 0; mi < 4; mi++) {
                const uint32_t x2u = __builtin_amdgcn_perm(xv[mi], xv[mi], 0x01000100u);
                const __half2 x2 = *reinterpret_cast<const __half2 *>(&x2u);
#pragma unroll
                for (int ni = 0; ni < 4; ni++) {
                    v4i acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[ni][0], a[mi][0], v4i{0, 0, 0, 0}, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[ni][1], a[mi][1], acc, 0, 0, 0);
                    uint32_t w01 = wv[ni][0], w23 = wv[ni][1];
                    __half2 p01 = *reinterpret_cast<const __half2 *>(&w01), p23 = *reinterpret_cast<const __half2 *>(&w23);
                    if (MODE == 4) {
                        p01 = __hmul2(p01, x2);
                        p23 = __hmul2(p23, x2);
                    }
                    float *o = out[mi][ni];
#define CV(v) (MODE == 3 ? (float)(v) : __int_as_float(v))
                    o[0] = fmaf(CV(acc[0]), __low2float(p01), o[0]);
                    o[1] = fmaf(CV(acc[1]), __high2float(p01), o[1]);
                    o[2] = fmaf(CV(acc[2]), __low2float(p23), o[2]);
                    o[3] = fmaf(CV(acc[3]), __high2float(p23), o[3]);
#undef CV
                }
            }
        } else if (MODE == 6) {
            // 16x16x64, software-pipelined: block b's two MFMAs are interleaved with the dequant of
            // block b - 1 (sched_group_barrier: 1 MFMA, 5 VALU, 1 MFMA, 5 VALU)
            v4i accs[2];
            accs[0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[0][0], a[0][0], v4i{0, 0, 0, 0}, 0, 0, 0);
            accs[0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[0][1], a[0][1], accs[0], 0, 0, 0);
#pragma unroll
            for (int bl = 1; bl <= 16; bl++) {
                const int mi = bl >> 2, ni = bl & 3, pm = (bl - 1) >> 2, pn = (bl - 1) & 3;
                if (bl < 16) {
                    accs[bl & 1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[ni][0], a[mi][0], v4i{0, 0, 0, 0}, 0, 0, 0);
                    accs[bl & 1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[ni][1], a[mi][1], accs[bl & 1], 0, 0, 0);
                }
                const v4i acc = accs[(bl - 1) & 1];
                const uint32_t x2u = __builtin_amdgcn_perm(xv[pm], xv[pm], 0x01000100u);
                const __half2 x2 = *reinterpret_cast<const __half2 *>(&x2u);
                const uint32_t w01 = wv[pn][0], w23 = wv[pn][1];
                const __half2 p01 = __hmul2(*reinterpret_cast<const __half2 *>(&w01), x2);
                const __half2 p23 = __hmul2(*reinterpret_cast<const __half2 *>(&w23), x2);
                float *o = out[pm][pn];
                o[0] = fmaf((float)acc[0], __low2float(p01), o[0]);
                o[1] = fmaf((float)acc[1], __high2float(p01), o[1]);
                o[2] = fmaf((float)acc[2], __low2float(p23), o[2]);
                o[3] = fmaf((float)acc[3], __high2float(p23), o[3]);
                if (bl < 16) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);
                }
            }
        } else if (MODE == 7) {
            // 32x32x32 pipelined: the 4 MFMAs of block (mi, ni) interleaved with the dequant of the
            // previous block (16 outputs: 16 cvt + 16 fma_mix + 8 pk_mul = 40 VALU, 10 per MFMA)
            v16i accs[2];
            auto mm = [&](int q, v16i c) {
                const int mi = q >> 1, ni = q & 1;
                c = __builtin_amdgcn_mfma_i32_32x32x32_i8(b[2 * ni][0], a[2 * mi][0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_i32_32x32x32_i8(b[2 * ni][1], a[2 * mi][1], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_i32_32x32x32_i8(b[2 * ni + 1][0], a[2 * mi + 1][0], c, 0, 0, 0);
                return __builtin_amdgcn_mfma_i32_32x32x32_i8(b[2 * ni + 1][1], a[2 * mi + 1][1], c, 0, 0, 0);
            };
            accs[0] = mm(0, v16i{});
#pragma unroll
            for (int q = 1; q <= 4; q++) {
                if (q < 4) accs[q & 1] = mm(q, v16i{});
                const int pm = (q - 1) >> 1, pn = (q - 1) & 1;
                const v16i acc = accs[(q - 1) & 1];
                const uint32_t x2u = __builtin_amdgcn_perm(xv[pm], xv[pm], 0x01000100u);
                const __half2 x2 = *reinterpret_cast<const __half2 *>(&x2u);
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const uint32_t w01 = wv[2 * pn + (r >> 1)][r & 1], w23 = wv[2 * pn + (r >> 1)][(r & 1) ^ 1];
                    const __half2 p01 = __hmul2(*reinterpret_cast<const __half2 *>(&w01), x2);
                    const __half2 p23 = __hmul2(*reinterpret_cast<const __half2 *>(&w23), x2);
                    float *o = &out32[pm][pn][4 * r];
                    o[0] = fmaf((float)acc[4 * r + 0], __low2float(p01), o[0]);
                    o[1] = fmaf((float)acc[4 * r + 1], __high2float(p01), o[1]);
                    o[2] = fmaf((float)acc[4 * r + 2], __low2float(p23), o[2]);
                    o[3] = fmaf((float)acc[4 * r + 3], __high2float(p23), o[3]);
                }
                if (q < 4)
                    for (int k = 0; k < 4; k++) {
                        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                        __builtin_amdgcn_sched_group_barrier(0x002, 10, 0);
                    }
            }
        } else {
            // 32x32x32: a wave tile of 64x64 = 2x2 blocks; k = 128 = 4 MFMAs per block
#pragma unroll
            for (int mi = 0; mi < 2; mi++)
#pragma unroll
                for (int ni = 0; ni < 2; ni++) {
                    v16i acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(b[2 * ni][0], a[2 * mi][0], v16i{}, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(b[2 * ni][1], a[2 * mi][1], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(b[2 * ni + 1][0], a[2 * mi + 1][0], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(b[2 * ni + 1][1], a[2 * mi + 1][1], acc, 0, 0, 0);
                    acc32[mi][ni] = acc;
                }
#pragma unroll
            for (int mi = 0; mi < 2; mi++) {
                const uint32_t x2u = __builtin_amdgcn_perm(xv[mi], xv[mi], 0x01000100u);
                const __half2 x2 = *reinterpret_cast<const __half2 *>(&x2u);
#pragma unroll
                for (int ni = 0; ni < 2; ni++)
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const uint32_t w01 = wv[2 * ni + (q >> 1)][q & 1], w23 = wv[2 * ni + (q >> 1)][(q & 1) ^ 1];
                        const __half2 p01 = __hmul2(*reinterpret_cast<const __half2 *>(&w01), x2);
                        const __half2 p23 = __hmul2(*reinterpret_cast<const __half2 *>(&w23), x2);
                        float *o = &out32[mi][ni][4 * q];
                        o[0] = fmaf((float)acc32[mi][ni][4 * q + 0], __low2float(p01), o[0]);
                        o[1] = fmaf((float)acc32[mi][ni][4 * q + 1], __high2float(p01), o[1]);
                        o[2] = fmaf((float)acc32[mi][ni][4 * q + 2], __low2float(p23), o[2]);
                        o[3] = fmaf((float)acc32[mi][ni][4 * q + 3], __high2float(p23), o[3]);
                    }
            }
        }
    }
    long long t1 = clock64();
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 4; j++)
#pragma unroll
            for (int r = 0; r < 4; r++) s += out[i][j][r];
    if (s == 1234.5f) sink[blockIdx.x] = s + lds[0];
    if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <int MODE, int waves>
static void run(const char *name) {
    long long *cyc;
    float *sink;
    hipMalloc(&cyc, 8);
    hipMalloc(&sink, 4096 * 4);
    const int iters = 2000;
    hipFuncSetAttribute((const void *)kern<MODE, waves>, hipFuncAttributeMaxDynamicSharedMemorySize, 100 * 1024);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 2; rep++) {
        hipEventRecord(e0);
        hipLaunchKernelGGL((kern<MODE, waves>), dim3(256), dim3(64 * waves), 100 * 1024, 0, iters, cyc, sink);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
    }
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    long long c;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    const int mfma_per_iter = (MODE == 2 || MODE == 7) ? 16 : 32;  // (modes 3-5: 16x16 like 1)            // per wave
    const double macs = (double)256 * waves * iters * 16 * 16 * 128 * 16;  // 16 blocks of 16x16x128 (or 4 of 32x32x128)
    const double wps = waves / 4.0;                            // waves per SIMD
    printf("%-28s waves/SIMD=%.0f  cycles/iter/wave=%7.1f  SIMD cycles per 16x16x128 block=%6.1f (ideal 32)  TOPS=%7.1f\n",
           name, wps, (double)c / iters, (double)c / iters / (16 * wps), 2 * macs / (ms * 1e-3) / 1e12);
    (void)mfma_per_iter;
}

int main() {
    run<9, 8>("bf16 16x16x32 mfma only");
    run<8, 8>("bf16 16x16x32 + dequant");
    run<1, 8>("16x16x64 + dequant");
    run<9, 4>("bf16 16x16x32 mfma only");
    run<8, 4>("bf16 16x16x32 + dequant");
    run<1, 4>("16x16x64 + dequant");
    run<10, 8>("16x16x64 biased + sub");
    run<10, 4>("16x16x64 biased + sub");
    if (getenv("UBD_PK_ONLY")) {
        run<1, 8>("16x16x64 + dequant");
        run<13, 8>("16x16x64 + dequant, no hoist");
        run<10, 8>("16x16x64 biased + sub");
        run<11, 8>("16x16x64 biased + pk_add");
        run<12, 8>("16x16x64 biased + pk_add, pipelined");
        run<6, 8>("16x16 pipelined");
        run<1, 4>("16x16x64 + dequant");
        run<11, 4>("16x16x64 biased + pk_add");
        run<12, 4>("16x16x64 biased + pk_add, pipelined");
        run<0, 8>("mfma only 16x16x64");
        return 0;
    }
    if (getenv("UBD_BF16_ONLY")) return 0;
    run<6, 4>("16x16 pipelined");
    run<7, 4>("32x32 pipelined");
    run<6, 8>("16x16 pipelined");
    run<7, 8>("32x32 pipelined");
    run<0, 16>("mfma only 16x16x64");
    run<1, 16>("16x16x64 + dequant");
    run<2, 16>("32x32x32 + dequant");
    run<6, 16>("16x16 pipelined");
    run<7, 16>("32x32 pipelined");
    run<0, 4>("mfma only 16x16x64");
    run<1, 4>("16x16x64 + dequant");
    run<2, 4>("32x32x32 + dequant");
    run<0, 8>("mfma only 16x16x64");
    run<1, 8>("16x16x64 + dequant");
    run<2, 8>("32x32x32 + dequant");
    run<3, 8>("16x16: cvt + fma_mix (no pk_mul)");
    run<4, 8>("16x16: fma_mix + pk_mul (no cvt)");
    run<5, 8>("16x16: fma_mix only");
    return 0;
}
