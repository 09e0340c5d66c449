/*
 * fq_oracle.c -- CPU restatement of FlexQ's W6Ax hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * This file is the parity oracle for the HIP kernels in flexq_amd/csrc.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only as the
 * checker.  Nothing in the product path links or calls it.
 *
 * Every function restates one piece of the reference (paths relative to /root/reference):
 *   fqo_pack_bitplanes     engine/src/pack/bit_packing.cu:76-133     (flexq_packing_kernel)
 *   fqo_pack_abq           engine/src/pack/bit_packing.cu:54-72      (abq_packing_kernel, KAT twin)
 *   fqo_unpack_bitplanes   inverse of the above, sign-extending as flexq_bmma_kernel.h:396-397
 *   fqo_quantize_engine    e2e/src/fastertransformer/kernels/flexqgemm/src/pack/bit_packing.cu:125-164
 *   fqo_compute_ref        engine/test_bgemm_kernel.cu:113-146        (the reference's own CPU oracle)
 *   fqo_gemm               the contract: int32 per-group accumulators (exact) dequantised with the
 *                          fp16-rounded scale product of flexq_bmma_kernel.h:360-364, summed in
 *                          double and rounded once to fp16.
 *   fqo_gemm_decode_order  the decode kernel's own fp32 summation order (S = 1): a bit-exact model of
 *                          the headline kernel's output, not a reference function.
 *   fqo_pack_fq6 / fqo_unpack_fq6   this build's own 6-bit weight image --
 *                          a model of the HIP packer, not a reference function.
 *   fqo_rmsnorm_quantize   e2e/src/fastertransformer/kernels/layernorm_kernels.cu:1851-2051
 *                          (residual + RMSNorm + quantize; the HIP kernel's summation order)
 *   fqo_silu_mul_ref       e2e/src/fastertransformer/kernels/activation_kernels.cu:133,245-450
 *                          (SiLU(gate) * up, double precision: a tolerance reference)
 *
 * Parity pinning: the reference ships no kernel golden vectors (inputs are time-seeded,
 * test_bgemm_kernel.cu:178).  The kernel-side functions are pinned by (1) the packing KAT of
 * engine/test_packing_kernel.cu:131-148 (two independent packers must agree) and (2) agreement
 * between fqo_gemm and the restated compute_ref within the reference's own tolerance.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

/* ---------------------------------------------------------------- fp16 helpers */

static float f16_to_f32(uint16_t h) {
    uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t exp = (h >> 10) & 0x1f;
    uint32_t man = h & 0x3ff;
    uint32_t bits;
    if (exp == 0) {
        if (man == 0) {
            bits = sign;
        } else { /* subnormal: renormalise */
            int e = -1;
            do { man <<= 1; e++; } while (!(man & 0x400));
            man &= 0x3ff;
            bits = sign | ((uint32_t)(127 - 15 - e) << 23) | (man << 13);
        }
    } else if (exp == 0x1f) {
        bits = sign | 0x7f800000u | (man << 13);
    } else {
        bits = sign | ((exp + 127 - 15) << 23) | (man << 13);
    }
    float f;
    memcpy(&f, &bits, 4);
    return f;
}

/* round-to-nearest-even double -> fp16 (no intermediate float, so no double rounding) */
static uint16_t f64_to_f16(double d) {
    uint16_t sign = signbit(d) ? 0x8000 : 0;
    double a = fabs(d);
    if (isnan(d)) return sign | 0x7e00;
    if (a >= 65520.0) return sign | 0x7c00; /* rounds to inf */
    if (a < 5.9604644775390625e-08 * 0.5) return sign; /* below half the min subnormal */
    int e;
    (void)frexp(a, &e); /* a = m * 2^e, m in [0.5,1) */
    /* fp16 normal range: exponent (e-1) in [-14, 15] */
    double q;
    if (e - 1 < -14) {
        /* subnormal: units of 2^-24 */
        q = a * 16777216.0; /* a / 2^-24 */
    } else {
        q = a * ldexp(1.0, 11 - e); /* 11 significant bits */
    }
    double r = nearbyint(q); /* default rounding mode = round-half-even */
    if (e - 1 < -14) {
        uint32_t v = (uint32_t)r; /* may become 0x400 = min normal, which is the correct encoding */
        return sign | (uint16_t)v;
    }
    if (r >= 2048.0) { r /= 2.0; e += 1; }
    int be = e - 1 + 15;
    if (be >= 31) return sign | 0x7c00;
    uint32_t mant = (uint32_t)r - 1024u;
    return sign | (uint16_t)((be << 10) | mant);
}

uint16_t fqo_f32_to_f16(float f) { return f64_to_f16((double)f); }
float fqo_f16_to_f32(uint16_t h) { return f16_to_f32(h); }
uint16_t fqo_f64_to_f16(double d) { return f64_to_f16(d); }

/* ---------------------------------------------------------------- bit-plane layout */

/* bit_packing.cu:75 "[k / 128, M / chunk_M, x_bits, chunk_M, 4], chunk_M = min(chunk_M, MMA_M)";
 * the index math is bit_packing.cu:121-127.  Rows R > 8 must be a multiple of 8: otherwise the
 * reference's chunk offsets overlap the next K-tile (SURVEY.md §2.2 "layout hazard"). */
static int bitplane_shape_ok(int R, int K, int bits) {
    if (R <= 0 || K <= 0 || K % 128 != 0 || bits < 1 || bits > 8) return 0;
    if (R > 8 && R % 8 != 0) return 0;
    return 1;
}

static inline size_t bitplane_index(int r, int kt32, int b, int R, int bits) {
    const int chunk = R < 8 ? R : 8;
    const int by = kt32 / 4, kw = kt32 % 4;
    return (size_t)by * ((size_t)R * bits * 4) + (size_t)(r / chunk) * (bits * chunk * 4) +
           (size_t)b * (chunk * 4) + (size_t)(r % chunk) * 4 + kw;
}

/* flexq_packing_kernel: bit b of element (r, k) goes to bit (31 - k%32) of word
 * [k/128][r/c][b][r%c][(k%128)/32] -- __brev(__ballot_sync(...)) at bit_packing.cu:109. */
int fqo_pack_bitplanes(const int32_t *in, int R, int K, int bits, int32_t *out) {
    if (!bitplane_shape_ok(R, K, bits)) return 1;
    memset(out, 0, (size_t)bits * R * (K / 32) * sizeof(int32_t));
    for (int r = 0; r < R; r++)
        for (int kt = 0; kt < K / 32; kt++)
            for (int b = 0; b < bits; b++) {
                uint32_t word = 0;
                for (int j = 0; j < 32; j++) {
                    uint32_t bit = ((uint32_t)in[(size_t)r * K + kt * 32 + j] >> b) & 1u;
                    word |= bit << (31 - j);
                }
                out[bitplane_index(r, kt, b, R, bits)] = (int32_t)word;
            }
    return 0;
}

/* Inverse: two's complement value, MSB plane weighted -2^(bits-1) (flexq_bmma_kernel.h:396-397,
 * test_bgemm_kernel.cu:123-127). */
int fqo_unpack_bitplanes(const int32_t *packed, int R, int K, int bits, int32_t *out) {
    if (!bitplane_shape_ok(R, K, bits)) return 1;
    for (int r = 0; r < R; r++)
        for (int kt = 0; kt < K / 32; kt++)
            for (int j = 0; j < 32; j++) {
                int32_t v = 0;
                for (int b = 0; b < bits; b++) {
                    uint32_t word = (uint32_t)packed[bitplane_index(r, kt, b, R, bits)];
                    int32_t bit = (word >> (31 - j)) & 1;
                    v += (b == bits - 1) ? -(bit << b) : (bit << b);
                }
                out[(size_t)r * K + kt * 32 + j] = v;
            }
    return 0;
}

/* abq_packing_kernel (bit_packing.cu:54-72): layout [bits][R][K/32], same MSB-first order.
 * Used only by the packing known-answer test (test_packing_kernel.cu:131-148). */
int fqo_pack_abq(const int32_t *in, int R, int K, int bits, uint32_t *out) {
    if (R <= 0 || K % 32 != 0) return 1;
    const size_t L = (size_t)R * (K / 32);
    for (int b = 0; b < bits; b++)
        for (size_t idx = 0; idx < L; idx++) {
            uint32_t v = 0;
            for (int i = 0; i < 32; i++) v |= (((uint32_t)in[idx * 32 + i] >> b) & 1u) << (31 - i);
            out[(size_t)b * L + idx] = v;
        }
    return 0;
}

/* ---------------------------------------------------------------- dynamic quantizer (engine) */

/* roundf(): half away from zero (CUDA round(float), e2e bit_packing.cu:160). */
static float round_half_away(float v) {
    float t = truncf(v);
    if (fabsf(v - t) >= 0.5f) t += copysignf(1.0f, v);
    return t;
}

/* Restates e2e .../flexqgemm/src/pack/bit_packing.cu:125-164 for one (row, 128-group):
 *   maxv_h = max(-1, |x|) in fp16 (exact);  maxv = float(maxv_h) / (2^(b-1)-1)  [fp32 IEEE div]
 *   scale_h = half(maxv) [RN];  q = clamp((int)roundf(float(x) / float(scale_h)), lo, hi)
 * The float->int conversion is CUDA's saturating cvt.rzi: NaN -> 0, +-inf -> INT_MAX/MIN, so an
 * all-zero group (0/0) quantises to 0 and a group whose scale underflows to 0 saturates.
 * Outputs: q int8 [M][K] row-major; xs fp16 [K/128][M] (this build's layout, group-major). */
int fqo_quantize_engine(const uint16_t *x, int M, int K, int bits, int8_t *q, uint16_t *xs) {
    if (M <= 0 || K <= 0 || K % 128 != 0 || (bits != 6 && bits != 8)) return 1;
    const int hi = (1 << (bits - 1)) - 1, lo = -(1 << (bits - 1));
    for (int m = 0; m < M; m++)
        for (int g = 0; g < K / 128; g++) {
            const uint16_t *xg = x + (size_t)m * K + (size_t)g * 128;
            float mx = -1.0f;
            for (int i = 0; i < 128; i++) {
                float a = fabsf(f16_to_f32(xg[i]));
                if (a > mx) mx = a; /* __hmax ignores a NaN operand */
            }
            float maxv = mx / (float)hi;
            uint16_t sh = fqo_f32_to_f16(maxv);
            float r = f16_to_f32(sh);
            xs[(size_t)g * M + m] = sh;
            for (int i = 0; i < 128; i++) {
                float v = round_half_away(f16_to_f32(xg[i]) / r);
                int qi;
                if (isnan(v)) qi = 0;
                else if (v >= (float)hi) qi = hi;
                else if (v <= (float)lo) qi = lo;
                else qi = (int)v;
                q[(size_t)m * K + (size_t)g * 128 + i] = (int8_t)qi;
            }
        }
    return 0;
}

/* ---------------------------------------------------------------- the reference's compute_ref */

/* Faithful restatement of compute_ref (test_bgemm_kernel.cu:113-146) including its arithmetic:
 * `float tmp += 1.0 * (int product) * w_scale_float * x_scale_float` -- the right-hand side is
 * evaluated in double and added to a float accumulator, bit-pair by bit-pair, k by k.
 * x_scale_dup is the reference layout half[K/128][2*ceil4(M)] (test_bgemm_kernel.cu:41-54). */
int fqo_compute_ref(const int32_t *w, const uint16_t *w_scale, const int32_t *x,
                    const uint16_t *x_scale_dup, uint16_t *ref_c, int M, int N, int K, int W_BIT,
                    int X_BIT) {
    if (!bitplane_shape_ok(M, K, X_BIT) || !bitplane_shape_ok(N, K, W_BIT)) return 1;
    const int chunk_m = M < 8 ? M : 8, chunk_n = N < 8 ? N : 8;
    const int xs_ld = 2 * ((M + 3) / 4 * 4);
    for (int m = 0; m < M; m++)
        for (int n = 0; n < N; n++) {
            float tmp = 0;
            for (int xb = 0; xb < X_BIT; xb++) {
                int xmul = (xb == X_BIT - 1) ? -(1 << xb) : (1 << xb);
                for (int wb = 0; wb < W_BIT; wb++) {
                    int wmul = (wb == W_BIT - 1) ? -(1 << wb) : (1 << wb);
                    for (int kt = 0; kt < K / 32; kt++) {
                        int w_int = w[(kt / 4) * (N * W_BIT * 4) + (n / chunk_n) * (W_BIT * chunk_n * 4) +
                                      wb * (chunk_n * 4) + (n % chunk_n) * 4 + (kt % 4)];
                        int x_int = x[(kt / 4) * (M * X_BIT * 4) + (m / chunk_m) * (X_BIT * chunk_m * 4) +
                                      xb * (chunk_m * 4) + (m % chunk_m) * 4 + (kt % 4)];
                        float wsf = f16_to_f32(w_scale[(kt / 4) * N + n]);
                        float xsf = f16_to_f32(x_scale_dup[(kt / 4) * xs_ld + 2 * m]);
                        for (int k = 0; k < 32; k++) {
                            int xv = ((1 << k) & x_int) != 0;
                            int wv = ((1 << k) & w_int) != 0;
                            tmp += 1.0 * (xmul * wmul * xv * wv) * wsf * xsf;
                        }
                    }
                }
            }
            ref_c[(size_t)m * N + n] = fqo_f32_to_f16(tmp);
        }
    return 0;
}

/* ---------------------------------------------------------------- the contract oracle */

/* D[m][n] = half( sum_g float(half(xs[g][m] * ws[g][n])) * acc[m][n][g] ),
 * acc[m][n][g] = sum_{k in group g} xq[m][k] * wq[n][k]  (exact int32).
 * The scale product is rounded to fp16 exactly like __hmul2 (flexq_bmma_kernel.h:360-364): the
 * fp32 product of two fp16 values is exact, so one RN to fp16 reproduces the hardware result.
 * The sum over groups is done in double and rounded once (the HIP kernel sums in fp32; tests
 * compare within 1e-3 relative plus an fp32-cancellation floor, see tests/common.py).
 * Optional outputs: acc [M][N][K/128] int32, mag [M][N] = sum_g |s_g * acc_g| (double). */
int fqo_gemm(const int8_t *xq, const uint16_t *xs, const int8_t *wq, const uint16_t *ws, int M, int N,
             int K, uint16_t *out, int32_t *acc_out, double *mag_out) {
    if (M <= 0 || N <= 0 || K <= 0 || K % 128 != 0) return 1;
    const int G = K / 128;
    for (int m = 0; m < M; m++)
        for (int n = 0; n < N; n++) {
            double sum = 0.0, mag = 0.0;
            for (int g = 0; g < G; g++) {
                const int8_t *xr = xq + (size_t)m * K + (size_t)g * 128;
                const int8_t *wr = wq + (size_t)n * K + (size_t)g * 128;
                int32_t a = 0;
                for (int i = 0; i < 128; i++) a += (int32_t)xr[i] * (int32_t)wr[i];
                float p = f16_to_f32(xs[(size_t)g * M + m]) * f16_to_f32(ws[(size_t)g * N + n]);
                double s = (double)f16_to_f32(fqo_f32_to_f16(p));
                sum += s * (double)a;
                mag += fabs(s * (double)a);
                if (acc_out) acc_out[((size_t)m * N + n) * G + g] = a;
            }
            out[(size_t)m * N + n] = f64_to_f16(sum);
            if (mag_out) mag_out[(size_t)m * N + n] = mag;
        }
    return 0;
}

/* The decode kernel's own fp32 summation order -- a bit-exact model of the production decode / chain
 * output for plans without a k-split (flexq_amd/csrc/fq_gemm.hip decode_body, S = 1; every LLaMA decode
 * shape at M = 1 and every chain link), so the headline's fp16 outputs can be checked bit for bit rather
 * than within a tolerance.  Not a reference function: the reference's own order (compute_ref,
 * fqo_compute_ref) differs in the last bits.  Per output (m, n): wave w of NW owns groups
 * [w*G/NW, (w+1)*G/NW) and accumulates c = fmaf(float(4 * acc_g), float(half(xs * ws)), c) from 0 in
 * group order (the MFMA sums 4*w, fq_common.h unpack_fq6); the workgroup sums the NW partials c * 0.25 in
 * wave order from 0 and rounds once to fp16. */
int fqo_gemm_decode_order(const int8_t *xq, const uint16_t *xs, const int8_t *wq, const uint16_t *ws, int M, int N,
                          int K, int NW, uint16_t *out) {
    if (M <= 0 || N <= 0 || K <= 0 || K % 128 != 0 || NW <= 0) return 1;
    const int G = K / 128;
    for (int m = 0; m < M; m++)
        for (int n = 0; n < N; n++) {
            float v = 0.0f;
            for (int w = 0; w < NW; w++) {
                float c = 0.0f;
                for (int g = (w * G) / NW; g < ((w + 1) * G) / NW; g++) {
                    const int8_t *xr = xq + (size_t)m * K + (size_t)g * 128;
                    const int8_t *wr = wq + (size_t)n * K + (size_t)g * 128;
                    int32_t a = 0;
                    for (int i = 0; i < 128; i++) a += (int32_t)xr[i] * (int32_t)wr[i];
                    const float p = f16_to_f32(fqo_f32_to_f16(f16_to_f32(xs[(size_t)g * M + m]) *
                                                              f16_to_f32(ws[(size_t)g * N + n])));
                    c = fmaf((float)(4 * a), p, c);
                }
                v = v + c * 0.25f;
            }
            out[(size_t)m * N + n] = fqo_f32_to_f16(v);
        }
    return 0;
}

/* Reference x_scale layout half[K/128][2*ceil4(M)], each scale duplicated as a half2 pair and the
 * row padding zeroed (base.h:35-39, test_bgemm_kernel.cu:41-54, e2e bit_packing.cu:152-156). */
int fqo_xs_to_ref_dup(const uint16_t *xs, int M, int K, uint16_t *dup) {
    const int ld = 2 * ((M + 3) / 4 * 4);
    for (int g = 0; g < K / 128; g++)
        for (int j = 0; j < ld; j += 2) {
            uint16_t v = (j / 2 < M) ? xs[(size_t)g * M + j / 2] : 0;
            dup[(size_t)g * ld + j] = v;
            dup[(size_t)g * ld + j + 1] = v;
        }
    return 0;
}

/* ---------------------------------------------------------------- this build's fq6 layout */

/* Model of the HIP packer's output (flexq_amd/csrc/fq_quant.hip).  Layout:
 *   uint32 [Npad/16][K/128][3 plane r][64 lane][2 kstep s],  Npad = ceil(N/16)*16 (pad cols = 0)
 *   lane l, kstep s hold column n = 16t + (l&15), k = 128g + 64s + 16(l>>4) + j, j = 0..15
 *   (the B operand of v_mfma_i32_16x16x64_i8 for k-step s);
 *   byte b of word (r, s): ((v[4r+b] & 63) << 2) | ((v[12+b] >> 2r) & 3).
 * A (16-column tile, group) block is 1.5 KiB = three 512 B planes; lane l's plane r is 8
 * contiguous bytes (both k-steps).  Unpacking (out_r = P_r & 0xFCFCFCFC, out_3 = sum_r
 * (P_r & 0x03030303) << (2r+2)) yields 4*v as int8: the MFMA B operand scaled by 4.
 * The image ends with the group scales blocked the same way: fp16 [Npad/16][K/128][16] at byte
 * offset Npad/16 * K/128 * 1536 (pad columns 0), 32 contiguous bytes per block. */
size_t fqo_fq6_bytes(int N, int K) { return (size_t)((N + 15) / 16) * (K / 128) * (1536 + 32); }

static inline size_t fq6_scale_index(int t, int g, int c, int G) { return ((size_t)t * G + g) * 16 + c; }

static inline size_t fq6_word(int t, int g, int r, int l, int s, int G) {
    return ((((size_t)t * G + g) * 3 + r) * 64 + l) * 2 + s;
}

static inline int fq6_col(int t, int l) { return 16 * t + (l & 15); }
static inline int fq6_k(int g, int s, int l, int j) { return 128 * g + 64 * s + 16 * (l >> 4) + j; }

int fqo_pack_fq6(const int8_t *wq, const uint16_t *ws, int N, int K, uint8_t *out) {
    if (N <= 0 || K % 128 != 0) return 1;
    const int NT = (N + 15) / 16, G = K / 128;
    uint32_t *o = (uint32_t *)out;
    uint16_t *sc = (uint16_t *)(out + (size_t)NT * G * 1536);
    memset(out, 0, fqo_fq6_bytes(N, K));
    for (int t = 0; t < NT; t++)
        for (int g = 0; g < G; g++)
            for (int c = 0; c < 16; c++)
                if (16 * t + c < N) sc[fq6_scale_index(t, g, c, G)] = ws[(size_t)g * N + 16 * t + c];
    for (int t = 0; t < NT; t++)
        for (int g = 0; g < G; g++)
            for (int s = 0; s < 2; s++)
                for (int l = 0; l < 64; l++) {
                    int n = fq6_col(t, l);
                    int v[16];
                    for (int j = 0; j < 16; j++) v[j] = (n < N) ? wq[(size_t)n * K + fq6_k(g, s, l, j)] : 0;
                    for (int r = 0; r < 3; r++) {
                        uint32_t w = 0;
                        for (int b = 0; b < 4; b++)
                            w |= (uint32_t)((((unsigned)v[4 * r + b] & 63u) << 2) |
                                            (((unsigned)v[12 + b] >> (2 * r)) & 3u)) << (8 * b);
                        o[fq6_word(t, g, r, l, s, G)] = w;
                    }
                }
    return 0;
}

int fqo_unpack_fq6(const uint8_t *packed, int N, int K, int8_t *wq, uint16_t *ws) {
    if (N <= 0 || K % 128 != 0) return 1;
    const int NT = (N + 15) / 16, G = K / 128;
    const uint32_t *p = (const uint32_t *)packed;
    const uint16_t *sc = (const uint16_t *)(packed + (size_t)NT * G * 1536);
    if (ws)
        for (int g = 0; g < G; g++)
            for (int n = 0; n < N; n++) ws[(size_t)g * N + n] = sc[fq6_scale_index(n / 16, g, n % 16, G)];
    for (int t = 0; t < NT; t++)
        for (int g = 0; g < G; g++)
            for (int s = 0; s < 2; s++)
                for (int l = 0; l < 64; l++) {
                    int n = fq6_col(t, l);
                    if (n >= N) continue;
                    uint32_t w[3];
                    for (int r = 0; r < 3; r++) w[r] = p[fq6_word(t, g, r, l, s, G)];
                    for (int j = 0; j < 16; j++) {
                        unsigned u;
                        if (j < 12) {
                            u = ((w[j / 4] >> (8 * (j % 4))) & 0xffu) >> 2;
                        } else {
                            int b = j - 12;
                            u = 0;
                            for (int r = 0; r < 3; r++) u |= ((w[r] >> (8 * b)) & 3u) << (2 * r);
                        }
                        wq[(size_t)n * K + fq6_k(g, s, l, j)] = (int8_t)((int)(u << 26) >> 26);
                    }
                }
    return 0;
}

/* ------------------------------------------------------------- quantizer arithmetic checks */
/* The HIP quantizer computes maxv = absmax / hi as a Newton-corrected product with the
 * correctly rounded constant y = RN(1/hi) (flexq_amd/csrc/fq_common.h quant_group16):
 *   q1 = RN(a * y);  r = fma(-q1, hi, a);  q = isfinite(q1) ? fma(r, y, q1) : q1.
 * Returns how many of the 65536 fp16 bit patterns a (as float, |a|), plus the absmax seed -1,
 * give q != RN(a / hi) (bitwise; NaN compares equal to NaN).  Test infrastructure only. */
long fqo_check_div_by_const(int hi) {
    const float fhi = (float)hi;
    const float y = (float)(1.0 / (double)hi);
    long bad = 0;
    for (int u = 0; u <= 65536; u++) {
        float a = u < 65536 ? fabsf(fqo_f16_to_f32((uint16_t)u)) : -1.0f;
        volatile float ref = a / fhi;
        float q1 = a * y;
        float r = fmaf(-q1, fhi, a);
        float q = isfinite(q1) ? fmaf(r, y, q1) : q1;
        if (isnan(ref) && isnan(q)) continue;
        uint32_t b0, b1;
        memcpy(&b0, (const void *)&ref, 4);
        memcpy(&b1, &q, 4);
        if (b0 != b1) bad++;
    }
    return bad;
}

/* The device quantizer's element step (flexq_amd/csrc/fq_common.h quant_group16): instead of the
 * IEEE quotient RN(x / s) rounded half away from zero, one fused multiply-add
 *     t = RN(x * rcb + copysign(0.5, x)),  rcb = RN(rc * (1 + 2^-20)),  rc = v_rcp_f32(s) (1 ulp),
 * truncated by v_cvt_i32_f32 (NaN -> 0, saturating) and clamped to [lo, hi].  x and s are fp16, so
 * a quotient that is not an exact tie k + 0.5 lies well beyond the reciprocal's error from one,
 * and the 2^-20 bias carries an exact tie across the truncation boundary.  This checks the claim
 * exhaustively: every fp16 absmax a (0 .. inf), s = half(a / hi) as the engine forms it, the
 * reciprocal rounded to nearest and moved by rc_ulp units in the last place, and every fp16 x
 * with |x| <= a or x NaN.  Returns the number of codes that differ from the reference's.
 * Test infrastructure only. */
static int cvt_i32_sat_f(float v) {
    if (isnan(v)) return 0;
    if (v >= 2147483648.0f) return 2147483647;
    if (v <= -2147483648.0f) return (int)0x80000000u;
    return (int)v; /* truncation */
}
long fqo_check_quant_fma(int bits, int rc_ulp) {
    const int hi = (1 << (bits - 1)) - 1, lo = -(1 << (bits - 1));
    const float bias = 1.0f + 0x1p-20f;
    long bad = 0;
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : bad)
    for (int ab = 0; ab <= 0x7c00; ab++) {
        const float a = fqo_f16_to_f32((uint16_t)ab);
        volatile float maxv = a / (float)hi;
        const float r = fqo_f16_to_f32(fqo_f32_to_f16(maxv));
        float rc = 1.0f / r;
        if (isfinite(rc) && rc != 0.0f)
            for (int k = 0; k < (rc_ulp < 0 ? -rc_ulp : rc_ulp); k++) rc = nextafterf(rc, rc_ulp < 0 ? 0.0f : INFINITY);
        volatile float rcbv = rc * bias;
        const float rcb = rcbv;
        for (int xb = 0; xb < 65536; xb++) {
            const uint16_t xa = (uint16_t)(xb & 0x7fff);
            if (xa > ab && xa <= 0x7c00) continue; /* |x| > absmax cannot occur in the group */
            const float x = fqo_f16_to_f32((uint16_t)xb);
            volatile float qv = x / r;
            const float v = round_half_away(qv);
            int ref;
            if (isnan(v)) ref = 0;
            else if (v >= (float)hi) ref = hi;
            else if (v <= (float)lo) ref = lo;
            else ref = (int)v;
            const float t = fmaf(x, rcb, copysignf(0.5f, x));
            int c = cvt_i32_sat_f(t);
            c = c < lo ? lo : (c > hi ? hi : c);
            if (c != ref) bad++;
        }
    }
    return bad;
}

/* ---------------------------------------------------------------- fused producers (§8(f)1) */

/* clamp_inf_for_half (e2e .../kernels/reduce_kernel_utils.cuh:357-361): +-(65504 - 1000), then fp16 */
static uint16_t half_clamp(float v) {
    const float c = v > 0.0f ? fminf(v, 65504.0f - 1000.0f) : fmaxf(v, -65504.0f + 1000.0f);
    return fqo_f32_to_f16(c);
}

/* Residual add + RMSNorm + quantization, restating generalAddResidualT5LayerNormFlexQFusion
 * (e2e .../kernels/layernorm_kernels.cu:1851-2051) with the arithmetic order of this build's
 * kernel (flexq_amd/csrc/fq_producers.hip), so that the comparison is bit-exact:
 *   r = half_clamp(float(in) + float(res))                                  (:1883)
 *   ss: thread t of T sums fmaf(v, v, acc) over its chunks c*T+t of 8 values in order; a 64-lane
 *       xor butterfly (1, 2, ..., 32: fq_common.h wave_sum64); the T/64 waves added in order.  T = 256, 512 or 1024 as
 *       the row has <= 256, <= 512 or more chunks (the kernel's workgroup size)
 *   rs = 1 / sqrt(ss / K + eps)        (the reference: rsqrtf, :1890)
 *   normed = half_clamp((float(r) * rs) * float(gamma))                     (:1898)
 *   codes/scales = fqo_quantize_engine(normed)   (the reference quantizes with the same rule, :1932-1990)
 * input may be NULL (no residual add).  residual is updated in place. */
int fqo_rmsnorm_quantize(const uint16_t *input, uint16_t *residual, const uint16_t *gamma, float eps,
                         int M, int K, int bits, int8_t *xq, uint16_t *xs, uint16_t *normed) {
    if (M <= 0 || K <= 0 || K % 128 || (bits != 6 && bits != 8)) return 1;
    const int nq = K / 8, T = nq <= 256 ? 256 : nq <= 512 ? 512 : 1024;
    float *acc = (float *)malloc(sizeof(float) * T);
    if (!acc) return 2;
    for (int m = 0; m < M; m++) {
        uint16_t *res = residual + (size_t)m * K;
        for (int t = 0; t < T; t++) acc[t] = 0.0f;
        for (int c = 0; c * T < nq; c++)
            for (int t = 0; t < T; t++) {
                const int q = c * T + t;
                if (q >= nq) continue;
                for (int e = 0; e < 8; e++) {
                    const size_t k = 8 * (size_t)q + e;
                    if (input) res[k] = half_clamp(f16_to_f32(input[(size_t)m * K + k]) + f16_to_f32(res[k]));
                    const float v = f16_to_f32(res[k]);
                    acc[t] = fmaf(v, v, acc[t]);
                }
            }
        float wsum[16];
        for (int w = 0; w < T / 64; w++) {
            float lane[64];
            for (int l = 0; l < 64; l++) lane[l] = acc[64 * w + l];
            for (int off = 1; off <= 32; off <<= 1) {
                float nxt[64];
                for (int l = 0; l < 64; l++) nxt[l] = lane[l] + lane[l ^ off];
                memcpy(lane, nxt, sizeof(lane));
            }
            wsum[w] = lane[0];
        }
        float ss = wsum[0];
        for (int w = 1; w < T / 64; w++) ss = ss + wsum[w];
        const float rs = 1.0f / sqrtf(ss / (float)K + eps);
        for (int k = 0; k < K; k++) {
            const float p = f16_to_f32(res[k]) * rs;
            normed[(size_t)m * K + k] = half_clamp(p * f16_to_f32(gamma[k]));
        }
    }
    free(acc);
    return fqo_quantize_engine(normed, M, K, bits, xq, xs);
}

/* 64-lane xor butterfly (offsets 1 .. 32) of one wave's values, then the waves in order: the bits of
 * the kernels' wave_sum64 + cross-wave sum (flexq_amd/csrc/fq_common.h) */
static float block_sum(const float *acc, int T) {
    float total = 0.0f;
    for (int w = 0; w < T / 64; w++) {
        float lane[64];
        for (int l = 0; l < 64; l++) lane[l] = acc[64 * w + l];
        for (int off = 1; off <= 32; off <<= 1) {
            float nxt[64];
            for (int l = 0; l < 64; l++) nxt[l] = lane[l] + lane[l ^ off];
            memcpy(lane, nxt, sizeof(lane));
        }
        total = w == 0 ? lane[0] : total + lane[0];
    }
    return total;
}

/* OPT-family residual + bias + LayerNorm + quantization, restating
 * generalAddBiasResidualLayerNormOpt2FlexQFusion (e2e .../kernels/layernorm_kernels.cu:316-575) with
 * this build's fixed summation order (flexq_amd/csrc/fq_common.h ln_add8 .. ln_apply8):
 *   v = ((0 + bias) + residual) + input in fp32, absent terms skipped (:357-385); h = half(v) is the
 *   residual output (:393-395); per half2 pair s += v0 + v1, q += v0*v0 + v1*v1 (:396-397), per thread
 *   over its 8-value chunks c*T + t in order, then block_sum; mean = (s / (K/2)) / 2,
 *   rs = 1 / sqrt(((q / (K/2)) / 2 - mean*mean) + eps) (:403-404, IEEE for rsqrtf);
 *   normed = ((h - half(mean)) * half(rs)) * gamma [+ beta], each an fp16 operation (:412-416);
 *   then the engine quantizer (:447-507).
 * input, bias, beta may be NULL; res_out (may be NULL) receives h. */
int fqo_layernorm_quantize(const uint16_t *input, const uint16_t *residual, const uint16_t *bias,
                           uint16_t *res_out, const uint16_t *gamma, const uint16_t *beta, float eps, int M,
                           int K, int bits, int8_t *xq, uint16_t *xs, uint16_t *normed) {
    if (M <= 0 || K <= 0 || K % 128 || (bits != 6 && bits != 8)) return 1;
    const int nq = K / 8, T = nq <= 256 ? 256 : nq <= 512 ? 512 : 1024;
    float *sacc = (float *)malloc(sizeof(float) * T), *qacc = (float *)malloc(sizeof(float) * T);
    uint16_t *h = (uint16_t *)malloc(sizeof(uint16_t) * K);
    if (!sacc || !qacc || !h) return 2;
    for (int m = 0; m < M; m++) {
        const size_t row = (size_t)m * K;
        for (int t = 0; t < T; t++) sacc[t] = qacc[t] = 0.0f;
        for (int c = 0; c * T < nq; c++)
            for (int t = 0; t < T; t++) {
                const int q = c * T + t;
                if (q >= nq) continue;
                for (int e = 0; e < 8; e += 2) {
                    float v[2];
                    for (int u = 0; u < 2; u++) {
                        const size_t k = 8 * (size_t)q + e + u;
                        float a = 0.0f;
                        if (bias) a = a + f16_to_f32(bias[k]);
                        a = a + f16_to_f32(residual[row + k]);
                        if (input) a = a + f16_to_f32(input[row + k]);
                        v[u] = a;
                        h[k] = fqo_f32_to_f16(a);
                    }
                    sacc[t] = sacc[t] + (v[0] + v[1]);
                    volatile float p0 = v[0] * v[0], p1 = v[1] * v[1];
                    qacc[t] = qacc[t] + (p0 + p1);
                }
            }
        if (res_out) memcpy(res_out + row, h, sizeof(uint16_t) * K);
        const float s = block_sum(sacc, T), qq = block_sum(qacc, T);
        const float n = (float)(K / 2);
        const float mean = (s / n) / 2.0f;
        volatile float mm = mean * mean;
        const float var = ((qq / n) / 2.0f - mm) + eps;
        const float rs = 1.0f / sqrtf(var);
        const double mh = f16_to_f32(fqo_f32_to_f16(mean)), rh = f16_to_f32(fqo_f32_to_f16(rs));
        for (int k = 0; k < K; k++) {
            double a = f16_to_f32(f64_to_f16(f16_to_f32(h[k]) - mh)); /* each step rounded to fp16 */
            a = f16_to_f32(f64_to_f16(a * rh));
            uint16_t o = f64_to_f16(a * f16_to_f32(gamma[k]));
            if (beta) o = f64_to_f16((double)f16_to_f32(o) + f16_to_f32(beta[k]));
            normed[row + k] = o;
        }
    }
    free(sacc);
    free(qacc);
    free(h);
    return fqo_quantize_engine(normed, M, K, bits, xq, xs);
}

/* SiLU(gate) * up in double precision, rounded once to fp16 (the tolerance reference of
 * flexq_generic_activation, e2e .../kernels/activation_kernels.cu:133,300; the kernels compute
 * it in fp32 with a fast exp, so they may differ by one fp16 ulp). gate/up rows stride ld. */
int fqo_silu_mul_ref(const uint16_t *gate, const uint16_t *up, int ld, int M, int N, uint16_t *act) {
    if (M <= 0 || N <= 0 || ld < N) return 1;
    for (int m = 0; m < M; m++)
        for (int n = 0; n < N; n++) {
            const double g = f16_to_f32(gate[(size_t)m * ld + n]), u = f16_to_f32(up[(size_t)m * ld + n]);
            act[(size_t)m * N + n] = fqo_f64_to_f16(g / (1.0 + exp(-g)) * u);
        }
    return 0;
}
