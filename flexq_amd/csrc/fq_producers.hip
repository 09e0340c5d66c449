// fq_producers.hip -- fused producers of the GEMM's quantized activations.
//
// The reference's serving path feeds its W6Ax GEMMs from fused "normalise/activate -> dynamic
// quantize -> bit-pack" kernels:
//   * residual add + T5/LLaMA RMSNorm + 6-bit pack: generalAddResidualT5LayerNormFlexQFusion
//     (e2e .../kernels/layernorm_kernels.cu:1851-2051; launch :2053-2106);
//   * SiLU(gate) * up + 6/8-bit pack for down_proj: flexq_generic_activation
//     (e2e .../kernels/activation_kernels.cu:245-450; launch :556-590).
// Here they produce this engine's activation format (int8 codes [M][K] + fp16 group scales
// [K/128][M], the input of fq_gemm_w6ax) with the engine quantizer's exact arithmetic
// (quant_group16, fq_common.h), and optionally the fp16 activations themselves.
//
// Design: the reference quantizes in a second phase that reads values other blocks are still
// writing (only blockIdx.y == 0 normalises the row, layernorm_kernels.cu:1879-1930 vs :1932;
// activation_kernels.cu:321-372 after a block-local __syncthreads): a cross-block race.  Here a
// workgroup owns whole 128-groups end to end, so the values it quantizes are its own registers.
//   * RMSNorm: one WG per row (a row-wide sum of squares) of T = 256, 512 or 1024 threads as the
//     row has <= 256, <= 512 or more chunks of 8 values (decode rows are latency-bound: more
//     threads, fewer serial chunks); each thread keeps its chunks and their gamma values in
//     registers between the two passes (K <= 32768).
//   * SiLU * up: elementwise, one 8-value chunk per thread, 16 threads per group.
// Both are HBM-bound streaming kernels: RMSNorm reads 4 B and writes 3-5 B per element, SiLU
// reads 4 B and writes 1-3 B.
//
// Arithmetic (the oracle, oracle/fq_oracle.c fqo_rmsnorm_quantize / fqo_silu_mul, restates it):
//   r      = half_clamp(float(input) + float(residual))              (layernorm_kernels.cu:1883)
//   ss     = sum of float(r)^2: per thread fmaf over its chunks c*T + t in order, a 64-lane xor
//            butterfly (1, 2, ..., 32; wave_sum64), then the T/64 waves in order
//   rs     = 1 / sqrt(ss / K + eps)            (IEEE; the reference uses rsqrtf, :1890)
//   normed = half_clamp((float(r) * rs) * float(gamma))              (:1898, two roundings)
//   act    = half(silu(float(gate)) * float(up)), silu(v) = v / (1 + exp(-v))
//            (activation_kernels.cu:133, 300; exp is the hardware's fast exp, as the
//            reference's __expf, and the division a v_rcp_f32 product: fq_common.h silu_mul8)
// half_clamp = clamp_inf_for_half (reduce_kernel_utils.cuh:357-361): clamp to +-(65504 - 1000),
// then round to fp16.
#include "fq_common.h"

constexpr int PR_THREADS = 256;  // SiLU kernel
constexpr int PR_KMAX = 32768;   // RMSNorm rows: T * 8 * MAXCH = 32768 for every T

// the 16 lanes of a group quantize and store their codes and the group's scale
__device__ __forceinline__ void quant_store(uint4 vals, int abits, bool valid, int8_t *xq_row_chunk,
                                            uint16_t *xs_slot, bool first_lane) {
    uint2 codes;
    const uint16_t sh = quant_group16(vals, abits, codes);
    if (valid) {
        *reinterpret_cast<uint2 *>(xq_row_chunk) = codes;
        if (first_lane) *xs_slot = sh;
    }
}

template <int T>
__global__ __launch_bounds__(T) void fq_rmsnorm_quant_kernel(const uint16_t *__restrict__ input,
                                                             const uint16_t *residual, uint16_t *res_out,
                                                             const uint16_t *__restrict__ gamma, float eps,
                                                             int M, int K, int abits, int8_t *__restrict__ xq,
                                                             uint16_t *__restrict__ xs,
                                                             uint16_t *__restrict__ normed) {
    constexpr int MAXCH = PR_KMAX / 8 / T;
    __shared__ float wsum[T / 64];
    const int m = blockIdx.x, t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const int nq = K / 8;  // chunks in the row
    const size_t row = (size_t)m * K;
    uint4 r[MAXCH], gm[MAXCH];
    float acc = 0.0f;
#pragma unroll
    for (int c = 0; c < MAXCH; c++) {
        const int q = c * T + t;
        r[c] = gm[c] = make_uint4(0, 0, 0, 0);
        if (c * T < nq && q < nq) {
            gm[c] = *reinterpret_cast<const uint4 *>(gamma + 8 * (size_t)q);  // in flight with the row
            uint4 res = *reinterpret_cast<const uint4 *>(residual + row + 8 * (size_t)q);
            if (input) {  // (res_out may be the residual itself: each thread owns its chunks)
                res = add_residual8(*reinterpret_cast<const uint4 *>(input + row + 8 * (size_t)q), res);
                *reinterpret_cast<uint4 *>(res_out + row + 8 * (size_t)q) = res;
            }
            r[c] = res;
            acc = sumsq8(res, acc);
        }
    }
    acc = wave_sum64(acc);
    if (lane == 0) wsum[wid] = acc;
    __syncthreads();
    float ss = wsum[0];
#pragma unroll
    for (int w = 1; w < T / 64; w++) ss = ss + wsum[w];
    const float rs = rms_scale(ss, K, eps);
#pragma unroll
    for (int c = 0; c < MAXCH; c++) {
        if (c * T >= nq) break;  // block-uniform
        const int q = c * T + t;
        const bool valid = q < nq;  // whole 16-lane groups (nq % 16 == 0)
        uint4 nv = make_uint4(0, 0, 0, 0);
        if (valid) {
            nv = rms_apply8(r[c], gm[c], rs);
            if (normed) *reinterpret_cast<uint4 *>(normed + row + 8 * (size_t)q) = nv;
        }
        const int gidx = q >> 4;  // 128-group of this chunk
        quant_store(nv, abits, valid, xq + row + 8 * (size_t)q, xs + (size_t)gidx * M + m, (t & 15) == 0);
    }
}

__global__ __launch_bounds__(PR_THREADS) void fq_silu_mul_quant_kernel(const uint16_t *__restrict__ gate,
                                                                       const uint16_t *__restrict__ up, int ld, int M,
                                                                       int N, int abits, int8_t *__restrict__ xq,
                                                                       uint16_t *__restrict__ xs,
                                                                       uint16_t *__restrict__ act) {
    const int m = blockIdx.y;
    const int q = blockIdx.x * PR_THREADS + threadIdx.x;  // chunk of 8 in the row
    const int nq = N / 8;
    const bool valid = q < nq;  // whole 16-lane groups (nq % 16 == 0)
    uint4 av = make_uint4(0, 0, 0, 0);
    if (valid) {
        av = silu_mul8(*reinterpret_cast<const uint4 *>(gate + (size_t)m * ld + 8 * (size_t)q),
                       *reinterpret_cast<const uint4 *>(up + (size_t)m * ld + 8 * (size_t)q));
        if (act) *reinterpret_cast<uint4 *>(act + (size_t)m * N + 8 * (size_t)q) = av;
    }
    quant_store(av, abits, valid, xq + (size_t)m * N + 8 * (size_t)q, xs + (size_t)(q >> 4) * M + m,
                (threadIdx.x & 15) == 0);
}

static bool aligned16(const void *p) { return ((uintptr_t)p & 15) == 0; }

// residual + input -> res_out (which may be the residual itself: fq_rmsnorm_quantize's in-place
// form); fq_rmsnorm_linear_w6ax's unfused path writes a separate buffer.
fq_status fq_rmsnorm_quantize_to(const uint16_t *input, const uint16_t *residual, uint16_t *res_out,
                                 const uint16_t *gamma, float eps, int M, int K, int abits, int8_t *xq, uint16_t *xs,
                                 uint16_t *normed_out, fq_stream_t stream) {
    if (!residual || !gamma || !xq || !xs || (input && !res_out)) return FQ_ERR_NULL;
    if (M <= 0 || K <= 0 || K % FQ_GROUP || K > PR_KMAX) return FQ_ERR_SHAPE;
    if (abits != 6 && abits != 8) return FQ_ERR_BITS;
    if (!aligned16(residual) || !aligned16(gamma) || !aligned16(xq) || (input && !aligned16(input)) ||
        (input && !aligned16(res_out)) || (normed_out && !aligned16(normed_out)))
        return FQ_ERR_SHAPE;
    const int nq = K / 8;  // the oracle (fqo_rmsnorm_quantize) sizes T the same way
#define FQ_RMS_LAUNCH(T)                                                                                         \
    hipLaunchKernelGGL(fq_rmsnorm_quant_kernel<T>, dim3(M), dim3(T), 0, (hipStream_t)stream, input, residual, \
                       res_out, gamma, eps, M, K, abits, xq, xs, normed_out)
    if (nq <= 256)
        FQ_RMS_LAUNCH(256);
    else if (nq <= 512)
        FQ_RMS_LAUNCH(512);
    else
        FQ_RMS_LAUNCH(1024);
#undef FQ_RMS_LAUNCH
    FQ_LAUNCH_CHECK();
    return FQ_OK;
}

extern "C" fq_status fq_rmsnorm_quantize(const uint16_t *input, uint16_t *residual, const uint16_t *gamma, float eps,
                                         int M, int K, int abits, int8_t *xq, uint16_t *xs, uint16_t *normed_out,
                                         fq_stream_t stream) {
    return fq_rmsnorm_quantize_to(input, residual, residual, gamma, eps, M, K, abits, xq, xs, normed_out, stream);
}

extern "C" fq_status fq_silu_mul_quantize(const uint16_t *gate, const uint16_t *up, int ld, int M, int N, int abits,
                                          int8_t *xq, uint16_t *xs, uint16_t *act_out, fq_stream_t stream) {
    if (!gate || !up || !xq || !xs) return FQ_ERR_NULL;
    if (M <= 0 || N <= 0 || N % FQ_GROUP || ld < N || ld % 8 || M > 65535) return FQ_ERR_SHAPE;
    if (abits != 6 && abits != 8) return FQ_ERR_BITS;
    if (!aligned16(gate) || !aligned16(up) || !aligned16(xq) || (act_out && !aligned16(act_out))) return FQ_ERR_SHAPE;
    const dim3 grid((N / 8 + PR_THREADS - 1) / PR_THREADS, M);
    hipLaunchKernelGGL(fq_silu_mul_quant_kernel, grid, dim3(PR_THREADS), 0, (hipStream_t)stream, gate, up, ld, M, N,
                       abits, xq, xs, act_out);
    FQ_LAUNCH_CHECK();
    return FQ_OK;
}

// ---- OPT-family LayerNorm producer: residual [+ input] [+ bias] -> LayerNorm (gamma, beta) -> codes.
// generalAddBiasResidualLayerNormOpt2FlexQFusion (e2e .../kernels/layernorm_kernels.cu:316-575; the
// pre-attention form invokeGeneralLayerNorm :2325-2420 is residual only, no bias, no input).  The
// reference normalises in block y = 0 and quantizes in every block of the row after a block-local
// barrier (the cross-block race of SURVEY.md §5); here one workgroup owns the row, as for RMSNorm.
// Arithmetic: fq_common.h ln_add8 .. ln_apply8 (restated by oracle/fq_oracle.c fqo_layernorm_quantize).
template <int T>
__global__ __launch_bounds__(T) void fq_layernorm_quant_kernel(const uint16_t *__restrict__ input,
                                                               const uint16_t *residual,
                                                               const uint16_t *__restrict__ bias, uint16_t *res_out,
                                                               const uint16_t *__restrict__ gamma,
                                                               const uint16_t *__restrict__ beta, float eps, int M,
                                                               int K, int abits, int8_t *__restrict__ xq,
                                                               uint16_t *__restrict__ xs,
                                                               uint16_t *__restrict__ normed) {
    constexpr int MAXCH = PR_KMAX / 8 / T;
    __shared__ float wsum[2 * (T / 64)];
    const int m = blockIdx.x, t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const int nq = K / 8;
    const size_t row = (size_t)m * K;
    uint4 h[MAXCH];
    float s = 0.0f, q = 0.0f;
#pragma unroll
    for (int c = 0; c < MAXCH; c++) {
        const int qi = c * T + t;
        h[c] = make_uint4(0, 0, 0, 0);
        if (c * T < nq && qi < nq) {
            const uint4 res = *reinterpret_cast<const uint4 *>(residual + row + 8 * (size_t)qi);
            uint4 in, bv;
            if (input) in = *reinterpret_cast<const uint4 *>(input + row + 8 * (size_t)qi);
            if (bias) bv = *reinterpret_cast<const uint4 *>(bias + 8 * (size_t)qi);
            float v[8];
            ln_add8(input ? &in : nullptr, res, bias ? &bv : nullptr, v);
            h[c] = ln_pack8(v);
            // (res_out may be the residual itself: each thread owns its chunks)
            if (res_out) *reinterpret_cast<uint4 *>(res_out + row + 8 * (size_t)qi) = h[c];
            ln_sums8(v, s, q);
        }
    }
    s = wave_sum64(s);
    q = wave_sum64(q);
    if (lane == 0) {
        wsum[wid] = s;
        wsum[T / 64 + wid] = q;
    }
    __syncthreads();
    float S = wsum[0], Q = wsum[T / 64];
#pragma unroll
    for (int w = 1; w < T / 64; w++) {
        S = S + wsum[w];
        Q = Q + wsum[T / 64 + w];
    }
    const float2 st = ln_stats(S, Q, K, eps);
#pragma unroll
    for (int c = 0; c < MAXCH; c++) {
        if (c * T >= nq) break;  // block-uniform
        const int qi = c * T + t;
        const bool valid = qi < nq;  // whole 16-lane groups (nq % 16 == 0)
        uint4 nv = make_uint4(0, 0, 0, 0);
        if (valid) {
            const uint4 g = *reinterpret_cast<const uint4 *>(gamma + 8 * (size_t)qi);
            uint4 b;
            if (beta) b = *reinterpret_cast<const uint4 *>(beta + 8 * (size_t)qi);
            nv = ln_apply8(h[c], st, g, beta ? &b : nullptr);
            if (normed) *reinterpret_cast<uint4 *>(normed + row + 8 * (size_t)qi) = nv;
        }
        quant_store(nv, abits, valid, xq + row + 8 * (size_t)qi, xs + (size_t)(qi >> 4) * M + m, (t & 15) == 0);
    }
}

static bool overlaps(const void *a, size_t na, const void *b, size_t nb) {
    if (!a || !b) return false;
    const uintptr_t x = (uintptr_t)a, y = (uintptr_t)b;
    return x < y + nb && y < x + na;
}

extern "C" fq_status fq_layernorm_quantize(const uint16_t *input, const uint16_t *residual, const uint16_t *bias,
                                           uint16_t *res_out, const uint16_t *gamma, const uint16_t *beta, float eps,
                                           int M, int K, int abits, int8_t *xq, uint16_t *xs, uint16_t *normed_out,
                                           fq_stream_t stream) {
    if (!residual || !gamma || !xq || !xs) return FQ_ERR_NULL;
    if (M <= 0 || K <= 0 || K % FQ_GROUP || K > PR_KMAX) return FQ_ERR_SHAPE;
    if (abits != 6 && abits != 8) return FQ_ERR_BITS;
    if (!aligned16(residual) || !aligned16(gamma) || !aligned16(xq) || (input && !aligned16(input)) ||
        (bias && !aligned16(bias)) || (beta && !aligned16(beta)) || (res_out && !aligned16(res_out)) ||
        (normed_out && !aligned16(normed_out)))
        return FQ_ERR_SHAPE;
    // res_out may be the residual (in place) but must not overlap the input, bias, gamma or beta
    const size_t rb = (size_t)M * K * 2, vb = (size_t)K * 2;
    if (res_out && (overlaps(res_out, rb, input, rb) || overlaps(res_out, rb, bias, vb) ||
                    overlaps(res_out, rb, gamma, vb) || overlaps(res_out, rb, beta, vb) ||
                    (res_out != residual && overlaps(res_out, rb, residual, rb))))
        return FQ_ERR_SHAPE;
    const int nq = K / 8;
#define FQ_LN_LAUNCH(T)                                                                                             \
    hipLaunchKernelGGL(fq_layernorm_quant_kernel<T>, dim3(M), dim3(T), 0, (hipStream_t)stream, input, residual,  \
                       bias, res_out, gamma, beta, eps, M, K, abits, xq, xs, normed_out)
    if (nq <= 256)
        FQ_LN_LAUNCH(256);
    else if (nq <= 512)
        FQ_LN_LAUNCH(512);
    else
        FQ_LN_LAUNCH(1024);
#undef FQ_LN_LAUNCH
    FQ_LAUNCH_CHECK();
    return FQ_OK;
}
