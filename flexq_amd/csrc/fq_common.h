// fq_common.h -- shared device helpers for the gfx950 W6Ax engine (no CUDA, no dual paths).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

#include "../../include/flexq_hip.h"

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float v16f __attribute__((ext_vector_type(16)));

#define FQ_GROUP 128
#define FQ_WAVE 64
// head of every GEMM workspace: the split-K tickets (one uint32 per 16-column tile, up to 65536
// tiles), zeroed once by fq_workspace_init and left zeroed by the kernels
constexpr size_t FQ_TICKET_BYTES = 256 * 1024;

// ---- fp16 bit-pattern helpers (values travel as uint16_t through the C ABI) ----------------
__device__ __forceinline__ float h2f(uint16_t h) { return __half2float(__ushort_as_half(h)); }
__device__ __forceinline__ uint16_t f2h(float f) { return __half_as_ushort(__float2half_rn(f)); }

// roundf semantics (half away from zero), the rounding of the reference quantizer
// (e2e .../flexqgemm/src/pack/bit_packing.cu:160 `round(float)`).
__device__ __forceinline__ float round_half_away(float v) {
    float t = __builtin_truncf(v);
    if (__builtin_fabsf(v - t) >= 0.5f) t += __builtin_copysignf(1.0f, v);
    return t;
}

// CUDA's saturating float->int (cvt.rzi.s32.f32) followed by clamp(lo, hi):
// NaN -> 0, +inf -> hi, -inf -> lo.
__device__ __forceinline__ int sat_clamp(float v, int lo, int hi) {
    const int c = (int)fminf(fmaxf(v, (float)lo), (float)hi);  // branch-free; exact in range
    return v == v ? c : 0;
}

// ---- dynamic group quantizer (one 128-wide group over 16 consecutive, 16-aligned lanes) ----
// Restates e2e .../flexqgemm/src/pack/bit_packing.cu:125-164 exactly: fp16 absmax seeded with
// -1 (:139; fmaxf drops NaN like __hmax), maxv = absmax / (2^(b-1)-1) in IEEE fp32, scale =
// half(maxv) round-to-nearest, q = clamp(roundf(float(x) / float(scale))) with CUDA's saturating
// conversion.  `raw` = this lane's 8 fp16; all 16 lanes of the group must execute the call.
// Returns the fp16 scale bits and the 8 codes packed as little-endian int8 bytes.
//
// The 16-lane max runs on DPP (quad_perm xor1/xor2, row_half_mirror, row_mirror: a full max
// over the 16-lane row without LDS).  The per-element quotient and its rounding are one fused
// multiply-add with a biased reciprocal instead of the IEEE division sequence (see the element
// step below for why the codes are identical).
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

__device__ __forceinline__ float max16(float m) {
    m = fmaxf(m, dpp_f32<0xB1>(m));   // quad_perm [1,0,3,2]
    m = fmaxf(m, dpp_f32<0x4E>(m));   // quad_perm [2,3,0,1]
    m = fmaxf(m, dpp_f32<0x141>(m));  // row_half_mirror: quad q <-> quad 1-q within 8 lanes
    m = fmaxf(m, dpp_f32<0x140>(m));  // row_mirror: half h <-> half 1-h within the 16-lane row
    return m;
}

// The same 16-lane max for values that are -1.0 or non-negative (never NaN): their bit patterns
// order like signed integers, so the reduction is four v_max_i32 with a DPP source (no NaN
// canonicalisation around each step, which fmaxf needs).
template <int CTRL>
__device__ __forceinline__ int dpp_i32(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ float max16_nonneg(float m) {
    int b = __float_as_int(m);
    b = max(b, dpp_i32<0xB1>(b));
    b = max(b, dpp_i32<0x4E>(b));
    b = max(b, dpp_i32<0x141>(b));
    b = max(b, dpp_i32<0x140>(b));
    return __int_as_float(b);
}

__device__ __forceinline__ int med3_i32(int v, int lo, int hi) {
    int r;
    asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(v), "v"(lo), "v"(hi));
    return r;
}

// v_cvt_i32_f32: truncation with the hardware's saturation (out of range clamps, NaN -> 0),
// the same results as CUDA's cvt.rzi.s32.f32 that the reference relies on.
__device__ __forceinline__ int cvt_i32_sat(float v) {
    int r;
    asm("v_cvt_i32_f32 %0, %1" : "=v"(r) : "v"(v));
    return r;
}

typedef float v2f __attribute__((ext_vector_type(2)));

// A group's scale from its absmax mx (a non-negative fp16 value, as fp32), and the element step's
// reciprocal rcb.  IEEE fp32 absmax / hi as a Newton-corrected product with y = RN(1/hi):
// bit-identical over every fp16 absmax (exhaustive: tests/test_oracle.py::
// test_quantizer_division_by_constant_is_exact).
// Element step: roundf(RN(x / r)) == trunc(RN(x * rcb + copysign(0.5, x))) with
// rcb = RN(v_rcp(r) * (1 + 2^-20)), one fused multiply-add per element.  x and r are fp16,
// so a quotient that is not an exact tie k + 0.5 lies far beyond the reciprocal's error from
// one, and the 2^-20 bias carries an exact tie across the truncation boundary.  Exhaustive
// over every fp16 absmax and element, both bit widths, the reciprocal off by up to 4 ulp
// (oracle/fq_oracle.c fqo_check_quant_fma, tests/test_oracle.py).  r = 0 (an all-zero group)
// gives 0 * inf = NaN and r = inf gives +-0.5: code 0, as the IEEE quotient's class does; the
// truncating, saturating v_cvt_i32_f32 maps NaN to 0 and +-inf to the int range.
__device__ __forceinline__ uint16_t quant_scale(float mx, int bits, float &rcb) {
    const int hi = (1 << (bits - 1)) - 1;
    const float fhi = (float)hi, y = bits == 8 ? (float)(1.0 / 127.0) : (float)(1.0 / 31.0);
    const float m1 = mx * y;
    const float maxv = __builtin_isfinite(m1) ? fmaf(fmaf(-m1, fhi, mx), y, m1) : m1;
    const uint16_t sh = f2h(maxv);
    rcb = __builtin_amdgcn_rcpf(h2f(sh)) * (1.0f + 0x1p-20f);
    return sh;
}

// The element step (above) for one fp16 value x (as fp32): its code, clamped to [lo, hi].
__device__ __forceinline__ int quant_code(float x, float rcb, int lo, int hi) {
    return med3_i32(cvt_i32_sat(fmaf(x, rcb, __builtin_copysignf(0.5f, x))), lo, hi);
}

// One (row, 128-group) per 16 lanes, 8 fp16 values per lane: absmax over the values converted to
// fp32 (fmaxf skips NaN, as the reference's __hmax), the element step on the converted values.
// (An integer-absmax variant -- a packed-u16 max over the fp16 bit patterns, one conversion instead
// of eight, v_fma_mix element steps, a NaN fallback -- was bit-identical and 0.8-1.1 % slower per
// step: DESIGN.md §8.)
__device__ __forceinline__ uint16_t quant_group16(uint4 raw, int bits, uint2 &codes) {
    const uint32_t wd[4] = {raw.x, raw.y, raw.z, raw.w};
    const int hi = (1 << (bits - 1)) - 1, lo = -(1 << (bits - 1));
    v2f v[4];
    float mx = -1.0f;  // the reference's seed; fmaxf skips NaN inputs, so mx is never NaN
#pragma unroll
    for (int i = 0; i < 4; i++) {
        v[i] = v2f{h2f((uint16_t)wd[i]), h2f((uint16_t)(wd[i] >> 16))};
        mx = fmaxf(mx, fmaxf(fabsf(v[i].x), fabsf(v[i].y)));
    }
    mx = max16_nonneg(mx);
    float rcb;
    const uint16_t sh = quant_scale(mx, bits, rcb);
    const v2f rcb2 = {rcb, rcb};
    int c[8];
#pragma unroll
    for (int i = 0; i < 4; i++) {  // packed fp32: v_pk_fma_f32
        const v2f hs = {__builtin_copysignf(0.5f, v[i].x), __builtin_copysignf(0.5f, v[i].y)};
        const v2f t = __builtin_elementwise_fma(v[i], rcb2, hs);
        c[2 * i] = med3_i32(cvt_i32_sat(t.x), lo, hi);
        c[2 * i + 1] = med3_i32(cvt_i32_sat(t.y), lo, hi);
    }
    // low bytes of 8 codes -> 2 dwords (v_perm_b32: selector 0x0c = zero byte)
    uint32_t w[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const uint32_t p01 = __builtin_amdgcn_perm((uint32_t)c[4 * h + 1], (uint32_t)c[4 * h], 0x0c0c0400u);
        const uint32_t p23 = __builtin_amdgcn_perm((uint32_t)c[4 * h + 3], (uint32_t)c[4 * h + 2], 0x0c0c0400u);
        w[h] = __builtin_amdgcn_perm(p23, p01, 0x05040100u);
    }
    codes = make_uint2(w[0], w[1]);
    return sh;
}

__device__ __forceinline__ float lo_f(uint32_t w) { return h2f((uint16_t)w); }
__device__ __forceinline__ float hi_f(uint32_t w) { return h2f((uint16_t)(w >> 16)); }

// ---- producer arithmetic, 8 fp16 values per call: fq_producers.hip's kernels and the decode
// kernel's fused prologues (fq_gemm.hip, PRO = 1 / 2 / 4) share these, so the two give the same bits.
// half_clamp = clamp_inf_for_half (reduce_kernel_utils.cuh:357-361): clamp to +-(65504 - 1000).
__device__ __forceinline__ float half_clamp_f(float v) {
    return v > 0.0f ? fminf(v, 65504.0f - 1000.0f) : fmaxf(v, -65504.0f + 1000.0f);
}
__device__ __forceinline__ uint32_t pack_h2(float a, float b) {
    return (uint32_t)f2h(a) | ((uint32_t)f2h(b) << 16);
}

// r = half_clamp(float(in) + float(res))                    (layernorm_kernels.cu:1883)
__device__ __forceinline__ uint4 add_residual8(uint4 in, uint4 res) {
    const uint32_t a[4] = {in.x, in.y, in.z, in.w}, b[4] = {res.x, res.y, res.z, res.w};
    uint32_t o[4];
#pragma unroll
    for (int i = 0; i < 4; i++)
        o[i] = pack_h2(half_clamp_f(lo_f(a[i]) + lo_f(b[i])), half_clamp_f(hi_f(a[i]) + hi_f(b[i])));
    return make_uint4(o[0], o[1], o[2], o[3]);
}
// acc += float(r)^2 over the 8 values in order (fmaf)
__device__ __forceinline__ float sumsq8(uint4 r, float acc) {
    const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const float v0 = lo_f(w[i]), v1 = hi_f(w[i]);
        acc = fmaf(v0, v0, acc);
        acc = fmaf(v1, v1, acc);
    }
    return acc;
}
// 1 / sqrt(ss / K + eps), IEEE (the reference uses rsqrtf, layernorm_kernels.cu:1890)
__device__ __forceinline__ float rms_scale(float ss, int K, float eps) {
    return 1.0f / __builtin_sqrtf(ss / (float)K + eps);
}
// normed = half_clamp((float(r) * rs) * float(gamma)), two roundings     (:1898)
__device__ __forceinline__ uint4 rms_apply8(uint4 r, uint4 g, float rs) {
    const uint32_t a[4] = {r.x, r.y, r.z, r.w}, gm[4] = {g.x, g.y, g.z, g.w};
    uint32_t o[4];
#pragma unroll
    for (int i = 0; i < 4; i++)
        o[i] = pack_h2(half_clamp_f(__fmul_rn(__fmul_rn(lo_f(a[i]), rs), lo_f(gm[i]))),
                       half_clamp_f(__fmul_rn(__fmul_rn(hi_f(a[i]), rs), hi_f(gm[i]))));
    return make_uint4(o[0], o[1], o[2], o[3]);
}
// act = half(silu(float(gate)) * float(up)), silu(v) = v * rcp(1 + exp(-v)) with the hardware's
// fast exp (the reference's __expf) and v_rcp_f32 (1 ulp) in place of the IEEE division
// (activation_kernels.cu:133, 300): the fp32 silu is within ~2^-22 relative of the exact value, so
// the fp16 product stays within one fp16 ulp of the exact one (the producers' tolerance), at a
// fraction of the division's instructions.  Non-finite cases match the division: g = -inf gives
// -inf * 0 = NaN (as -inf / inf), a large negative g gives -0.
__device__ __forceinline__ uint4 silu_mul8(uint4 g4, uint4 u4) {
    const uint32_t g[4] = {g4.x, g4.y, g4.z, g4.w}, u[4] = {u4.x, u4.y, u4.z, u4.w};
    uint32_t o[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const float g0 = lo_f(g[i]), g1 = hi_f(g[i]);
        const float s0 = g0 * __builtin_amdgcn_rcpf(1.0f + __expf(-g0));
        const float s1 = g1 * __builtin_amdgcn_rcpf(1.0f + __expf(-g1));
        o[i] = pack_h2(__fmul_rn(s0, lo_f(u[i])), __fmul_rn(s1, hi_f(u[i])));
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}

// ---- OPT-family LayerNorm producer arithmetic (generalAddBiasResidualLayerNormOpt2FlexQFusion,
// e2e .../kernels/layernorm_kernels.cu:316-575), 8 fp16 values per call:
//   v      = ((0 + float(bias)) + float(residual)) + float(input)   in fp32, absent terms skipped (:357-385)
//   h      = half(v)                                                 (the residual output, :393-395)
//   sums   s += v[2i] + v[2i+1],  q += v[2i] * v[2i] + v[2i+1] * v[2i+1]   per half2 pair (:396-397)
//   mean   = (s / (K/2)) / 2,  rs = 1 / sqrt(((q / (K/2)) / 2 - mean * mean) + eps)   (:403-404; IEEE
//            where the reference has rsqrtf)
//   normed = ((h - half(mean)) * half(rs)) * gamma [+ beta]   every step an fp16 operation (:412-416)
// The reference's fp32 sums follow its launch shape; this build's order (per thread over its chunks,
// the pairs of a chunk in order, wave_sum64, the waves in order) is the one the oracle restates.
__device__ __forceinline__ void ln_add8(const uint4 *in, const uint4 &res, const uint4 *bias, float (&v)[8]) {
#pragma clang fp contract(off)
    const uint32_t r[4] = {res.x, res.y, res.z, res.w};
#pragma unroll
    for (int i = 0; i < 4; i++) {
        float a0 = 0.0f, a1 = 0.0f;
        if (bias) {
            const uint32_t b[4] = {bias->x, bias->y, bias->z, bias->w};
            a0 = a0 + lo_f(b[i]);
            a1 = a1 + hi_f(b[i]);
        }
        a0 = a0 + lo_f(r[i]);
        a1 = a1 + hi_f(r[i]);
        if (in) {
            const uint32_t x[4] = {in->x, in->y, in->z, in->w};
            a0 = a0 + lo_f(x[i]);
            a1 = a1 + hi_f(x[i]);
        }
        v[2 * i] = a0;
        v[2 * i + 1] = a1;
    }
}
__device__ __forceinline__ uint4 ln_pack8(const float (&v)[8]) {
    return make_uint4(pack_h2(v[0], v[1]), pack_h2(v[2], v[3]), pack_h2(v[4], v[5]), pack_h2(v[6], v[7]));
}
__device__ __forceinline__ void ln_sums8(const float (&v)[8], float &s, float &q) {
#pragma clang fp contract(off)
#pragma unroll
    for (int i = 0; i < 4; i++) {
        s = s + (v[2 * i] + v[2 * i + 1]);
        q = q + (__fmul_rn(v[2 * i], v[2 * i]) + __fmul_rn(v[2 * i + 1], v[2 * i + 1]));
    }
}
// (mean, 1 / sqrt(var + eps)) from the row sums; K = the row length
__device__ __forceinline__ float2 ln_stats(float s, float q, int K, float eps) {
#pragma clang fp contract(off)
    const float n = (float)(K / 2);
    const float mean = (s / n) / 2.0f;
    const float var = ((q / n) / 2.0f - __fmul_rn(mean, mean)) + eps;
    return make_float2(mean, 1.0f / __builtin_sqrtf(var));
}
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
// normed = ((h - mean_h) * rs_h) * gamma [+ beta], packed fp16 (v_pk_sub/mul/add_f16, round to nearest)
__device__ __forceinline__ uint4 ln_apply8(uint4 h, float2 st, uint4 gamma, const uint4 *beta) {
#pragma clang fp contract(off)
    const _Float16 mh = (_Float16)st.x, rh = (_Float16)st.y;
    const h2v m2 = {mh, mh}, r2 = {rh, rh};
    const uint32_t hw[4] = {h.x, h.y, h.z, h.w}, gw[4] = {gamma.x, gamma.y, gamma.z, gamma.w};
    uint32_t o[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        h2v a = __builtin_bit_cast(h2v, hw[i]);
        a = ((a - m2) * r2) * __builtin_bit_cast(h2v, gw[i]);
        if (beta) {
            const uint32_t bw[4] = {beta->x, beta->y, beta->z, beta->w};
            a = a + __builtin_bit_cast(h2v, bw[i]);
        }
        o[i] = __builtin_bit_cast(uint32_t, a);
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}

// Sum of a float over the 64 lanes of a wave, in a fixed tree: lane pairs, quads, 8- and 16-lane
// halves on DPP (after each step every lane of a block holds the block's sum, so a mirror partner
// is as good as the xor partner), then the four 16-lane rows as (r0 + r1) + (r2 + r3).  The same
// bits as an xor butterfly over offsets 1, 2, 4, 8, 16, 32 (oracle/fq_oracle.c
// fqo_rmsnorm_quantize); returns the wave-uniform total.
__device__ __forceinline__ float wave_sum64(float v) {
    v = v + dpp_f32<0xB1>(v);   // quad_perm [1,0,3,2]: lane ^ 1
    v = v + dpp_f32<0x4E>(v);   // quad_perm [2,3,0,1]: lane ^ 2
    v = v + dpp_f32<0x141>(v);  // row_half_mirror: the other quad of the 8
    v = v + dpp_f32<0x140>(v);  // row_mirror: the other 8 of the 16
    const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
    const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
    const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
    const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
    return (r0 + r1) + (r2 + r3);
}

// arguments of a producer fused into the decode linear's prologue (fq_gemm.hip, PRO = 1 / 2)
struct DecodePro {
    const uint16_t *in;     // PRO 1 / 4: added to the residual (or null); PRO 2: up
    const uint16_t *gamma;  // PRO 1 / 4
    uint16_t *res_out;      // PRO 1 with `in`, PRO 4: residual + in (never the residual itself)
    float eps;              // PRO 1 / 4
    int ldh;                // row stride (elements) of xh and `in` (PRO 2; K otherwise)
    const uint16_t *beta;   // PRO 4 (or null)
    const uint16_t *bias;   // PRO 4 (or null)
    const struct fq_gather *wgat;  // peer-store gather kernel: the gather whose output is x, waited
    uint32_t *werr;                //   for in the prologue (or null: x is ready); its error word
    uint32_t *chain;        // decode chain (fq_linear_chain_w6ax): the launch's sync words
    int link;               //   this linear's position in the chain
    uint32_t epoch;         //   the launch's epoch (granule tags)
    const uint64_t *hx;     //   granules holding x (the previous linear's hand-off), or null: x is ready
    uint64_t *hd;           //   this linear's hand-off granules (null: the chain's last linear)
    int cpro;               //   the linear's producer: 0 none, 1 residual add + RMSNorm, 2 SiLU * up
    const uint64_t *hin;    //   granules holding `in` (the previous linear's hand-off), or null
    uint64_t *hr;           //   RMSNorm: granules of res_out for a later linear (or null)
    bool cwrite;            //   linear 0: wave 0 copies the chain's argument block to LDS at cdesc_lds:
    uint32_t cdesc_lds;     //     plain chains: 512 B, loaded as the launch starts (dvx, dvy per lane);
    uint64_t kargs;         //     producer chains: 1 KiB, loaded behind linear 0's ring from kargs
    uint32_t dvx, dvy;
    uint32_t nxt_w, nxt_p;  //   LDS addresses of the next linear's weight pointer and packed fields (its
                            //   ring is issued by this linear's tail), or 0: the last linear
    bool pre;               //   this linear's ring was issued by the previous linear's tail
};

// ---- fq6 weight unpack ----------------------------------------------------------------------
// Three packed dwords -> the 16-byte MFMA B operand, every byte = 4*w (w in the top 6 bits).
// Layout contract: oracle/fq_oracle.c fqo_pack_fq6 and DESIGN.md §3.
__device__ __forceinline__ v4i unpack_fq6(uint32_t p0, uint32_t p1, uint32_t p2) {
    const uint32_t HI = 0xFCFCFCFCu, LO = 0x03030303u;
    v4i o;
    o[0] = (int)(p0 & HI);
    o[1] = (int)(p1 & HI);
    o[2] = (int)(p2 & HI);
    o[3] = (int)(((p0 & LO) << 2) | ((p1 & LO) << 4) | ((p2 & LO) << 6));
    return o;
}

// Host helpers ------------------------------------------------------------------------------
#define FQ_LAUNCH_CHECK()                                                  \
    do {                                                                   \
        if (hipGetLastError() != hipSuccess) return FQ_ERR_HIP;            \
    } while (0)

static inline int fq_cdiv(long a, long b) { return (int)((a + b - 1) / b); }
