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
    if (v != v) return 0;
    if (v >= (float)hi) return hi;
    if (v <= (float)lo) return lo;
    return (int)v;
}

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
