// fq_lds.h -- LDS / wait-count helpers shared by the gfx950 GEMM kernels (fq_gemm.hip, fq_seq.hip).
// LDS accesses are inline asm on purpose: hipcc cannot tell them from LDS-DMA still landing and
// would guard each with s_waitcnt vmcnt(0); every wait here is counted by hand.
#pragma once
#include "fq_common.h"

#define LDS_PTR(p) ((__attribute__((address_space(3))) void *)(p))

__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char *)(p);
}
__device__ __forceinline__ v4i ds_read_b128(uint32_t a) {
    v4i v;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a));
    return v;
}
typedef unsigned v2u __attribute__((ext_vector_type(2)));
__device__ __forceinline__ v2u ds_read_b64(uint32_t a) {
    v2u v;
    asm volatile("ds_read_b64 %0, %1" : "=v"(v) : "v"(a));
    return v;
}
__device__ __forceinline__ void ds_write_b64(uint32_t a, uint2 v) {
    asm volatile("ds_write_b64 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ void ds_write_b128(uint32_t a, v4i v) {
    asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ uint32_t ds_read_b32(uint32_t a) {
    uint32_t v;
    asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"(a));
    return v;
}
__device__ __forceinline__ void ds_write_b32(uint32_t a, uint32_t v) {
    asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ uint32_t ds_read_u16(uint32_t a) {
    uint32_t v;
    asm volatile("ds_read_u16 %0, %1" : "=v"(v) : "v"(a));
    return v;
}

// immediate-offset forms (offset < 64 KiB folded into the instruction)
template <int OFF>
__device__ __forceinline__ v4i ds_read_b128_at(uint32_t a) {
    v4i v;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(OFF));
    return v;
}
template <int OFF>
__device__ __forceinline__ v2u ds_read_b64_at(uint32_t a) {
    v2u v;
    asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(OFF));
    return v;
}
template <int OFF>
__device__ __forceinline__ uint32_t ds_read_u16_at(uint32_t a) {
    uint32_t v;
    asm volatile("ds_read_u16 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(OFF));
    return v;
}

template <int OFF>
__device__ __forceinline__ uint32_t ds_read_b32_at(uint32_t a) {
    uint32_t v;
    asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(OFF));
    return v;
}

// offset k * STEP for a k that is a constant once the caller's loop is unrolled: the switch folds
// to one immediate-offset read (no v_add for the address); any other k takes the register form
#define FQ_DS_READ_K(NAME, T, AT, REG)                                                                  \
    template <int STEP>                                                                                \
    __device__ __forceinline__ T NAME(uint32_t a, int k) {                                             \
        switch (k) {                                                                                   \
            case 0: return AT<0>(a);                                                                   \
            case 1: return AT<STEP>(a);                                                                \
            case 2: return AT<2 * STEP>(a);                                                            \
            case 3: return AT<3 * STEP>(a);                                                            \
            case 4: return AT<4 * STEP>(a);                                                            \
            case 5: return AT<5 * STEP>(a);                                                            \
            case 6: return AT<6 * STEP>(a);                                                            \
            case 7: return AT<7 * STEP>(a);                                                            \
            default: return REG(a + k * STEP);                                                         \
        }                                                                                              \
    }
FQ_DS_READ_K(ds_read_b128_k, v4i, ds_read_b128_at, ds_read_b128)
FQ_DS_READ_K(ds_read_b32_k, uint32_t, ds_read_b32_at, ds_read_b32)
FQ_DS_READ_K(ds_read_u16_k, uint32_t, ds_read_u16_at, ds_read_u16)
#undef FQ_DS_READ_K

// fp16 x2 product w * (x.lo, x.lo): v_pk_mul_f16 with the high lane also reading x's low half
// (op_sel_hi), i.e. __hmul2(w, half2(x.lo, x.lo)) without the v_perm that builds the pair
__device__ __forceinline__ uint32_t pk_mul_f16_lo(uint32_t w, uint32_t x) {
    typedef _Float16 h2_ __attribute__((ext_vector_type(2)));
    const _Float16 xl = __builtin_bit_cast(_Float16, (uint16_t)x);
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(h2_, w) * h2_{xl, xl});  // (the splat folds into op_sel_hi)
}

// s_waitcnt vmcnt(BASE + k) for a wave-uniform runtime k (immediates only); vmcnt(0) past 7
template <int BASE>
__device__ __forceinline__ void wait_vm_plus(int k) {
#define FQ_WAIT_PLUS(j)                                                           \
    if (k == (j) && BASE + (j) <= 63) {                                           \
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(BASE + (j) <= 63 ? BASE + (j) : 0) : "memory"); \
        return;                                                                   \
    }
    FQ_WAIT_PLUS(0) FQ_WAIT_PLUS(1) FQ_WAIT_PLUS(2) FQ_WAIT_PLUS(3) FQ_WAIT_PLUS(4) FQ_WAIT_PLUS(5)
    FQ_WAIT_PLUS(6) FQ_WAIT_PLUS(7)
#undef FQ_WAIT_PLUS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int U, int D>
__device__ __forceinline__ void wait_ring(int later) {
    // s_waitcnt takes an immediate: `later` (< D) blocks of U DMA instructions may stay in flight
#define FQ_WAIT_CASE(k)                                                                 \
    if constexpr (D > (k)) {                                                            \
        if (later == (k)) {                                                             \
            asm volatile("s_waitcnt vmcnt(%0)" ::"i"((k) * U) : "memory");              \
            return;                                                                     \
        }                                                                               \
    }
    FQ_WAIT_CASE(11) FQ_WAIT_CASE(10) FQ_WAIT_CASE(9) FQ_WAIT_CASE(8) FQ_WAIT_CASE(7) FQ_WAIT_CASE(6)
    FQ_WAIT_CASE(5) FQ_WAIT_CASE(4) FQ_WAIT_CASE(3) FQ_WAIT_CASE(2) FQ_WAIT_CASE(1)
#undef FQ_WAIT_CASE
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// the ring's steady state: D - 1 younger blocks of U DMA instructions stay in flight
template <int U, int D>
__device__ __forceinline__ void wait_ring_steady() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"((D - 1) * U) : "memory");
}

// Activation rows in LDS are 128 B (one group) with their eight 16-byte chunks XOR-swizzled by
// (row & 7): the A-operand read (16 rows x 16 B per k-chunk) is then conflict-free per 8 lanes.
__host__ __device__ inline int xswz(int row, int chunk) { return (chunk ^ (row & 7)) * 16; }


// ---- decode weight-image block and staged-region sizes (fq_gemm.hip, fq_seq.hip) ----
constexpr int FQ_BLOCK = 1536;  // bytes of one (16-column tile, group) fq6 block
__host__ __device__ inline int decode_xsr(int MT) { return MT <= 16 ? 16 : MT; }
// staged regions, rounded up to whole DMA instructions (each writes 64 lanes' worth)
__host__ __device__ inline int decode_wsst_bytes(int nb) { return ((nb + 31) / 32) * 1024; }
__host__ __device__ inline int decode_xsst_bytes(int ng, int MT) { return ((ng * decode_xsr(MT) + 63) / 64) * 256; }
__host__ __device__ inline int decode_xst_bytes(int ng, int M) { return ((ng * M + 7) / 8) * 1024; }
