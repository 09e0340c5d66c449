// fq_gemm.hip -- W6A6 / W6A8 GEMM with per-group dequantization for gfx950 (CDNA4).
//
// Contraction: the reference emulates INT6 x INT6 with 36 binary MMAs per bit-pair set
// (mma.m8n8k128.b1.and.popc, engine/src/bgemm/bgemm.cuh:431-450).  Here a 6-bit weight is
// unpacked in registers into the top 6 bits of an int8 (value 4w, fq_common.h unpack_fq6) and
// the contraction runs on v_mfma_i32_32x32x32_i8 with int32 accumulation, reset every 128-wide
// group.  acc4 = 4 * sum_k x*w exactly (|acc4| <= 2^21), so float(acc4) is exact and the final
// x0.25 is exact: the result equals sum_g float(half(xs*ws)) * acc_g accumulated in fp32,
// which is the reference's dequant (flexq_bmma_kernel.h:359-373) with the bit-pair sum moved
// inside the integer accumulator.
//
// MFMA operand maps (32x32x32 i8): lane l holds A[row l&31][k = 16*(l>>5) + j] and
// B[k = 16*(l>>5) + j][col l&31], j = 0..15 -- any k relabelling shared by A and B gives the same
// sum; C/D: col = l&31, row = (r&3) + 8*(r>>2) + 4*(l>>5) (dtype-independent on gfx950).
#include "fq_common.h"

__device__ __forceinline__ int acc_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// Valid accumulator registers for a row tile of MT rows (rows >= MT are never stored).
template <int MT> struct RowRegs { static constexpr int RV = MT <= 8 ? 4 : (MT <= 16 ? 8 : 16); };

// =============================================================================================
// Decode / small-M kernel (M <= 32): HBM-bound weight streaming.
//
// Work items are (n-tile t of 32 columns, k-split z).  A workgroup (one per CU, persistent over
// items w, w + grid, ...) streams each item's contiguous fq6 blocks (3 KiB = 32 columns x one
// 128-wide group); its NW waves take contiguous group sub-ranges, so a tile's partial sums meet
// in LDS (one barrier per item) and S = 1 needs no cross-CU reduction.  Measured on MI355X
// (tools/ubench_stream.hip): one CU streams at most ~50 GB/s while the chip reaches ~6.5 TB/s,
// so whole tiles per CU keep the chip at the aggregate limit; only small N (tensor-parallel
// shards) split K (S > 1, one item per WG).
//   * Ring: D weight slots per wave filled by LDS-DMA (global_load_lds_dwordx4 nt, three 1 KiB
//     planes per block), retired by hand-counted `s_waitcnt vmcnt(U * in-flight)`, and running
//     ahead across item boundaries.  LDS reads are inline asm (hipcc would guard them with
//     vmcnt(0) against the in-flight DMA); the per-item barrier is a raw s_barrier (a
//     __syncthreads() would drain the ring).
//   * Staging (XS/SS = 0): a few wide LDS-DMA instructions in the prologue stage the blocks'
//     w-scales / x-scales and (M <= 4) activation rows, so the loop moves weights only.  When the
//     staged bytes would not fit LDS (very long K), they ride in each ring slot instead (XS/SS = 1).
//   * S > 1: the WG publishes its fp32 partial tile with write-through (sc1) stores, drains them,
//     takes one agent-scope ticket, and the last WG of the tile sums the S slabs in z order
//     (sc1 loads, all in flight together).  Deterministic: fixed order, no float atomics.
//     (MI355X_MICROARCH.md "Valid forms", row 1.)
// =============================================================================================
#define LDS_PTR(p) ((__attribute__((address_space(3))) void *)(p))

__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char *)(p);
}
__device__ __forceinline__ v4i ds_read_b128(uint32_t a) {
    v4i v;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a));
    return v;
}
__device__ __forceinline__ uint32_t ds_read_u16(uint32_t a) {
    uint32_t v;
    asm volatile("ds_read_u16 %0, %1" : "=v"(v) : "v"(a));
    return v;
}

template <int U>
__device__ __forceinline__ void wait_ring(int later) {
    // s_waitcnt takes an immediate: `later` blocks (U DMA instructions each) may stay in flight
    switch (later) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(%0)" ::"i"(U) : "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * U) : "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(%0)" ::"i"(3 * U) : "memory"); break;
    }
}

// XS: activation rows staged (0, M <= 4 only) or carried per ring slot (1).
// SS: w-/x-scales staged (0) or carried per ring slot (1).
// A sub-dword LDS-DMA writes lane l's value zero-extended to dword l of the destination.
template <int MT, int XS, int SS> struct DecodeCfg {
    static constexpr int XP = XS ? (MT <= 8 ? 1 : MT / 8) : 0;  // 1 KiB activation pieces per slot
    static constexpr int WS_OFF = 3072 + XP * 1024;              // slot scales (SS = 1): 32 + MT dwords
    static constexpr int XS_OFF = WS_OFF + 128;
    static constexpr int SLOT = SS ? XS_OFF + MT * 4 : WS_OFF;
    static constexpr int U = 3 + XP + (SS ? 2 : 0);              // ring DMA instructions per block
    static constexpr int D = MT <= 4 ? 4 : (MT <= 16 ? 3 : 2);   // ring depth
};

__host__ __device__ inline int decode_slot(int MT, int XS, int SS) {
    const int XP = XS ? (MT <= 8 ? 1 : MT / 8) : 0;
    return SS ? 3072 + XP * 1024 + 128 + MT * 4 : 3072 + XP * 1024;
}
__host__ __device__ inline int decode_depth(int MT) { return MT <= 4 ? 4 : (MT <= 16 ? 3 : 2); }
// staged regions, rounded up to whole DMA instructions (each writes 64 lanes' worth)
__host__ __device__ inline int decode_wsst_bytes(int nb, bool even) { return even ? ((nb + 3) / 4) * 256 : ((nb + 1) / 2) * 256; }
__host__ __device__ inline int decode_xsst_bytes(int ng, int MT) { return ((ng * MT + 63) / 64) * 256; }
__host__ __device__ inline int decode_xst_bytes(int ng, int M) {
    const int per = 64 / (8 * M);
    return ((ng + per - 1) / per) * per * M * 128;
}
// per-wave LDS: [ring D x SLOT][ws: nb x (16|32) dwords][xs: ng x MT dwords][x: ng x M x 128 B]
__host__ __device__ inline int decode_wave_lds(int MT, int XS, int SS, int ng, int nb, int M, bool even) {
    int b = decode_depth(MT) * decode_slot(MT, XS, SS);
    if (!SS) b += decode_wsst_bytes(nb, even) + decode_xsst_bytes(ng, MT);
    if (!XS) b += decode_xst_bytes(ng, M);
    return b;
}

template <int MT, int NW, int XS, int SS, bool DBG, int ABL = 0>
__global__ __launch_bounds__(NW * 64) void fq_gemm_decode_kernel(
    const int8_t *__restrict__ xq, const uint16_t *__restrict__ xs, const uint32_t *__restrict__ wpk,
    const uint16_t *__restrict__ ws, int M, int N, int K, uint16_t *__restrict__ d,
    int32_t *__restrict__ acc_dbg, float *__restrict__ slabs, uint32_t *__restrict__ tickets, int S, int IPW) {
    using C = DecodeCfg<MT, XS, SS>;
    constexpr int D = C::D, RV = RowRegs<MT>::RV;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int G = K / FQ_GROUP, NT = (N + 31) / 32;
    const int items = NT * S;
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nit = (items - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;  // >= 1
    // k-split z is the same for all of this WG's items (S == 1, or one item per WG)
    const int z = (int)blockIdx.x % S;
    const int gz0 = (int)((long)z * G / S), gz1 = (int)((long)(z + 1) * G / S);
    const int Gz = gz1 - gz0;
    const int ngmax = (Gz + NW - 1) / NW;
    const int ga = gz0 + (int)((long)wid * Gz / NW), gb = gz0 + (int)((long)(wid + 1) * Gz / NW);
    const int ng = gb - ga;  // groups per item for this wave (may be 0)
    const int n = ng * nit;  // blocks in this wave's sequence
    const bool even = (N & 1) == 0;  // w-scale rows are dword aligned: 4 blocks per staging DMA

    const int wl = decode_wave_lds(MT, XS, SS, ngmax, ngmax * IPW, M, even);
    char *ring = smem + wid * wl;
    char *ws_st = ring + D * C::SLOT;                                       // staged w-scales
    char *xs_st = ws_st + (SS ? 0 : decode_wsst_bytes(ngmax * IPW, even));  // staged x-scales
    char *x_st = xs_st + (SS ? 0 : decode_xsst_bytes(ngmax, MT));           // staged activations
    const int EM = M * 32;                                                  // live elements of a tile
    float *red = reinterpret_cast<float *>(smem + NW * wl);                 // [2][NW][M*32]
    int *flag = reinterpret_cast<int *>(red + 2 * NW * EM);

    auto item_tile = [&](int it) { return ((int)blockIdx.x + it * (int)gridDim.x) / S; };

    if (n > 0 && !SS && !(ABL & 8)) {  // ---- prologue staging (issued first: the ring waits retire it in order)
        if (even) {
            for (int i0 = 0; i0 < n; i0 += 4) {  // w-scales: 4 blocks per instruction, 2 columns per lane
                const int i = i0 + (lane >> 4) < n ? i0 + (lane >> 4) : n - 1;
                const int col = 32 * item_tile(i / ng) + 2 * (lane & 15);
                __builtin_amdgcn_global_load_lds(ws + (long)(ga + i % ng) * N + (col < N ? col : N - 2),
                                                 LDS_PTR(ws_st + i0 * 64), 4, 0, 0);
            }
        } else {
            for (int i0 = 0; i0 < n; i0 += 2) {  // w-scales: 2 blocks per instruction, ushort per lane
                const int i = i0 + (lane >> 5) < n ? i0 + (lane >> 5) : n - 1;
                const int col = 32 * item_tile(i / ng) + (lane & 31);
                __builtin_amdgcn_global_load_lds(ws + (long)(ga + i % ng) * N + (col < N ? col : N - 1),
                                                 LDS_PTR(ws_st + i0 * 128), 2, 0, 0);
            }
        }
        for (int i0 = 0; i0 < ng; i0 += 64 / MT) {  // x-scales: MT per group, ushort per lane
            const int i = i0 + lane / MT, row = lane % MT;
            __builtin_amdgcn_global_load_lds(xs + (long)(ga + (i < ng ? i : ng - 1)) * M + (row < M ? row : M - 1),
                                             LDS_PTR(xs_st + i0 * MT * 4), 2, 0, 0);
        }
    }
    if (n > 0 && !XS && !(ABL & 8)) {  // activation rows: 8 lanes x 16 B per row and group
        const int per = 64 / (8 * M);
        for (int i0 = 0; i0 < ng; i0 += per) {
            const int i = i0 + lane / (8 * M), row = (lane / 8) % M;
            if (lane < per * 8 * M)
                __builtin_amdgcn_global_load_lds(xq + (long)row * K + (long)(ga + (i < ng ? i : ng - 1)) * FQ_GROUP + (lane & 7) * 16,
                                                 LDS_PTR(x_st + i0 * M * 128), 16, 0, 0);
        }
    }

    // ---- the ring over the wave's block sequence
    const char *wbytes = reinterpret_cast<const char *>(wpk) + lane * 16;
    auto issue = [&](int i, int slot) {
        const int t = item_tile(i / ng), g = ga + i % ng;
        char *dst = ring + slot * C::SLOT;
        const char *src = wbytes + ((long)t * G + g) * 3072;
#pragma unroll
        for (int r = 0; r < 3; r++)
            __builtin_amdgcn_global_load_lds(src + r * 1024, LDS_PTR(dst + r * 1024), 16, 0, 2 /*nt*/);
#pragma unroll
        for (int p = 0; p < C::XP; p++) {  // activation rows, 16 B per lane, row-major [MT][128]
            const int c = p * 64 + lane, row = c >> 3;
            __builtin_amdgcn_global_load_lds(xq + (long)(row < M ? row : M - 1) * K + (long)g * FQ_GROUP + (c & 7) * 16,
                                             LDS_PTR(dst + 3072 + p * 1024), 16, 0, 0);
        }
        if (SS) {  // 32 w-scales (ushort, lanes 0..31) and MT x-scales (ushort, lanes 0..MT-1)
            if (lane < 32) {
                const int col = 32 * t + lane;
                __builtin_amdgcn_global_load_lds(ws + (long)g * N + (col < N ? col : N - 1), LDS_PTR(dst + C::WS_OFF), 2, 0, 0);
            }
            if (lane < MT)
                __builtin_amdgcn_global_load_lds(xs + (long)g * M + (lane < M ? lane : M - 1), LDS_PTR(dst + C::XS_OFF), 2, 0, 0);
        }
    };
    const int pro = n < D ? n : D;
    for (int i = 0; i < pro; i++) issue(i, i);

    const int arow = (lane & 31) < M ? (lane & 31) : M - 1;  // rows >= M mirror row M-1 (unused)
    const int Npad = NT * 32;
    int i = 0;  // position in the wave's block sequence
    for (int it = 0; it < nit; it++) {
        const int t = item_tile(it);
        const int col = 32 * t + (lane & 31);
        float cur[16];
#pragma unroll
        for (int r = 0; r < 16; r++) cur[r] = 0.f;
        for (int j = 0; j < ng; j++, i++) {
            const int g = ga + j, slot = i % D;
            const int later = (n - 1 - i) < (D - 1) ? (n - 1 - i) : (D - 1);
            wait_ring<C::U>(later);  // this slot (and every older DMA, the staging included) landed
            const uint32_t sp = lds_addr(ring + slot * C::SLOT);
            const v4i p0 = ds_read_b128(sp + lane * 16);
            const v4i p1 = ds_read_b128(sp + 1024 + lane * 16);
            const v4i p2 = ds_read_b128(sp + 2048 + lane * 16);
            v4i a[4];
            const uint32_t xap = XS ? sp + 3072 + arow * FQ_GROUP + 16 * (lane >> 5)
                                    : lds_addr(x_st + (j * M + arow) * FQ_GROUP + 16 * (lane >> 5));
#pragma unroll
            for (int s = 0; s < 4; s++) a[s] = ds_read_b128(xap + 32 * s);
            const uint32_t wsa = SS ? sp + C::WS_OFF + 4 * (lane & 31)
                                    : lds_addr(ws_st) + (even ? i * 64 + 2 * (lane & 31) : i * 128 + 4 * (lane & 31));
            const uint32_t wsv = ds_read_u16(wsa);
            v4i xd[RV / 4];  // x-scales of rows 8q+4h .. +3, one per dword
            const uint32_t xsa = SS ? sp + C::XS_OFF : lds_addr(xs_st + j * MT * 4);
#pragma unroll
            for (int q = 0; q < RV / 4; q++) xd[q] = ds_read_b128(xsa + 4 * (8 * q + 4 * (lane >> 5)));
            // every read has landed, and the slot's bytes are in registers before its refill
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            if (i + D < n) issue(i + D, slot);

            if (ABL & 2) {
                cur[0] += (float)(p0[0] ^ p1[1] ^ p2[2] ^ a[3][0]) + (float)wsv + (float)xd[0][0];
                continue;
            }
            v16i acc = {0};
#pragma unroll
            for (int s = 0; s < 4; s++)
                acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[s], unpack_fq6(p0[s], p1[s], p2[s]), acc, 0, 0, 0);
            const __half2 w2 = __half2half2(__ushort_as_half((uint16_t)wsv));
#pragma unroll
            for (int q = 0; q < RV / 4; q++) {  // rows 8q+4h .. +3
                const uint32_t x01 = __builtin_amdgcn_perm((uint32_t)xd[q][1], (uint32_t)xd[q][0], 0x05040100u);
                const uint32_t x23 = __builtin_amdgcn_perm((uint32_t)xd[q][3], (uint32_t)xd[q][2], 0x05040100u);
                const __half2 p01 = __hmul2(*reinterpret_cast<const __half2 *>(&x01), w2);  // fp16-rounded
                const __half2 p23 = __hmul2(*reinterpret_cast<const __half2 *>(&x23), w2);  // scale product
                cur[4 * q + 0] = fmaf((float)acc[4 * q + 0], __low2float(p01), cur[4 * q + 0]);
                cur[4 * q + 1] = fmaf((float)acc[4 * q + 1], __high2float(p01), cur[4 * q + 1]);
                cur[4 * q + 2] = fmaf((float)acc[4 * q + 2], __low2float(p23), cur[4 * q + 2]);
                cur[4 * q + 3] = fmaf((float)acc[4 * q + 3], __high2float(p23), cur[4 * q + 3]);
            }
            if (DBG) {
#pragma unroll
                for (int r = 0; r < RV; r++) {
                    const int row = acc_row(r, lane);
                    if (row < M && col < N) acc_dbg[((long)row * N + col) * G + g] = acc[r] >> 2;
                }
            }
        }

        // ---- item end: fixed-order reduction of the NW waves' partial tiles through LDS
        // (raw s_barrier: the ring's DMA for the next item stays in flight; red is double-buffered
        // by item parity so a fast wave's next write cannot race this item's reads)
        float *rb = red + (it & 1) * NW * EM;
        if (ABL & 4) {
            if (lane < 32 && col < N) d[col] = f2h(cur[0]);
            continue;
        }
#pragma unroll
        for (int r = 0; r < RV; r++) {
            const int row = acc_row(r, lane);
            if (row < M) rb[wid * EM + row * 32 + (lane & 31)] = cur[r] * 0.25f;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        for (int e = threadIdx.x; e < EM; e += NW * 64) {
            float v = 0.f;
#pragma unroll
            for (int w = 0; w < NW; w++) v += rb[w * EM + e];
            const int row = e >> 5, nn = 32 * t + (e & 31);
            if (S == 1) {
                if (nn < N) d[(long)row * N + nn] = f2h(v);
            } else {
                __hip_atomic_store(&slabs[((long)z * M + row) * Npad + nn], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    if (S == 1 || (ABL & 4)) return;

    // ---- split-K fix-up (one item per WG when S > 1): write-through slabs, one ticket per WG,
    // the last arriver of the tile reduces the S slabs in z order
    const int t = item_tile(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t prev = __hip_atomic_fetch_add(&tickets[t], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = (prev == (uint32_t)(S - 1));
        if (last) __hip_atomic_store(&tickets[t], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *flag = last;
    }
    __syncthreads();
    if (!*flag) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keep the loads below the ticket
    for (int e = threadIdx.x; e < EM; e += NW * 64) {
        const int row = e >> 5, nn = 32 * t + (e & 31);
        float v = 0.f;
        for (int z0 = 0; z0 < S; z0 += 8) {  // 8 independent loads per round trip
            float part[8];
#pragma unroll
            for (int u = 0; u < 8; u++)
                part[u] = (z0 + u < S) ? __hip_atomic_load(&slabs[((long)(z0 + u) * M + row) * Npad + nn],
                                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                       : 0.f;
#pragma unroll
            for (int u = 0; u < 8; u++)
                if (z0 + u < S) v += part[u];
        }
        if (nn < N) d[(long)row * N + nn] = f2h(v);
    }
}

// =============================================================================================
// Prefill kernel (M > 32): MFMA-bound.  Block tile 128 x 128, 4 waves as 2 (M) x 2 (N), each
// wave 64 x 64 = 2 x 2 tiles of 32x32.  Per 128-wide group the block stages
//   A: 128 rows x 128 B int8, XOR-swizzled 16-B chunks (chunk ^ ((row>>1)&7)) so the
//      ds_read_b128 of 16 consecutive rows hits 16 distinct bank slots;
//   B: 4 n-tiles x 3 KiB packed weights, a straight copy of the fq6 blocks (3 planes x 64 lanes
//      x 16 B), read back as three conflict-free ds_read_b128 per n-tile and group;
//   the 128 x-scales and 128 w-scales of the group,
// in registers one group ahead (global loads issued before the MFMAs, LDS writes after), with
// two LDS buffers.  Group accumulators are int32; dequant is fp32 FMA per group.
// =============================================================================================
constexpr int PF_BM = 128, PF_BN = 128;
constexpr int PF_A_BYTES = PF_BM * FQ_GROUP;        // 16 KiB
constexpr int PF_B_BYTES = (PF_BN / 32) * 3072;  // 12 KiB
constexpr int PF_STAGE = PF_A_BYTES + PF_B_BYTES + 2 * PF_BM * 2 + 2 * PF_BN * 2;  // + xs, ws (x2 spare)

struct PrefillStage {
    uint4 a[4];
    uint4 b[3];
    uint16_t xsv, wsv;
};

__device__ __forceinline__ int a_lds_off(int row, int chunk) { return row * 128 + 16 * (chunk ^ ((row >> 1) & 7)); }

__device__ __forceinline__ void prefill_gload(PrefillStage &st, const int8_t *__restrict__ xq,
                                              const uint16_t *__restrict__ xs,
                                              const uint32_t *__restrict__ wpk,
                                              const uint16_t *__restrict__ ws, int M, int N, int K,
                                              int G, int m0, int t0, int NT, int g, int tid) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int c = tid + 256 * j;  // 1024 chunks of 16 B
        const int row = c >> 3, cc = c & 7;
        const int m = m0 + row;
        if (m < M) st.a[j] = *reinterpret_cast<const uint4 *>(xq + (long)m * K + g * FQ_GROUP + cc * 16);
        else st.a[j] = make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 3; j++) {
        const int c = tid + 256 * j;  // 768 chunks of 16 B = 4 n-tiles x 3 KiB
        const int nt = c / 192, within = c - nt * 192;
        const int t = t0 + nt;
        if (t < NT) st.b[j] = reinterpret_cast<const uint4 *>(wpk + (long)(t * G + g) * 768)[within];
        else st.b[j] = make_uint4(0, 0, 0, 0);
    }
    st.xsv = 0;
    st.wsv = 0;
    if (tid < PF_BM) {
        const int m = m0 + tid;
        if (m < M) st.xsv = xs[(long)g * M + m];
    } else {
        const int n = t0 * 32 + (tid - PF_BM);
        if (n < N) st.wsv = ws[(long)g * N + n];
    }
}

__device__ __forceinline__ void prefill_swrite(const PrefillStage &st, char *buf, int tid) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int c = tid + 256 * j;
        *reinterpret_cast<uint4 *>(buf + a_lds_off(c >> 3, c & 7)) = st.a[j];
    }
    char *bb = buf + PF_A_BYTES;
#pragma unroll
    for (int j = 0; j < 3; j++) *reinterpret_cast<uint4 *>(bb + (tid + 256 * j) * 16) = st.b[j];
    uint16_t *sc = reinterpret_cast<uint16_t *>(buf + PF_A_BYTES + PF_B_BYTES);
    sc[tid] = (tid < PF_BM) ? st.xsv : st.wsv;  // [0,128) x-scales, [128,256) w-scales
}

template <bool DBG>
__global__ __launch_bounds__(256, 2) void fq_gemm_prefill_kernel(
    const int8_t *__restrict__ xq, const uint16_t *__restrict__ xs, const uint32_t *__restrict__ wpk,
    const uint16_t *__restrict__ ws, int M, int N, int K, uint16_t *__restrict__ d,
    int32_t *__restrict__ acc_dbg) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int G = K / FQ_GROUP, NT = (N + 31) / 32;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;

    // XCD-aware block order: consecutive logical tiles on one XCD share A rows through its L2.
    const int nbx = gridDim.x, nby = gridDim.y, nwg = nbx * nby;
    const int bid = blockIdx.y * nbx + blockIdx.x;
    const int xcd = bid % 8, q = nwg / 8, rr = nwg % 8;
    const int lid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / 8;
    const int bn = lid % nby, bm = lid / nby;  // N fastest: blocks sharing an A panel are adjacent
    const int m0 = bm * PF_BM, t0 = bn * (PF_BN / 32);

    float out[2][2][16];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int j = 0; j < 2; j++)
#pragma unroll
            for (int r = 0; r < 16; r++) out[i][j][r] = 0.f;

    PrefillStage st;
    prefill_gload(st, xq, xs, wpk, ws, M, N, K, G, m0, t0, NT, 0, tid);
    prefill_swrite(st, smem, tid);
    __syncthreads();

    for (int g = 0; g < G; g++) {
        char *buf = smem + (g & 1) * PF_STAGE;
        if (g + 1 < G) prefill_gload(st, xq, xs, wpk, ws, M, N, K, G, m0, t0, NT, g + 1, tid);

        v4i bp[2][3];
#pragma unroll
        for (int ni = 0; ni < 2; ni++) {
            const char *bsrc = buf + PF_A_BYTES + (wn * 2 + ni) * 3072 + lane * 16;
#pragma unroll
            for (int r = 0; r < 3; r++) bp[ni][r] = *reinterpret_cast<const v4i *>(bsrc + r * 1024);
        }
        v16i acc[2][2];
#pragma unroll
        for (int s = 0; s < 4; s++) {
            v4i a[2], b[2];
#pragma unroll
            for (int mi = 0; mi < 2; mi++) {
                const int row = wm * 64 + mi * 32 + (lane & 31);
                a[mi] = *reinterpret_cast<const v4i *>(buf + a_lds_off(row, 2 * s + (lane >> 5)));
            }
#pragma unroll
            for (int ni = 0; ni < 2; ni++) b[ni] = unpack_fq6(bp[ni][0][s], bp[ni][1][s], bp[ni][2][s]);
#pragma unroll
            for (int mi = 0; mi < 2; mi++)
#pragma unroll
                for (int ni = 0; ni < 2; ni++) {
                    if (s == 0) acc[mi][ni] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[mi], b[ni], v16i{0}, 0, 0, 0);
                    else acc[mi][ni] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
                }
        }

        const uint16_t *sc = reinterpret_cast<const uint16_t *>(buf + PF_A_BYTES + PF_B_BYTES);
#pragma unroll
        for (int ni = 0; ni < 2; ni++) {
            const int col = wn * 64 + ni * 32 + (lane & 31);
            const __half2 w2 = __half2half2(__ushort_as_half(sc[PF_BM + col]));
#pragma unroll
            for (int mi = 0; mi < 2; mi++) {
                const uint16_t *xr = sc + wm * 64 + mi * 32 + 4 * (lane >> 5);
#pragma unroll
                for (int q4 = 0; q4 < 4; q4++) {
                    const uint2 xv = *reinterpret_cast<const uint2 *>(xr + 8 * q4);
                    const __half2 p01 = __hmul2(*reinterpret_cast<const __half2 *>(&xv.x), w2);
                    const __half2 p23 = __hmul2(*reinterpret_cast<const __half2 *>(&xv.y), w2);
                    float *o = out[mi][ni] + 4 * q4;
                    const v16i &c = acc[mi][ni];
                    o[0] = fmaf((float)c[4 * q4 + 0], __low2float(p01), o[0]);
                    o[1] = fmaf((float)c[4 * q4 + 1], __high2float(p01), o[1]);
                    o[2] = fmaf((float)c[4 * q4 + 2], __low2float(p23), o[2]);
                    o[3] = fmaf((float)c[4 * q4 + 3], __high2float(p23), o[3]);
                }
                if (DBG) {
                    const int n = t0 * 32 + col;
#pragma unroll
                    for (int r = 0; r < 16; r++) {
                        const int m = m0 + wm * 64 + mi * 32 + acc_row(r, lane);
                        if (m < M && n < N) acc_dbg[((long)m * N + n) * G + g] = acc[mi][ni][r] >> 2;
                    }
                }
            }
        }
        if (g + 1 < G) {
            prefill_swrite(st, smem + ((g + 1) & 1) * PF_STAGE, tid);
        }
        __syncthreads();
    }

#pragma unroll
    for (int mi = 0; mi < 2; mi++)
#pragma unroll
        for (int ni = 0; ni < 2; ni++) {
            const int n = t0 * 32 + wn * 64 + ni * 32 + (lane & 31);
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int m = m0 + wm * 64 + mi * 32 + acc_row(r, lane);
                if (m < M && n < N) d[(long)m * N + n] = f2h(out[mi][ni][r] * 0.25f);
            }
        }
}

// =============================================================================================
// Host side: plan + launch
// =============================================================================================
struct DecodePlan {
    int MT, NW, S, grid, IPW, XS, SS;
};

// waves per WG (one WG per CU): 8 for M <= 8, 4 for the larger M > 8 ring slots
template <int MT> struct DecodeWaves { static constexpr int NW = MT <= 8 ? 8 : 4; };
static int decode_waves(int MT) { return MT <= 8 ? 8 : 4; }
static const size_t kLdsMax = 160 * 1024;

static int device_cus() {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
    }
    return cus;
}

static size_t decode_lds_bytes(const DecodePlan &p, int M, int N, int K) {
    const int Gz = (K / FQ_GROUP + p.S - 1) / p.S;
    const int ngmax = (Gz + p.NW - 1) / p.NW;
    return (size_t)p.NW * decode_wave_lds(p.MT, p.XS, p.SS, ngmax, ngmax * p.IPW, M, (N & 1) == 0) +
           (size_t)2 * p.NW * M * 32 * 4 + 16;
}

static DecodePlan decode_plan(int M, int N, int K) {
    DecodePlan p;
    p.MT = M <= 4 ? 4 : (M <= 8 ? 8 : (M <= 16 ? 16 : 32));
    p.NW = decode_waves(p.MT);
    const int NT = (N + 31) / 32, G = K / FQ_GROUP;
    const int cus = device_cus();
    // Few tiles: split K so that ~one item per CU streams (never below one group per wave).
    // Many tiles: whole tiles, WGs persistent over them (items w, w + grid, ...).
    int S = 1;
    if (NT < cus) {
        S = cus / NT;
        int cap = G / p.NW;
        if (cap < 1) cap = 1;
        if (S > cap) S = cap;
        if (S < 1) S = 1;
    }
    p.S = S;
    const int items = NT * S;
    p.grid = items < cus ? items : cus;
    p.IPW = (items + p.grid - 1) / p.grid;
    // staging choice: the most staged variant that fits LDS
    const int modes[3][2] = {{0, 0}, {1, 0}, {1, 1}};
    for (int m = (p.MT <= 4 ? 0 : 1); m < 3; m++) {
        p.XS = modes[m][0];
        p.SS = modes[m][1];
        if (decode_lds_bytes(p, M, N, K) <= kLdsMax) break;
    }
    return p;
}

static const size_t kTicketBytes = 256 * 1024;  // tickets for up to 65536 n-tiles

extern "C" size_t fq_gemm_workspace_bytes(int M, int N, int K) {
    if (M <= 0 || N <= 0 || K <= 0 || K % FQ_GROUP) return 0;
    if (M > 32) return 0;
    DecodePlan p = decode_plan(M, N, K);
    if (p.S == 1) return 0;
    const size_t Npad = (size_t)((N + 31) / 32) * 32;
    return kTicketBytes + (size_t)p.S * M * Npad * sizeof(float);
}

extern "C" fq_status fq_workspace_init(void *workspace, size_t bytes, fq_stream_t stream) {
    if (!bytes) return FQ_OK;
    if (!workspace) return FQ_ERR_NULL;
    if (hipMemsetAsync(workspace, 0, bytes < kTicketBytes ? bytes : kTicketBytes, (hipStream_t)stream) != hipSuccess)
        return FQ_ERR_HIP;
    return FQ_OK;
}

#ifdef FQ_DEV_ABLATION
#include <cstdlib>
static int dev_ablation() {
    const char *e = getenv("FQ_DEV_ABLATION");
    return e ? atoi(e) : 0;
}
#endif

template <int MT, int XS, int SS, bool DBG>
static fq_status launch_decode(const DecodePlan &p, const int8_t *xq, const uint16_t *xs,
                               const void *wpk, const uint16_t *ws, int M, int N, int K, uint16_t *d,
                               int32_t *acc_dbg, void *workspace, hipStream_t stream) {
    constexpr int NW = DecodeWaves<MT>::NW;
    uint32_t *tickets = p.S > 1 ? (uint32_t *)workspace : nullptr;
    float *slabs = p.S > 1 ? (float *)((char *)workspace + kTicketBytes) : nullptr;
    const size_t lds = decode_lds_bytes(p, M, N, K);
#ifdef FQ_DEV_ABLATION
    if (!DBG && MT == 4 && XS == 0 && SS == 0) {
        const int abl = dev_ablation();
#define FQ_ABL(v)                                                                                          \
    if (abl == v) {                                                                                          \
        hipLaunchKernelGGL((fq_gemm_decode_kernel<MT, NW, XS, SS, DBG, v>), dim3(p.grid), dim3(NW * 64), lds,  \
                           stream, xq, xs, (const uint32_t *)wpk, ws, M, N, K, d, acc_dbg, slabs, tickets,    \
                           p.S, p.IPW);                                                                      \
        FQ_LAUNCH_CHECK();                                                                                   \
        return FQ_OK;                                                                                        \
    }
        FQ_ABL(2) FQ_ABL(4) FQ_ABL(6) FQ_ABL(8) FQ_ABL(14)
#undef FQ_ABL
    }
#endif
    hipLaunchKernelGGL((fq_gemm_decode_kernel<MT, NW, XS, SS, DBG>), dim3(p.grid), dim3(NW * 64), lds, stream,
                       xq, xs, (const uint32_t *)wpk, ws, M, N, K, d, acc_dbg, slabs, tickets, p.S, p.IPW);
    FQ_LAUNCH_CHECK();
    return FQ_OK;
}

template <int MT, bool DBG>
static fq_status dispatch_modes(const DecodePlan &p, const int8_t *xq, const uint16_t *xs, const void *wpk,
                                const uint16_t *ws, int M, int N, int K, uint16_t *d, int32_t *acc_dbg,
                                void *workspace, hipStream_t stream) {
    if (MT <= 4 && p.XS == 0) return launch_decode<MT, 0, 0, DBG>(p, xq, xs, wpk, ws, M, N, K, d, acc_dbg, workspace, stream);
    if (p.SS == 0) return launch_decode<MT, 1, 0, DBG>(p, xq, xs, wpk, ws, M, N, K, d, acc_dbg, workspace, stream);
    return launch_decode<MT, 1, 1, DBG>(p, xq, xs, wpk, ws, M, N, K, d, acc_dbg, workspace, stream);
}

template <bool DBG>
static fq_status dispatch_decode(const DecodePlan &p, const int8_t *xq, const uint16_t *xs,
                                 const void *wpk, const uint16_t *ws, int M, int N, int K, uint16_t *d,
                                 int32_t *acc_dbg, void *workspace, hipStream_t stream) {
    if (decode_lds_bytes(p, M, N, K) > kLdsMax) return FQ_ERR_SHAPE;  // cannot happen for K <= 2^20
    switch (p.MT) {
        case 4: return dispatch_modes<4, DBG>(p, xq, xs, wpk, ws, M, N, K, d, acc_dbg, workspace, stream);
        case 8: return dispatch_modes<8, DBG>(p, xq, xs, wpk, ws, M, N, K, d, acc_dbg, workspace, stream);
        case 16: return dispatch_modes<16, DBG>(p, xq, xs, wpk, ws, M, N, K, d, acc_dbg, workspace, stream);
        default: return dispatch_modes<32, DBG>(p, xq, xs, wpk, ws, M, N, K, d, acc_dbg, workspace, stream);
    }
}

extern "C" fq_status fq_gemm_w6ax(const int8_t *xq, const uint16_t *xs, const void *w_packed,
                                  const uint16_t *ws, int M, int N, int K, int abits, uint16_t *d,
                                  int32_t *acc_dbg, void *workspace, size_t workspace_bytes,
                                  fq_stream_t stream) {
    if (!xq || !xs || !w_packed || !ws || !d) return FQ_ERR_NULL;
    if (M <= 0 || N <= 0 || K <= 0 || K % FQ_GROUP) return FQ_ERR_SHAPE;
    if ((size_t)((N + 31) / 32) > kTicketBytes / 4) return FQ_ERR_SHAPE;
    if (abits != 6 && abits != 8) return FQ_ERR_BITS;
    // The kernels are bit-width agnostic (int8 activations, values bounded by abits); abits is
    // validated for API parity with FLEXQGEMMWrapper(X_BITS, W_BITS, SIGNED).
    hipStream_t s = (hipStream_t)stream;
    if (M <= 32) {
        DecodePlan p = decode_plan(M, N, K);
        const size_t need = fq_gemm_workspace_bytes(M, N, K);
        if (need && (!workspace || workspace_bytes < need)) return FQ_ERR_WORKSPACE;
        return acc_dbg ? dispatch_decode<true>(p, xq, xs, w_packed, ws, M, N, K, d, acc_dbg, workspace, s)
                       : dispatch_decode<false>(p, xq, xs, w_packed, ws, M, N, K, d, acc_dbg, workspace, s);
    }
    const int NT = (N + 31) / 32;
    dim3 grid((M + PF_BM - 1) / PF_BM, (NT + 3) / 4);
    const size_t lds = 2 * (size_t)PF_STAGE;
    if (acc_dbg)
        hipLaunchKernelGGL(fq_gemm_prefill_kernel<true>, grid, dim3(256), lds, s, xq, xs,
                           (const uint32_t *)w_packed, ws, M, N, K, d, acc_dbg);
    else
        hipLaunchKernelGGL(fq_gemm_prefill_kernel<false>, grid, dim3(256), lds, s, xq, xs,
                           (const uint32_t *)w_packed, ws, M, N, K, d, acc_dbg);
    FQ_LAUNCH_CHECK();
    return FQ_OK;
}
