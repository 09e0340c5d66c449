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
//   grid  = (n-tiles of 32 columns, S k-splits); block = NW waves splitting the WG's groups.
//   Each wave streams 3 KiB of packed weights per group as 4 x dwordx3 loads per lane (768 B
//   contiguous per wave instruction), one group ahead in registers.  Partial sums are reduced
//   across the WG's waves through LDS in a fixed order; with S > 1 the WG writes an fp32 slab
//   and the last-arriving WG of the n-tile (agent-scope release/acquire, Guideline 16) sums the
//   S slabs in order and writes fp16.  Deterministic: no float atomics.
// =============================================================================================
typedef unsigned u3 __attribute__((ext_vector_type(3)));

struct DecodeFrag {
    u3 w[4];
    v4i a[4];
    uint16_t ws;
};

template <int MT>
__device__ __forceinline__ void decode_load(DecodeFrag &f, const int8_t *__restrict__ xq,
                                            const uint32_t *__restrict__ wpk,
                                            const uint16_t *__restrict__ ws, int M, int N, int K,
                                            int G, int t, int g, int lane) {
    const u3 *wp = reinterpret_cast<const u3 *>(wpk + ((long)(t * G + g) * 4) * 192) + lane;
#pragma unroll
    for (int s = 0; s < 4; s++) f.w[s] = __builtin_nontemporal_load(wp + s * 64);
    const int row = lane & 31;
    const int8_t *ap = xq + (long)row * K + g * FQ_GROUP + 16 * (lane >> 5);
#pragma unroll
    for (int s = 0; s < 4; s++) {
        if (row < M) f.a[s] = *reinterpret_cast<const v4i *>(ap + 32 * s);
        else f.a[s] = v4i{0, 0, 0, 0};
    }
    const int n = 32 * t + (lane & 31);
    f.ws = (n < N) ? ws[(long)g * N + n] : (uint16_t)0;
}

template <int MT, bool DBG>
__device__ __forceinline__ void decode_compute(const DecodeFrag &f, const uint16_t *xs_s, int RS,
                                               int gl, int g, int G, int lane, int M, int N, int t,
                                               float (&out)[16], int32_t *__restrict__ acc_dbg) {
    constexpr int RV = RowRegs<MT>::RV;
    v16i acc = {0};
#pragma unroll
    for (int s = 0; s < 4; s++) {
        v4i b = unpack_fq6(f.w[s].x, f.w[s].y, f.w[s].z);
        acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(f.a[s], b, acc, 0, 0, 0);
    }
    const __half2 w2 = __half2half2(__ushort_as_half(f.ws));
    const uint16_t *xr = xs_s + gl * RS + 4 * (lane >> 5);
#pragma unroll
    for (int q = 0; q < RV / 4; q++) {
        const uint2 xv = *reinterpret_cast<const uint2 *>(xr + 8 * q);  // rows 8q+4h .. +3
        const __half2 x01 = *reinterpret_cast<const __half2 *>(&xv.x);
        const __half2 x23 = *reinterpret_cast<const __half2 *>(&xv.y);
        const __half2 p01 = __hmul2(x01, w2);  // the fp16-rounded scale product (__hmul2)
        const __half2 p23 = __hmul2(x23, w2);
        out[4 * q + 0] = fmaf((float)acc[4 * q + 0], __low2float(p01), out[4 * q + 0]);
        out[4 * q + 1] = fmaf((float)acc[4 * q + 1], __high2float(p01), out[4 * q + 1]);
        out[4 * q + 2] = fmaf((float)acc[4 * q + 2], __low2float(p23), out[4 * q + 2]);
        out[4 * q + 3] = fmaf((float)acc[4 * q + 3], __high2float(p23), out[4 * q + 3]);
    }
    if (DBG) {
        const int n = 32 * t + (lane & 31);
#pragma unroll
        for (int r = 0; r < RV; r++) {
            const int row = acc_row(r, lane);
            if (row < M && n < N) acc_dbg[((long)row * N + n) * G + g] = acc[r] >> 2;
        }
    }
}

template <int MT, int NW, bool DBG>
__global__ __launch_bounds__(NW * 64) void fq_gemm_decode_kernel(
    const int8_t *__restrict__ xq, const uint16_t *__restrict__ xs, const uint32_t *__restrict__ wpk,
    const uint16_t *__restrict__ ws, int M, int N, int K, uint16_t *__restrict__ d,
    int32_t *__restrict__ acc_dbg, float *__restrict__ partial, uint32_t *__restrict__ counters,
    int S) {
    constexpr int RV = RowRegs<MT>::RV;
    constexpr int RS = MT < 8 ? 8 : MT;  // LDS row stride of the staged x-scales
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int G = K / FQ_GROUP;
    const int t = blockIdx.x, z = blockIdx.y;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int gz0 = (int)((long)z * G / S), gz1 = (int)((long)(z + 1) * G / S);
    const int Gz = gz1 - gz0;

    // LDS carve: [Gz][RS] fp16 x-scales | [NW][MT][32] fp32 reduction | flag
    uint16_t *xs_s = reinterpret_cast<uint16_t *>(smem);
    const int xs_bytes = ((Gz * RS * 2) + 15) & ~15;
    float *red = reinterpret_cast<float *>(smem + xs_bytes);
    int *flag = reinterpret_cast<int *>(smem + xs_bytes + NW * MT * 32 * 4);

    for (int i = threadIdx.x; i < Gz * RS; i += NW * 64) {
        const int gl = i / RS, row = i % RS;
        xs_s[i] = (row < M) ? xs[(long)(gz0 + gl) * M + row] : (uint16_t)0;
    }
    __syncthreads();

    const int g0 = gz0 + (int)((long)wid * Gz / NW), g1 = gz0 + (int)((long)(wid + 1) * Gz / NW);
    float out[16];
#pragma unroll
    for (int r = 0; r < 16; r++) out[r] = 0.f;

    if (g0 < g1) {
        DecodeFrag fa, fb;
        decode_load<MT>(fa, xq, wpk, ws, M, N, K, G, t, g0, lane);
        int g = g0;
        for (; g + 1 < g1; g += 2) {
            decode_load<MT>(fb, xq, wpk, ws, M, N, K, G, t, g + 1, lane);
            decode_compute<MT, DBG>(fa, xs_s, RS, g - gz0, g, G, lane, M, N, t, out, acc_dbg);
            if (g + 2 < g1) decode_load<MT>(fa, xq, wpk, ws, M, N, K, G, t, g + 2, lane);
            decode_compute<MT, DBG>(fb, xs_s, RS, g + 1 - gz0, g + 1, G, lane, M, N, t, out, acc_dbg);
        }
        if (g < g1) decode_compute<MT, DBG>(fa, xs_s, RS, g - gz0, g, G, lane, M, N, t, out, acc_dbg);
    }

    // fixed-order reduction of the NW waves' partial tiles
#pragma unroll
    for (int r = 0; r < RV; r++) {
        const int row = acc_row(r, lane);
        if (row < MT) red[(wid * MT + row) * 32 + (lane & 31)] = out[r] * 0.25f;
    }
    __syncthreads();

    const int Npad = ((N + 31) / 32) * 32;
    for (int i = threadIdx.x; i < MT * 32; i += NW * 64) {
        const int row = i >> 5, col = i & 31;
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < NW; w++) v += red[w * MT * 32 + i];
        const int n = 32 * t + col;
        if (row < M) {
            if (S == 1) {
                if (n < N) d[(long)row * N + n] = f2h(v);
            } else {
                partial[((long)z * M + row) * Npad + n] = v;
            }
        }
    }
    if (S == 1) return;

    // split-K fix-up: publish the slab, the last arriver of this n-tile reduces in z order
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t prev = __hip_atomic_fetch_add(&counters[t], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = (prev == (uint32_t)(S - 1));
        if (last) {
            __hip_atomic_store(&counters[t], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        *flag = last;
    }
    __syncthreads();
    if (!*flag) return;
    for (int i = threadIdx.x; i < M * 32; i += NW * 64) {
        const int row = i >> 5, col = i & 31;
        const int n = 32 * t + col;
        float v = 0.f;
        for (int zz = 0; zz < S; zz++) v += partial[((long)zz * M + row) * Npad + n];
        if (n < N) d[(long)row * N + n] = f2h(v);
    }
}

// =============================================================================================
// Prefill kernel (M > 32): MFMA-bound.  Block tile 128 x 128, 4 waves as 2 (M) x 2 (N), each
// wave 64 x 64 = 2 x 2 tiles of 32x32.  Per 128-wide group the block stages
//   A: 128 rows x 128 B int8, XOR-swizzled 16-B chunks (chunk ^ ((row>>1)&7)) so the
//      ds_read_b128 of 16 consecutive rows hits 16 distinct bank slots;
//   B: 4 n-tiles x 4 k-steps x 64 lanes x 12 B packed weights, padded to 16 B per lane;
//   the 128 x-scales and 128 w-scales of the group,
// in registers one group ahead (global loads issued before the MFMAs, LDS writes after), with
// two LDS buffers.  Group accumulators are int32; dequant is fp32 FMA per group.
// =============================================================================================
constexpr int PF_BM = 128, PF_BN = 128;
constexpr int PF_A_BYTES = PF_BM * FQ_GROUP;        // 16 KiB
constexpr int PF_B_BYTES = (PF_BN / 32) * 4 * 64 * 16;  // 16 KiB
constexpr int PF_STAGE = PF_A_BYTES + PF_B_BYTES + 2 * PF_BM * 2 + 2 * PF_BN * 2;  // + xs, ws (x2 spare)

struct PrefillStage {
    uint4 a[4];
    uint3 b[4];
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
    for (int j = 0; j < 4; j++) {
        const int slot = tid + 256 * j;  // (nt, s, lane) = 4 x 4 x 64
        const int nt = slot >> 8, sl = slot & 255;
        const int t = t0 + nt;
        if (t < NT) st.b[j] = reinterpret_cast<const uint3 *>(wpk + ((long)(t * G + g) * 4) * 192)[sl];
        else st.b[j] = make_uint3(0, 0, 0);
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
    for (int j = 0; j < 4; j++) {
        const int slot = tid + 256 * j;
        *reinterpret_cast<uint3 *>(bb + slot * 16) = st.b[j];
    }
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
            for (int ni = 0; ni < 2; ni++) {
                const int nt = wn * 2 + ni;
                const uint4 p = *reinterpret_cast<const uint4 *>(buf + PF_A_BYTES + ((nt * 4 + s) * 64 + lane) * 16);
                b[ni] = unpack_fq6(p.x, p.y, p.z);
            }
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
    int MT, NW, S;
};

static DecodePlan decode_plan(int M, int N, int K) {
    DecodePlan p;
    p.MT = M <= 4 ? 4 : (M <= 8 ? 8 : (M <= 16 ? 16 : 32));
    p.NW = 4;
    const int NT = (N + 31) / 32, G = K / FQ_GROUP;
    // aim for >= 2048 waves (8 per CU) with at least one group per wave
    int S = (2048 + NT * p.NW - 1) / (NT * p.NW);
    const int smax = G / p.NW > 0 ? G / p.NW : 1;
    if (S > smax) S = smax;
    if (S < 1) S = 1;
    p.S = S;
    return p;
}

static const int kCounterBytes = 256 * 1024;  // counters for up to 65536 n-tiles

extern "C" size_t fq_gemm_workspace_bytes(int M, int N, int K) {
    if (M <= 0 || N <= 0 || K <= 0 || K % FQ_GROUP) return 0;
    if (M > 32) return 0;
    DecodePlan p = decode_plan(M, N, K);
    if (p.S == 1) return 0;
    const size_t Npad = (size_t)((N + 31) / 32) * 32;
    return kCounterBytes + (size_t)p.S * M * Npad * sizeof(float);
}

extern "C" fq_status fq_workspace_init(void *workspace, size_t bytes, fq_stream_t stream) {
    if (!bytes) return FQ_OK;
    if (!workspace) return FQ_ERR_NULL;
    if (hipMemsetAsync(workspace, 0, bytes < (size_t)kCounterBytes ? bytes : (size_t)kCounterBytes,
                       (hipStream_t)stream) != hipSuccess)
        return FQ_ERR_HIP;
    return FQ_OK;
}

template <int MT, int NW, bool DBG>
static fq_status launch_decode(const DecodePlan &p, const int8_t *xq, const uint16_t *xs,
                               const void *wpk, const uint16_t *ws, int M, int N, int K, uint16_t *d,
                               int32_t *acc_dbg, void *workspace, hipStream_t stream) {
    const int NT = (N + 31) / 32, G = K / FQ_GROUP;
    const int Gz = (G + p.S - 1) / p.S;
    const int RS = MT < 8 ? 8 : MT;
    const size_t lds = (((size_t)Gz * RS * 2 + 15) & ~(size_t)15) + (size_t)NW * MT * 32 * 4 + 16;
    uint32_t *counters = nullptr;
    float *partial = nullptr;
    if (p.S > 1) {
        counters = (uint32_t *)workspace;
        partial = (float *)((char *)workspace + kCounterBytes);
    }
    hipLaunchKernelGGL((fq_gemm_decode_kernel<MT, NW, DBG>), dim3(NT, p.S), dim3(NW * 64), lds, stream,
                       xq, xs, (const uint32_t *)wpk, ws, M, N, K, d, acc_dbg, partial, counters, p.S);
    FQ_LAUNCH_CHECK();
    return FQ_OK;
}

template <bool DBG>
static fq_status dispatch_decode(const DecodePlan &p, const int8_t *xq, const uint16_t *xs,
                                 const void *wpk, const uint16_t *ws, int M, int N, int K, uint16_t *d,
                                 int32_t *acc_dbg, void *workspace, hipStream_t stream) {
    switch (p.MT) {
        case 4: return launch_decode<4, 4, DBG>(p, xq, xs, wpk, ws, M, N, K, d, acc_dbg, workspace, stream);
        case 8: return launch_decode<8, 4, DBG>(p, xq, xs, wpk, ws, M, N, K, d, acc_dbg, workspace, stream);
        case 16: return launch_decode<16, 4, DBG>(p, xq, xs, wpk, ws, M, N, K, d, acc_dbg, workspace, stream);
        default: return launch_decode<32, 4, DBG>(p, xq, xs, wpk, ws, M, N, K, d, acc_dbg, workspace, stream);
    }
}

extern "C" fq_status fq_gemm_w6ax(const int8_t *xq, const uint16_t *xs, const void *w_packed,
                                  const uint16_t *ws, int M, int N, int K, int abits, uint16_t *d,
                                  int32_t *acc_dbg, void *workspace, size_t workspace_bytes,
                                  fq_stream_t stream) {
    if (!xq || !xs || !w_packed || !ws || !d) return FQ_ERR_NULL;
    if (M <= 0 || N <= 0 || K <= 0 || K % FQ_GROUP) return FQ_ERR_SHAPE;
    if ((N + 31) / 32 > kCounterBytes / 4) return FQ_ERR_SHAPE;
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
