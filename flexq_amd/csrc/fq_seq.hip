// fq_seq.hip -- a chain of decode linears (quantize + W6Ax GEMM each) in ONE persistent launch.
//
// What it replaces: a sequence of FLEXQGEMMWrapper::gemm(const half* A ...) calls on one stream
// (e2e .../flexqgemm/flexq_gemm_wrapper.cu:99-122), as FT issues them per decoder layer
// (FfnLayer.cc:371-401,521-561, LlamaV2ContextAttentionLayer.cc:145-161,506-522).  Each linear
// computes exactly what fq_linear_w6ax computes on its fused decode path (same group ranges per
// wave, same quantizer, same summation order), so the outputs are bit-identical to launching
// the linears one by one with a one-WG-per-tile plan (S = 1).
//
// Why one launch: at decode sizes a linear streams 13-70 MB in ~5-12 us, and every launch paid
// ~3 us of fixed cost (launch gap, prologue DMA burst, first HBM round trip, and the tail where
// early CUs sit idle).  Here the grid stays resident (one 576-thread WG per CU)
// and walks the chain:
//   * 8 streaming waves per WG own contiguous group ranges of the WG's 16-column tiles, exactly
//     as fq_gemm_decode_kernel<FUSE>.  As soon as a wave has consumed its last block of linear j
//     it issues up to P (<= 8) ring blocks + the w-scale staging of linear j+1 -- weights do not
//     depend on activations -- so the tail of linear j and the hand-off below overlap HBM
//     traffic of linear j+1.  In steady state the ring keeps SQ_DIST blocks in flight (the
//     decode kernel's measured optimum).
//   * a 9th "control" wave reduces the 8 partial tiles, stores d with write-through (sc1) 8-byte
//     stores, drains them, and adds one agent-scope arrival to linear j's counter; before linear
//     j+1 it polls (sc1, bounded) the counter of the linear j+1 depends on and releases its WG
//     with a barrier; the streaming waves then read x_{j+1} with sc1 loads and quantize it.
//     This is row 1 of MI355X_MICROARCH.md "Hand-offs measured with sc1 loads" (one lane per
//     storing WG, agent atomic add, sc1 poll by the wave that then joins a barrier, 8-B sc1
//     stores, 8-B sc1 loads, hipMalloc memory, one WG per CU).
//   * dependencies are found on the host from byte-range overlaps (RAW x_j/d_i, WAR d_j/x_i,
//     WAW d_j/d_i); a linear with none starts without waiting.
//   * counters are left zero: the WG whose arrival completes the LAST linear resets them (every
//     WG has passed all of its polls by then).  A poll that spins past its bound sets the
//     error word and gives up (results then undefined, never a hang).
#include <algorithm>

#include "fq_lds.h"

struct FqSeqDesc {          // one linear of the chain; built on the host, read-only in the launch
    const uint16_t *x;      // fp16 [M][ldx]
    const char *w;          // weight image
    uint16_t *d;            // fp16 [M][N]
    int N, K, ldx, abits;
    int NT, G, iq, ir;      // 16-column tiles, 128-groups, tiles / grid, tiles % grid
    int dep;                // wait for linear `dep` to complete (-1: none)
    int pad;
};
static_assert(sizeof(FqSeqDesc) == 64, "descriptor layout");

// hand-off words and payload go through GLOBAL (address space 1) pointers: flat_ accesses are
// not among the measured sc1 hand-off forms (cdna_hip_programming.md Guideline 16)
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) uint32_t gu32;

constexpr int SQ_NW = 8;                      // streaming waves
constexpr int SQ_THREADS = (SQ_NW + 1) * 64;  // + the control wave
constexpr int SQ_DIST = 3;                    // steady-state ring distance (blocks in flight)
constexpr int SQ_PMAX = 8;                    // ring slots / prologue prefetch per wave, at most
constexpr int SQ_MT = 4;                      // rows per MFMA row group used (M <= 4)
constexpr int SQ_XSR = 16;                    // x-scale record per group in LDS (dwords)
constexpr unsigned SQ_SPIN_MAX = 1u << 21;    // poll bound (~1 s), then the error word is set

#ifdef FQ_DEV_ABLATION
// development timeline (tools/seq_stamps.py): per (WG, linear) s_memrealtime stamps (100 MHz)
//   control wave: 0 released past B2, 1 past B1, 7 stores drained, 2 flag stored
//   wave 0: 3 x quantized, 4 first block landed, 5 stream done; wave 7: 6 stream done
constexpr int SQ_STAMP_L = 160;
__device__ unsigned long long g_sq_stamps[256 * SQ_STAMP_L * 8];
#define SQ_STAMP(j, k)                                                                     \
    if (lane == 0 && bid < 256 && (j) < SQ_STAMP_L) {                                       \
        g_sq_stamps[(bid * SQ_STAMP_L + (j)) * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); \
    }
#else
#define SQ_STAMP(j, k)
#endif

__global__ __launch_bounds__(SQ_THREADS) void fq_seq_kernel(const FqSeqDesc *__restrict__ descs, int L, int M,
                                                           gu32 *flag, gu32 *err, int P, int wl, int wsst,
                                                           int xsst, int redoff) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int bid = blockIdx.x, grid = gridDim.x;
    const int EM = M * 16;
    float *red = reinterpret_cast<float *>(smem + redoff);  // [item][wave][M*16]

    if (wid == SQ_NW) {
        // ================= control wave: reduce, publish, arrive; poll the next dependency
        // one sweep: lane l checks the flags of WGs 4l .. 4l+3 (16 B, two 8-B sc1 loads)
        auto flags_reach = [&](uint32_t target) -> bool {
            const int w0 = 4 * lane;
            bool ok = true;
            if (w0 < grid) {
                const unsigned long long a = __hip_atomic_load((gu64 *)(flag + w0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned long long b = __hip_atomic_load((gu64 *)(flag + w0 + 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t f[4] = {(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)};
#pragma unroll
                for (int k = 0; k < 4; k++) ok &= (w0 + k >= grid) || f[k] >= target;
            }
            return __builtin_amdgcn_ballot_w64(!ok) == 0;
        };
        auto wait_flags = [&](uint32_t target) {  // bounded: the error word, never a hang
            for (unsigned spins = 0; !flags_reach(target);) {
                __builtin_amdgcn_s_sleep(2);
                if (++spins == SQ_SPIN_MAX) {
                    if (lane == 0) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
            }
        };
        for (int j = 0; j < L; j++) {
            const int dep = descs[j].dep;
            if (dep >= 0) wait_flags((uint32_t)dep + 1);  // ONE wave polls the producers' flags
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (compiler only: loads stay below)
            __builtin_amdgcn_s_barrier();  // B2: the streaming waves may read x_j / overwrite d_j
            SQ_STAMP(j, 0);
            __builtin_amdgcn_s_barrier();  // B1: partial tiles of linear j are in red
            SQ_STAMP(j, 1);
            const FqSeqDesc &D = descs[j];
            const int N = D.N;
            const int nit = D.iq + (bid < D.ir ? 1 : 0);
            const int quads = nit * M * 4;
            for (int q = lane; q < quads; q += 64) {
                const int it = q / (M * 4), rem = q - it * (M * 4);
                const int row = rem >> 2, c4 = (rem & 3) * 4;
                const float *rp = red + (it * SQ_NW) * EM + row * 16 + c4;
                float v0 = 0.f, v1 = 0.f, v2 = 0.f, v3 = 0.f;
#pragma unroll
                for (int w = 0; w < SQ_NW; w++) {  // fixed order, as fq_gemm_decode_kernel
                    const float4 p = *reinterpret_cast<const float4 *>(rp + w * EM);
                    v0 += p.x;
                    v1 += p.y;
                    v2 += p.z;
                    v3 += p.w;
                }
                const int n0 = 16 * (bid + it * grid) + c4;
                if (n0 < N) {  // N % 4 == 0: the quad is whole
                    const unsigned long long o = (unsigned long long)f2h(v0) | ((unsigned long long)f2h(v1) << 16) |
                                                 ((unsigned long long)f2h(v2) << 32) | ((unsigned long long)f2h(v3) << 48);
                    __hip_atomic_store((gu64 *)(D.d + (long)row * N + n0), o,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sc1 (write-through)
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the stores are out before the flag
            SQ_STAMP(j, 7);
            if (lane == 0) __hip_atomic_store(&flag[bid], (uint32_t)j + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            SQ_STAMP(j, 2);
        }
        if (bid == 0) {  // every WG done with the chain (so none polls any more): leave zeros
            wait_flags((uint32_t)L);
            for (int w = lane; w < grid; w += 64) __hip_atomic_store(&flag[w], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }

    // ================= streaming waves
    char *ring = smem + wid * wl;
    char *ws_st = ring + P * FQ_BLOCK;
    char *xs_st = ws_st + wsst;
    char *x_st = xs_st + xsst;
    const int qsub = lane & 15;
    const int arow = (lane & 15) < M ? (lane & 15) : M - 1;  // A rows >= M mirror row M-1

    // state of the linear whose blocks are being issued
    int G = 0, ga = 0, ng = 0, nit = 0, n = 0;
    int rit = 0, rj = 0, nxt = 0, sl_issue = 0;
    const char *wsrc = nullptr;
    const uint16_t *wsb = nullptr;

    auto issue = [&]() {  // next block (item rit, group ga + rj) -> slot sl_issue
        const int t = bid + rit * grid;
        const char *src = wsrc + ((long)t * G + ga + rj) * FQ_BLOCK;
        char *dst = ring + sl_issue * FQ_BLOCK;
        __builtin_amdgcn_global_load_lds(src, LDS_PTR(dst), 16, 0, 2 /*nt*/);
        if (lane < 32) __builtin_amdgcn_global_load_lds(src + 1024, LDS_PTR(dst + 1024), 16, 0, 2);
        if (++rj == ng) {
            rj = 0;
            ++rit;
        }
        ++nxt;
        if (++sl_issue == P) sl_issue = 0;
    };
    // prologue of linear j: ring block 0, the w-scale staging, ring blocks 1 .. min(P, n) - 1
    auto prologue = [&](int j) {
        const FqSeqDesc &D = descs[j];
        G = D.G;
        ga = (wid * G) >> 3;  // SQ_NW = 8
        ng = (((wid + 1) * G) >> 3) - ga;
        nit = D.iq + (bid < D.ir ? 1 : 0);
        n = ng * nit;
        wsrc = D.w + lane * 16;
        wsb = reinterpret_cast<const uint16_t *>(D.w + (size_t)D.NT * G * FQ_BLOCK);
        rit = rj = nxt = sl_issue = 0;
        if (n == 0) return;
        issue();
        for (int i0 = 0; i0 < n; i0 += 32) {  // w-scales: 32 blocks (32 B = 2 lanes each) per instruction
            const int i = i0 + (lane >> 1) < n ? i0 + (lane >> 1) : n - 1;
            const int it = i / ng;
            __builtin_amdgcn_global_load_lds(wsb + ((long)(bid + it * grid) * G + ga + (i - it * ng)) * 16 + 8 * (lane & 1),
                                             LDS_PTR(ws_st + i0 * 32), 16, 0, 0);
        }
        const int first = n < P ? n : P;
        while (nxt < first) issue();
    };

    prologue(0);
    for (int j = 0; j < L; j++) {
        const FqSeqDesc &D = descs[j];
        __builtin_amdgcn_s_barrier();  // B2: linear j's dependency is complete
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (compiler only: the x loads stay below)

        // ---- x_j: sc1 loads (16 B per lane as two 8-B loads), quantized into x_st / xs_st
        const int R = ng * M, abits = D.abits;
        for (int r0 = 0; r0 < R; r0 += 32) {
            uint4 raw[8];
#pragma unroll
            for (int c = 0; c < 8; c++) {
                int rg = r0 + 4 * c + (lane >> 4);
                rg = rg < R ? rg : R - 1;
                const int jj = M == 1 ? rg : rg / M, row = rg - jj * M;
                gu64 *src = (gu64 *)(D.x + (long)row * D.ldx + (long)(ga + jj) * FQ_GROUP + qsub * 8);
                if (r0 + 4 * c < R) {
                    const unsigned long long lo = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const unsigned long long hi = __hip_atomic_load(src + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    raw[c] = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
                }
            }
#pragma unroll
            for (int c = 0; c < 8; c++) {
                if (r0 + 4 * c < R) {  // wave-uniform
                    const int rg = r0 + 4 * c + (lane >> 4);
                    uint2 codes;
                    const uint16_t sh = quant_group16(raw[c], abits, codes);
                    if (rg < R) {
                        const int jj = M == 1 ? rg : rg / M, row = rg - jj * M;
                        ds_write_b64(lds_addr(x_st + rg * 128 + xswz(row, qsub >> 1) + (qsub & 1) * 8), codes);
                        if (qsub == 0) ds_write_b32(lds_addr(xs_st + (jj * SQ_XSR + row) * 4), sh);
                    }
                }
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // codes and scales are in LDS (wave-local)
        if (wid == 0) SQ_STAMP(j, 3);

        // ---- the stream: nit items x ng groups; ring slots refilled to distance SQ_DIST
        int i = 0, sl = 0;
        for (int it = 0; it < nit; it++) {
            float cur[4] = {0.f, 0.f, 0.f, 0.f};
            for (int jj = 0; jj < ng; jj++, i++) {
                wait_ring<2, SQ_PMAX>(nxt - 1 - i);  // block i (and everything older) landed
#ifdef FQ_DEV_ABLATION
                if (i == 0 && wid == 0) SQ_STAMP(j, 4);
#endif
                const uint32_t sp = lds_addr(ring + sl * FQ_BLOCK);
                const v2u p0 = ds_read_b64(sp + lane * 8);
                const v2u p1 = ds_read_b64(sp + 512 + lane * 8);
                const v2u p2 = ds_read_b64(sp + 1024 + lane * 8);
                const uint32_t xrow = lds_addr(x_st + (jj * M + arow) * FQ_GROUP);
                v4i a0 = ds_read_b128(xrow + xswz(arow, lane >> 4));
                v4i a1 = ds_read_b128(xrow + xswz(arow, 4 + (lane >> 4)));
                const uint32_t wsv = ds_read_u16(lds_addr(ws_st) + i * 32 + 2 * (lane & 15));
                const v4i xd = ds_read_b128(lds_addr(xs_st + jj * SQ_XSR * 4) + 16 * (lane >> 4));
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot is in registers
                __builtin_amdgcn_sched_barrier(0);
                if (nxt < n && nxt <= i + SQ_DIST) issue();
                if (++sl == P) sl = 0;

                const v4i b0 = unpack_fq6(p0[0], p1[0], p2[0]), b1 = unpack_fq6(p0[1], p1[1], p2[1]);
                const __half2 w2 = __half2half2(__ushort_as_half((uint16_t)wsv));
                v4i acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, b0, v4i{0, 0, 0, 0}, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, b1, acc, 0, 0, 0);
                const uint32_t x01 = __builtin_amdgcn_perm((uint32_t)xd[1], (uint32_t)xd[0], 0x05040100u);
                const uint32_t x23 = __builtin_amdgcn_perm((uint32_t)xd[3], (uint32_t)xd[2], 0x05040100u);
                const __half2 s01 = __hmul2(*reinterpret_cast<const __half2 *>(&x01), w2);  // fp16-rounded
                const __half2 s23 = __hmul2(*reinterpret_cast<const __half2 *>(&x23), w2);  // scale product
                cur[0] = fmaf((float)acc[0], __low2float(s01), cur[0]);
                cur[1] = fmaf((float)acc[1], __high2float(s01), cur[1]);
                cur[2] = fmaf((float)acc[2], __low2float(s23), cur[2]);
                cur[3] = fmaf((float)acc[3], __high2float(s23), cur[3]);
            }
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int row = 4 * (lane >> 4) + r;
                if (row < M) red[(it * SQ_NW + wid) * EM + row * 16 + (lane & 15)] = cur[r] * 0.25f;
            }
        }
        if (wid == 0) SQ_STAMP(j, 5);
        if (wid == SQ_NW - 1) SQ_STAMP(j, 6);
        if (j + 1 < L) prologue(j + 1);  // weights of the next linear stream during the hand-off
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // B1: partial tiles of linear j are in red
    }
}

// =============================================================================================
// Host side
// =============================================================================================
static int seq_device_cus() {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
    }
    return cus;
}

#ifdef FQ_DEV_ABLATION
#include <cstdlib>
static int seq_dev_knob() {
    const char *e = getenv("FQ_SEQ_KNOB");
    return e ? atoi(e) : 0;
}
extern "C" int fq_dev_seq_stamps(unsigned long long *host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_sq_stamps), sizeof(unsigned long long) * n) == hipSuccess ? 0 : 1;
}
#endif

static const int kSeqMaxGrid = 1024;  // flag words (one per WG)
static size_t seq_counter_bytes(int) { return (size_t)kSeqMaxGrid * 4; }
static size_t seq_desc_offset(int count) { return seq_counter_bytes(count) + 16; }

extern "C" size_t fq_linear_seq_workspace_bytes(int count) {
    if (count <= 0) return 0;
    return seq_desc_offset(count) + (size_t)count * sizeof(FqSeqDesc);
}

extern "C" size_t fq_linear_seq_error_offset(int count) { return count > 0 ? seq_counter_bytes(count) : 0; }

static bool ranges_overlap(const void *a, size_t na, const void *b, size_t nb) {
    const uintptr_t a0 = (uintptr_t)a, b0 = (uintptr_t)b;
    return a0 < b0 + nb && b0 < a0 + na;
}

extern "C" fq_status fq_linear_seq_prepare(const fq_linear_desc *lin, int count, int M, void *workspace,
                                           size_t workspace_bytes, fq_linear_seq *plan, void *host_scratch,
                                           fq_stream_t stream) {
    if (!lin || !plan || !workspace || !host_scratch) return FQ_ERR_NULL;
    *plan = fq_linear_seq{};
    if (count <= 0 || M <= 0 || M > SQ_MT) return FQ_ERR_SHAPE;
    if (workspace_bytes < fq_linear_seq_workspace_bytes(count) || ((uintptr_t)workspace & 15)) return FQ_ERR_WORKSPACE;
    const int grid = seq_device_cus();
    if (grid > kSeqMaxGrid) return FQ_ERR_SHAPE;
    FqSeqDesc *h = reinterpret_cast<FqSeqDesc *>(host_scratch);
    int wsst = 0, xsst = 0, xst = 0, redb = 0;
    for (int j = 0; j < count; j++) {
        const fq_linear_desc &l = lin[j];
        if (!l.x || !l.w_packed || !l.d) return FQ_ERR_NULL;
        if (l.N <= 0 || l.K <= 0 || l.K % FQ_GROUP || l.N % 4 || l.ldx < l.K || l.ldx % 8) return FQ_ERR_SHAPE;
        if (((uintptr_t)l.x & 15) || ((uintptr_t)l.d & 7) || ((uintptr_t)l.w_packed & 15)) return FQ_ERR_SHAPE;
        if (l.abits != 6 && l.abits != 8) return FQ_ERR_BITS;
        FqSeqDesc &d = h[j];
        d = FqSeqDesc{};
        d.x = l.x;
        d.w = (const char *)l.w_packed;
        d.d = l.d;
        d.N = l.N;
        d.K = l.K;
        d.ldx = l.ldx;
        d.abits = l.abits;
        d.NT = (l.N + 15) / 16;
        d.G = l.K / FQ_GROUP;
        d.iq = d.NT / grid;
        d.ir = d.NT % grid;
        // the latest earlier linear this one conflicts with (RAW, WAR, WAW on byte ranges)
        const size_t xb = ((size_t)(M - 1) * l.ldx + l.K) * 2, db = (size_t)M * l.N * 2;
        d.dep = -1;
        for (int i = j - 1; i >= 0 && d.dep < 0; i--) {
            const size_t xbi = ((size_t)(M - 1) * lin[i].ldx + lin[i].K) * 2, dbi = (size_t)M * lin[i].N * 2;
            if (ranges_overlap(l.x, xb, lin[i].d, dbi) || ranges_overlap(l.d, db, lin[i].x, xbi) ||
                ranges_overlap(l.d, db, lin[i].d, dbi))
                d.dep = i;
        }
        const int ngmax = (d.G + SQ_NW - 1) / SQ_NW, ipw = (d.NT + grid - 1) / grid;
        wsst = std::max(wsst, decode_wsst_bytes(ngmax * ipw));
        xsst = std::max(xsst, decode_xsst_bytes(ngmax, SQ_MT));
        xst = std::max(xst, decode_xst_bytes(ngmax, M));
        redb = std::max(redb, ipw * SQ_NW * M * 16 * 4);
    }
    // ring slots: as many as fit (3 .. 8); one WG per CU in any case (>= 81 KB of LDS)
    int P = SQ_PMAX;
#ifdef FQ_DEV_ABLATION
    const int knob = seq_dev_knob();
    if (knob & 1)
        for (int j = 0; j < count; j++) h[j].dep = -1;  // no waits (pure streaming)
    if (knob & 2) P = SQ_DIST;                          // no deep prefetch
#endif
    while (P >= SQ_DIST && (size_t)SQ_NW * (P * FQ_BLOCK + wsst + xsst + xst) + redb > 160 * 1024) P--;
    if (P < SQ_DIST) return FQ_ERR_SHAPE;
    const int wl = P * FQ_BLOCK + wsst + xsst + xst;
    const int redoff = SQ_NW * wl;
    size_t lds = (size_t)redoff + redb;
    if (lds < 81 * 1024) lds = 81 * 1024;
    hipStream_t s = (hipStream_t)stream;
    char *ws = (char *)workspace;
    if (hipMemsetAsync(ws, 0, seq_desc_offset(count), s) != hipSuccess) return FQ_ERR_HIP;
    if (hipMemcpyAsync(ws + seq_desc_offset(count), h, (size_t)count * sizeof(FqSeqDesc), hipMemcpyHostToDevice, s) !=
        hipSuccess)
        return FQ_ERR_HIP;
    plan->count = count;
    plan->M = M;
    plan->grid = grid;
    plan->slots = P;
    plan->wave_lds = wl;
    plan->wsst = wsst;
    plan->xsst = xsst;
    plan->redoff = redoff;
    plan->lds_bytes = (int)lds;
    plan->workspace = workspace;
    return FQ_OK;
}

extern "C" size_t fq_linear_seq_host_scratch_bytes(int count) { return count > 0 ? (size_t)count * sizeof(FqSeqDesc) : 0; }

extern "C" fq_status fq_linear_seq_run(const fq_linear_seq *p, fq_stream_t stream) {
    if (!p || !p->workspace) return FQ_ERR_NULL;
    if (p->count <= 0) return FQ_ERR_SHAPE;
    char *ws = (char *)p->workspace;
    hipLaunchKernelGGL(fq_seq_kernel, dim3(p->grid), dim3(SQ_THREADS), p->lds_bytes, (hipStream_t)stream,
                       reinterpret_cast<const FqSeqDesc *>(ws + seq_desc_offset(p->count)), p->count, p->M,
                       (gu32 *)ws, (gu32 *)(ws + seq_counter_bytes(p->count)),
                       p->slots, p->wave_lds, p->wsst, p->xsst, p->redoff);
    FQ_LAUNCH_CHECK();
    return FQ_OK;
}
