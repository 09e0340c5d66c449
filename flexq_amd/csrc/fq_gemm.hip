// fq_gemm.hip -- W6A6 / W6A8 GEMM with per-group dequantization for gfx950 (CDNA4).
//
// Contraction: the reference emulates INT6 x INT6 with 36 binary MMAs per bit-pair set
// (mma.m8n8k128.b1.and.popc, engine/src/bgemm/bgemm.cuh:431-450).  Here a 6-bit weight is
// unpacked in registers into the top 6 bits of an int8 (value 4w, fq_common.h unpack_fq6) and
// the contraction runs on v_mfma_i32_16x16x64_i8 with int32 accumulation, reset every 128-wide
// group (two k-steps of 64).  acc4 = 4 * sum_k x*w exactly (|acc4| <= 2^21), so float(acc4) is
// exact and the final x0.25 is exact: the result equals sum_g float(half(xs*ws)) * acc_g
// accumulated in fp32, which is the reference's dequant (flexq_bmma_kernel.h:359-373) with the
// bit-pair sum moved inside the integer accumulator.
//
// MFMA operand maps (16x16x64 i8): lane l holds A[row l&15][k = 16*(l>>4) + j] and
// B[k = 16*(l>>4) + j][col l&15], j = 0..15 -- any k relabelling shared by A and B gives the same
// sum; C/D: col = l&15, row = 4*(l>>4) + r, r = 0..3 (cdna_hip_programming.md §3).  The fq6
// weight layout stores exactly these B operands (16-column tiles, fq_quant.hip).
#include "fq_lds.h"
#include <cstdlib>
#include <mutex>
#include <unordered_map>
#include <type_traits>

// =============================================================================================
// Decode / small-M kernel (M <= 32): HBM-bound weight streaming.
//
// Work items are (n-tile t of 16 columns, k-split z).  A workgroup (one per CU, persistent over
// items w, w + grid, ...) streams each item's contiguous fq6 blocks (1.5 KiB = 16 columns x one
// 128-wide group); its NW waves take contiguous group sub-ranges, so a tile's partial sums meet
// in LDS and S = 1 needs no cross-CU reduction.  Measured on MI355X (tools/stamps.py): a CU
// streams ~24 GB/s when the whole chip streams, so the per-CU work must be even -- 16-column
// tiles make the LLaMA widths (4096 k) divide evenly over 256 CUs, and a cross-CU split-K
// fix-up (~1.2 us) is reserved for narrow N (tensor-parallel shards).
//   * Ring: D weight slots per wave filled by LDS-DMA (global_load_lds_dwordx4 nt: one 1 KiB and
//     one 512 B instruction per block), retired by hand-counted `s_waitcnt vmcnt(U * in-flight)`,
//     running ahead across item boundaries.  LDS reads are inline asm (hipcc would guard them
//     with vmcnt(0) against the in-flight DMA); item-end barriers are raw s_barrier (a
//     __syncthreads() would drain the ring).
//   * Staging (XS/SS = 0): a few wide LDS-DMA instructions in the prologue stage the blocks'
//     w-scales / x-scales and the activation rows, so the loop moves weights only.  When the
//     staged bytes would not fit LDS (very long K), they ride in each ring slot instead (XS/SS = 1).
//   * FUSE: the kernel quantizes the fp16 activations itself (see below).
//   * S > 1: each item's fp32 partial tile goes out with write-through (sc1) stores; after the
//     loop the WG drains them once, takes one agent-scope ticket per item, and the last WG of a
//     tile sums the S slabs in z order (sc1 loads, 8 in flight).  Deterministic: fixed order,
//     no float atomics.  (MI355X_MICROARCH.md "Valid forms", row 1.)
// =============================================================================================

// decode chain: a producer link waiting for granules loads its ready values behind the ring (0: ahead)
#ifndef FQ_CHAIN_LATE_READY
#define FQ_CHAIN_LATE_READY 1
#endif
// decode chain: s_sleep between two polls of the hand-off granules
#ifndef FQ_CHAIN_SLEEP
#define FQ_CHAIN_SLEEP 1
#endif
// cache policy of the weight stream's LDS-DMA (aux: 2 = nt, once-read bytes)
#ifndef FQ_W_AUX
#define FQ_W_AUX 2
#endif
// waves per WG (one WG per CU): 8, or 4 for 32-row tiles (their reduction buffers are larger)
#ifndef FQ_DECODE_WAVES
#define FQ_DECODE_WAVES 8
#endif
__host__ __device__ constexpr int decode_waves(int MT) { return MT <= 16 ? FQ_DECODE_WAVES : FQ_DECODE_WAVES / 2; }
// ring depth: up to 8 slots within a per-wave ring budget of 16 KiB (8 waves) / 32 KiB (4 waves),
// halved when M > 4 rows of activations are staged (they take the LDS instead)
#ifndef FQ_RING_BUDGET
#define FQ_RING_BUDGET 4608
#endif
#ifndef FQ_RING_DMAX
#define FQ_RING_DMAX 3
#endif
// (64-row tiles, activations per slot: three slots of a block + 64 activation rows + their scales,
// so the weight stream keeps three blocks per wave in flight as the small-M kernels do)
__host__ __device__ constexpr int decode_ring_budget(int MT, int XS) {
    return MT >= 64 && XS ? 3 * (FQ_BLOCK + 8 * 1024 + 64 + 64 * 4)
                          : (decode_waves(MT) == 8 ? FQ_RING_BUDGET : 2 * FQ_RING_BUDGET) / (XS == 0 && MT > 4 ? 2 : 1);
}
__host__ __device__ constexpr int decode_depth_cap(int U) { return 63 / U + 1 < FQ_RING_DMAX ? 63 / U + 1 : FQ_RING_DMAX; }
__host__ __device__ constexpr int decode_depth_for(int MT, int XS, int slot, int U) {
    // (D - 1) * U must fit the 6-bit vmcnt immediate; at least 2 slots
    return decode_ring_budget(MT, XS) / slot < 2 ? 2
           : decode_ring_budget(MT, XS) / slot < decode_depth_cap(U) ? decode_ring_budget(MT, XS) / slot
                                                                     : decode_depth_cap(U);
}

// XS: activation rows staged for the wave's groups (0) or carried per ring slot (1).
// SS: w-/x-scales staged (0) or carried per ring slot (1).
// XSR: x-scale record per group in LDS (dwords; rows >= M are read but never used).
template <int MT, int XS, int SS> struct DecodeCfg {
    static constexpr int RG = MT <= 16 ? 1 : MT / 16;            // 16-row MFMA row groups
    static constexpr int XSR = 16 * RG;
    static constexpr int XP = XS ? (MT <= 8 ? 1 : MT / 8) : 0;  // 1 KiB activation pieces per slot
    static constexpr int WS_OFF = FQ_BLOCK + XP * 1024;         // slot scales (SS = 1)
    static constexpr int XS_OFF = WS_OFF + 64;
    static constexpr int SLOT = SS ? XS_OFF + XSR * 4 : WS_OFF;
    static constexpr int U = 2 + XP + (SS ? 2 : 0);              // ring DMA instructions per block
    static constexpr int D = decode_depth_for(MT, XS, SLOT, U);   // ring depth
};

__host__ __device__ inline int decode_slot(int MT, int XS, int SS) {
    const int XP = XS ? (MT <= 8 ? 1 : MT / 8) : 0;
    return SS ? FQ_BLOCK + XP * 1024 + 64 + decode_xsr(MT) * 4 : FQ_BLOCK + XP * 1024;
}

// fused quantizer: fp16 window of xwin (group, row) pairs (a multiple of 4, at most 32 = 8 KiB)
__host__ __device__ inline int decode_xwin_bytes(int ng, int M, int xwin) { return (ng * M < xwin ? (ng * M + 3) / 4 * 4 : xwin) * 256; }
// per-wave LDS: [ring D x SLOT][ws: nb x 8 dwords][xs: ng x XSR dwords][x: ng x M x 128 B]
//               [FUSE: fp16 window]
// (wm windows side by side: 3 for the RMSNorm prologue -- residual, input, gamma --, 2 for SiLU * up)
// fp16 windows a fused producer's prologue fetches: RMSNorm 3 (residual, input, gamma), SiLU 2 (gate,
// up), LayerNorm 5 (residual, input, gamma, beta, bias)
__host__ __device__ constexpr int decode_pro_windows(int pro) { return pro == 1 ? 3 : pro == 2 ? 2 : pro == 4 ? 5 : 1; }
__host__ __device__ inline int decode_wave_lds(int MT, int XS, int SS, int ng, int nb, int M, int xwin, int wm = 1) {
    const int XP = XS ? (MT <= 8 ? 1 : MT / 8) : 0;
    int b = decode_depth_for(MT, XS, decode_slot(MT, XS, SS), 2 + XP + (SS ? 2 : 0)) * decode_slot(MT, XS, SS);
    if (!SS) b += decode_wsst_bytes(nb) + decode_xsst_bytes(ng, MT);
    if (!XS) b += decode_xst_bytes(ng, M);
    if (xwin) b += wm * decode_xwin_bytes(ng, M, xwin);
    return b;
}

#define FQ_CSTAMP_LINKS 8
#ifdef FQ_DEV_ABLATION
// development timeline: per WG (wave 0) s_memrealtime stamps (100 MHz), tools/stamps.py
__device__ unsigned long long g_fq_stamps[1024 * 8];
#define FQ_STAMP(k)                                                                  \
    if ((ABL & 16) && threadIdx.x == 0 && blockIdx.x < 1024) {                       \
        g_fq_stamps[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime();        \
    }
// decode chain timeline: per (WG, linear) wave-0 stamps 0 linear start, 1 ring issued, 2 input
// quantized, 3 first block landed, 4 stream done, 5 linear end (tools/chain_stamps.py)
__device__ unsigned long long g_fq_cstamps[1024 * FQ_CSTAMP_LINKS * 8];
#define FQ_CSTAMP(k)                                                                                   \
    if (CHN && threadIdx.x == 0 && blockIdx.x < 1024 && pro.link < FQ_CSTAMP_LINKS) {                  \
        g_fq_cstamps[((long)blockIdx.x * FQ_CSTAMP_LINKS + pro.link) * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); \
    }
#else
#define FQ_STAMP(k)
#define FQ_CSTAMP(k)
#endif

// ---- peer-store gather (column-parallel decode, fq_linear_w6ax_gather): each rank stores its output
// tiles straight into every rank's [M][ld] gather buffer (IPC-mapped device pointers; on an 8-GPU
// node these are stores over xGMI) at column offset col0, so the all-gather is the GEMM epilogue.
// Stores are system-scope write-through (sc0 sc1), 4 bytes = two adjacent columns each.  After the
// last workgroup's ticket (every workgroup's stores drained first), it raises this rank's flag in
// every rank's flag array to gen + 1; fq_gather_wait_kernel on each rank waits for all P flags.
__device__ __forceinline__ void gather_store2(const fq_gather *__restrict__ gat, int P, int row, int col,
                                              float v0, float v1) {
    const uint32_t pk = (uint32_t)f2h(v0) | ((uint32_t)f2h(v1) << 16);
    const long off = (long)row * gat->ld + gat->col0 + col;
    for (int q = 0; q < P; q++)
        __hip_atomic_store(reinterpret_cast<uint32_t *>(gat->out[q] + off), pk, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void gather_publish(const fq_gather *__restrict__ gat) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave drains its peer stores
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t prev = __hip_atomic_fetch_add(gat->done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == gridDim.x - 1) {  // the last workgroup: every store of this launch has drained
            __hip_atomic_store(gat->done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t val = __hip_atomic_load(gat->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the fence's own wait can be dropped)
            for (int q = 0; q < gat->P; q++)
                __hip_atomic_store(gat->flags[q] + gat->rank, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            // this call's generation: the consumer (fq_gather_wait, or the next linear's prologue,
            // gather_poll) waits for every rank's flag to reach it
            __hip_atomic_store(gat->gen, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// The wait of a peer-store gather folded into the next linear's prologue (fq_linear_w6ax_gather_after):
// wave 0 polls this rank's P flag words -- lane q rank q's word, system-scope loads of the uncached
// flag array, s_sleep between polls -- until every one has reached the gather's generation (raised
// by its last publish), while the linear's weight-ring DMAs, issued before, are in flight; the other
// waves wait at a raw s_barrier (it does not drain their DMAs).  No acquire fence: the gather
// buffers are uncached device memory (flexq_amd/dist.py PeerGather), stored system-scope and
// drained by every peer before its flag, so a load issued after the poll matched reads the data
// (an acquire's vmcnt(0) would also wait for the ring).  Bounded like fq_gather_wait: ~1 s, then the
// error word is set and the launch goes on (results undefined, never a hang); once it is set, later
// polls return at once.  Every wave of the workgroup must call it.
__device__ __forceinline__ void gather_poll(const fq_gather *__restrict__ g, uint32_t *__restrict__ err, int wid) {
    if (wid == 0) {
        const int lane = threadIdx.x & 63;
        if (!(err && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u)) {
            const uint32_t target = __hip_atomic_load(g->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t *mine = g->flags[g->rank];
            bool ok = lane >= g->P;
            for (int spin = 0; spin < (1 << 20); spin++) {
                if (!ok) ok = __hip_atomic_load(mine + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= target;
                if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;
                __builtin_amdgcn_s_sleep(8);
            }
            if (__builtin_amdgcn_ballot_w64(!ok) != 0 && lane == 0 && err)
                __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    __builtin_amdgcn_s_barrier();
}

// ---- decode chain (fq_linear_chain_w6ax): consecutive dependent linears in ONE persistent launch,
// one workgroup per CU.  Linear l + 1 issues its weight ring and w-scale staging (which depend on
// nothing) first and only then waits for its activations, so the wait hides under the first blocks
// of its stream instead of sitting behind a kernel boundary (~1.75 us) and the next
// launch's ramp.
// Hand-off: data-tagged 8-byte granules {two fp16 outputs, tag} (MI355X_MICROARCH.md price list,
// granule rows; R2: a granule is one naturally aligned 8-byte sc1 store and needs no ordering).  A
// linear whose output feeds the next one writes each pair of outputs twice: to the caller's d, and
// as a granule into its hand-off buffer in the workspace.  The consumer's waves load their own
// activation slices from that buffer with sc1 buffer loads and re-load until every granule carries
// the expected tag -- no flag, no counter, no drain, no second round trip for the data.
// The hand-off buffers live in the chain workspace (fq_chain_workspace_init), which nothing but
// chain launches writes: zero at first, then granules of earlier launches.  Tag = E + 1, E = the
// epoch word every workgroup reads as the launch starts (a run's hand-off buffers are disjoint), so
// no granule an earlier launch left matches.  Every workgroup adds 1 to its shard of a start counter
// after reading E; workgroup 0, in linear 1's prologue, waits until all have (they have long since),
// then stores E + 1 and zeroes the shards for the next launch.  The launch whose tag is 2^31 - 1 ends
// with a fan-in whose last workgroup zeroes the hand-off region and the epoch (tags never repeat
// over a granule's lifetime, and never have bit 31 set).  Bounded: a wait that does not end within
// ~1 s sets the error word and goes on; with the error word set later waits return at once.  A linear
// whose wait failed writes fp16 NaN outputs (its granules carry them); every workgroup that waited on
// the missing input timed out with it and set the sticky word, which the next linear reads as it
// starts, so it fails at once and writes NaN in turn: every output downstream of a failure is NaN
// (results are never undefined-but-plausible) at no cost to the normal path.
constexpr int FQ_CHAIN_MAX = 8;
constexpr size_t FQ_CHAIN_SYNC_BYTES = 4096;       // chain workspace: sync words, then the hand-offs
constexpr int FQ_CHAIN_EPOCH = 8, FQ_CHAIN_ERR = 9, FQ_CHAIN_DONE = 10;  // sync words, 128 B apart;
                                                                           // 0..7: the start counter
constexpr int FQ_CHAIN_HOST = 11;  // 8 bytes: device address of the bound host status word (or 0)
__device__ __forceinline__ uint32_t chain_tag(uint32_t epoch) { return epoch + 1u; }
// A wait timed out: the sticky device error word (later waits on this workspace return at once) and,
// when the caller bound one (fq_chain_bind_status), the host status word -- a system-scope vector store
// into pinned host memory, read by the host entry point before its next launch (FQ_ERR_TIMEOUT).
__device__ __forceinline__ void chain_fail(uint32_t *__restrict__ sync) {
    __hip_atomic_store(sync + 32 * FQ_CHAIN_ERR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t h = __hip_atomic_load(reinterpret_cast<uint64_t *>(sync + 32 * FQ_CHAIN_HOST), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    if (h) __hip_atomic_store(reinterpret_cast<uint32_t *>(h), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    // (the failure path retires its own loads: otherwise a load left pending on this rare path makes the
    // compiler wait vmcnt(0) -- the next linear's whole ring -- at the chain's link loop head)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
// The epoch is loaded as the launch starts and first needed a linear later: every use goes through
// this (volatile: not hoisted to the load), so no wave waits for it before its first DMA.
__device__ __forceinline__ uint32_t chain_late(uint32_t v) {
    asm volatile("" : "+v"(v));
    return v;
}

// the caller's output pair (plain 4-byte store) and, for a linear the next one reads, its granule
__device__ __forceinline__ void chain_store2(uint16_t *__restrict__ d, uint64_t *__restrict__ hd, uint32_t tag, int N,
                                             int row, int col, float v0, float v1) {
    const uint32_t pk = (uint32_t)f2h(v0) | ((uint32_t)f2h(v1) << 16);
    const long f = (long)row * N + col;
    *reinterpret_cast<uint32_t *>(d + f) = pk;
    if (hd) __hip_atomic_store(hd + (f >> 1), ((uint64_t)tag << 32) | pk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Workgroup 0 advances the epoch once every workgroup has read it (each adds to the start counter
// after its first linear, whose tag needed the epoch): wave 0 loads the counter's shards as linear 1
// starts (chain_epoch_load, not waited for), and after linear 1's stores (chain_epoch_update) it
// stores epoch + 1 and zeroes the shards if all had arrived -- they have, a linear earlier -- else it
// polls for them there (bounded).
__device__ __forceinline__ uint32_t chain_epoch_load(uint32_t *__restrict__ sync) {
    const int lane = threadIdx.x & 63;
    return lane < 8 ? __hip_atomic_load(sync + 32 * lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
}
__device__ __forceinline__ void chain_epoch_update(uint32_t *__restrict__ sync, uint32_t epoch, uint32_t seen, int grid) {
    const int lane = threadIdx.x & 63;
    const uint32_t target = lane < 8 ? (uint32_t)((grid - lane + 7) >> 3) : 0u;
    bool ok = seen >= target;
    for (int spin = 0; spin < (1 << 20) && __builtin_amdgcn_ballot_w64(!ok) != 0; spin++) {
        __builtin_amdgcn_s_sleep(2);
        if (!ok) ok = __hip_atomic_load(sync + 32 * lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target;
    }
    if (__builtin_amdgcn_ballot_w64(!ok) != 0) {
        if (lane == 0) chain_fail(sync);
    } else if (lane < 8) {
        __hip_atomic_store(sync + 32 * lane, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (lane == 0) __hip_atomic_store(sync + 32 * FQ_CHAIN_EPOCH, epoch + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ---- deferred split-K fix-up of the decode kernels.  Every item's partial tile went out as
// write-through (sc1) slab stores; one drain, then one agent-scope ticket per item (taken in
// parallel, one lane each), and the last arriver of a tile sums its S slabs in z order.
// Memory ordering (MI355X_MICROARCH.md, "Valid forms", first row of the sc1 hand-off table,
// which replaces the agent release/acquire pair -- ~1.7 us each per launch -- under four
// conditions, all held here): (1) every load of the slabs is a global sc1 load (relaxed
// agent-scope atomic loads below); (2) every slab byte was stored sc1 (relaxed agent-scope
// atomic stores, 4 B each); (3) every storing wave drains its stores (vmcnt(0)) before the
// workgroup barrier behind which one lane per item adds to the item's ticket; (4) the ticket is
// an agent-scope atomic add, the workgroup whose add returned S - 1 is the consumer, its loading
// waves wait on a workgroup barrier after the add (the LDS flag), the buffer is hipMalloc'd and
// there is one workgroup per CU.
// Hand-off rule for this file: nothing here POLLS.  A consumer learns that it is last from the
// value its own atomic add returned, so no wave ever waits on another workgroup.  Any future poll
// must be a global_/buffer_ sc1 load to registers (never an LDS-DMA into LDS: such a line can sit
// in the poller's XCD L2 and never see another XCD's atomic -- DESIGN.md §8, the round-2 tail-split
// hang), followed by ONE agent acquire, with a bounded spin that ends in a printf of the ticket
// value and __builtin_trap() (MI355X_MICROARCH.md "Valid forms", Consumer bullet).
template <int NW, bool GAT>
__device__ __forceinline__ void decode_splitk_fixup(int nit, int S, int M, int N, int Npad, int EM, int t0,
                                                    int tstep, float *__restrict__ slabs,
                                                    uint32_t *__restrict__ tickets, uint16_t *__restrict__ d,
                                                    int *flag, const fq_gather *__restrict__ gat) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
    __syncthreads();
    if ((int)threadIdx.x < nit) {
        const int tt = t0 + (int)threadIdx.x * tstep;
        const uint32_t prev = __hip_atomic_fetch_add(&tickets[tt], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = (prev == (uint32_t)(S - 1));
        if (last) __hip_atomic_store(&tickets[tt], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        flag[threadIdx.x] = last;
    }
    __syncthreads();  // (the flag is read behind this barrier: the slab loads cannot move above it)
    const int GP = GAT ? gat->P : 0;  // (gather: two adjacent columns per thread, 4-byte stores)
    for (int it = 0; it < nit; it++) {
        if (!flag[it]) continue;  // workgroup-uniform
        const int t = t0 + it * tstep;
        if (GAT) {
            for (int e = 2 * threadIdx.x; e < EM; e += 2 * NW * 64) {
                const int row = e >> 4, nn = 16 * t + (e & 15);
                float v0 = 0.f, v1 = 0.f;
                for (int z0 = 0; z0 < S; z0++) {
                    v0 += __hip_atomic_load(&slabs[((long)z0 * M + row) * Npad + nn], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    v1 += __hip_atomic_load(&slabs[((long)z0 * M + row) * Npad + nn + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                gather_store2(gat, GP, row, nn, v0, v1);
            }
            continue;
        }
        for (int e = threadIdx.x; e < EM; e += NW * 64) {
            const int row = e >> 4, nn = 16 * t + (e & 15);
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
}

// ---- the next linear's codes in the decode GEMM's epilogue (fq_gemm_w6ax_q at M <= 16, S = 1; VERDICT
// r05 item 2).  A 16-column tile never holds a whole 128-column group, so the group's absmax has to cross
// workgroups: every workgroup's output pairs go out as agent-scope (sc1) stores; it drains them, takes one
// agent-scope ticket per 128-column group of its tiles (8 tiles, fewer at the right edge), and the last
// arriver of a group re-loads the group's M x 128 outputs (sc1 loads) and quantizes them exactly as
// fq_quantize_act does (quant_group16), reading d's leading qM * qK values as the flat [qM][qK] next input
// (N % 128 == 0: a 128-column group of d is a group of the next input).  The hand-off rule of
// decode_splitk_fixup below: nothing polls; the last arriver learns it from its own add, and it resets
// the ticket for the next launch.
struct DecodeQ {
    int8_t *qxq;    // int8 [qM][qK]
    uint16_t *qxs;  // fp16 [qK / 128][qM]
    int qM, qK, qbits;
};
template <int NW>
__device__ __forceinline__ void decode_qe_epilogue(int nit, int M, int N, int t0, int tstep, uint32_t *__restrict__ tickets,
                                                   const uint16_t *__restrict__ d, int *flag, const DecodeQ &qe) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 output stores
    __syncthreads();
    const long lim = (long)qe.qM * qe.qK;
    const int NT = N >> 4;
    for (int it = threadIdx.x; it < nit; it += NW * 64) {
        const int q = (t0 + it * tstep) >> 3;
        int last = 0;
        if ((long)q * FQ_GROUP < lim) {  // (row 0 of the group is part of the next input)
            const int nt = NT - 8 * q < 8 ? NT - 8 * q : 8;
            const uint32_t prev = __hip_atomic_fetch_add(&tickets[q], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last = prev == (uint32_t)(nt - 1);
            if (last) __hip_atomic_store(&tickets[q], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        flag[it] = last;
    }
    __syncthreads();  // (the flags are read behind this barrier: the re-loads cannot move above it)
    const int pr = threadIdx.x >> 4, qsub = threadIdx.x & 15;  // 16 lanes per (row, group), 8 values each
    for (int it = 0; it < nit; it++) {
        if (!flag[it]) continue;  // workgroup-uniform
        const int q = (t0 + it * tstep) >> 3;
        for (int row = pr; row < M; row += NW * 4) {
            const long f0 = (long)row * N + (long)q * FQ_GROUP;  // the group's flat index
            if (f0 >= lim) continue;  // (uniform over the row's 16 lanes, as quant_group16's DPP needs)
            const uint64_t *src = reinterpret_cast<const uint64_t *>(d + f0 + qsub * 8);
            const uint64_t a = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint64_t b = __hip_atomic_load(src + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            uint2 codes;
            const uint16_t sh = quant_group16(make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)),
                                              qe.qbits, codes);
            *reinterpret_cast<uint2 *>(qe.qxq + f0 + qsub * 8) = codes;
            if (qsub == 0) {
                const long r2 = f0 / qe.qK;
                qe.qxs[(f0 - r2 * qe.qK) / FQ_GROUP * qe.qM + r2] = sh;
            }
        }
    }
}

// Producer fused into the FUSE prologue (fq_rmsnorm_linear_w6ax / fq_silu_linear_w6ax):
//   PRO = 1: xh is the residual; r = half_clamp(in + residual) when `in`, RMSNorm with gamma, then
//            the quantizer (M = 1, K = 4 * 128 * NW, S = 1: wave w's four groups are exactly the
//            512-thread producer's chunks 64w .. 64w + 63, so the sum of squares is formed in the
//            same order -- per lane, the 64-lane butterfly, the waves in order -- and the codes are
//            fq_rmsnorm_quantize's bits).  Workgroup 0 writes r to res_out.
//   PRO = 2: xh is the gate, `in` the up projection (row stride ldh): act = half(silu(gate) * up).
// The arithmetic is fq_common.h's, shared with fq_producers.hip.
// (DecodePro: fq_common.h)
// development ablation of the fused producers (timing only, wrong results): 1 = no cross-lane /
// cross-wave reduction, 2 = no input / gamma DMA, 4 = SiLU as a plain product, 8 = no up DMA
#ifndef FQ_PRO_ABL
#define FQ_PRO_ABL 0
#endif

// The decode stream loop's V2 form (buffer-resource weight DMA with scalar block offsets, refill
// right after the slot's plane reads, dequant lagged one block); 0 = the round-3 loop (A/B builds)
#ifndef FQ_DEC_V2
#define FQ_DEC_V2 1
#endif

// Dequantize one block's MFMA accumulators (the reference's epilogue order,
// flexq_bmma_kernel.h:359-373): c[r] += float(acc[r]) * float(half(xs * ws)).
template <int ABL>
__device__ __forceinline__ void dequant4(float (&c)[4], v4i acc, __half2 p01, __half2 p23) {
    if (ABL & 1024) {  // (development: no dequant, accumulators kept alive)
        c[0] = __int_as_float(__float_as_int(c[0]) ^ acc[0] ^ acc[1] ^ acc[2] ^ acc[3]);
        return;
    }
    c[0] = fmaf((float)acc[0], __low2float(p01), c[0]);
    c[1] = fmaf((float)acc[1], __high2float(p01), c[1]);
    c[2] = fmaf((float)acc[2], __low2float(p23), c[2]);
    c[3] = fmaf((float)acc[3], __high2float(p23), c[3]);
}

// The decode chain's next linear, started by this linear's tail: its ring's first D weight blocks and
// its w-scale staging -- exactly the DMAs, slots and order its own prologue would issue (decode_body,
// V2 fused plan, S = 1: t0 = the WG, tstep = the grid) -- right after this linear's last barrier (the
// dynamic LDS is free from there).  The next linear's input wait is a wait for every older DMA of the
// wave (vmcnt retires in order), so issuing its ring here instead of after the descriptor read and
// the prologue's index math moves that wait earlier.  nxt_w / nxt_p: LDS addresses of the next link's
// weight pointer and packed fields (decode_pack).
#ifndef FQ_CHAIN_AHEAD
#define FQ_CHAIN_AHEAD 1
#endif
// The ring prologue's placement and order, shared by decode_body and chain_ring_ahead (which issues a
// chain linear's first ring blocks from the previous linear's tail, and must put exactly those blocks in
// exactly the slots decode_body then reads): the wave's LDS region, its staged w-scales
// after the D ring slots, the first block's byte offset in the image and the jump from an item's last
// group to the next item's first.
struct RingGeom {
    char *ring;      // slot i at ring + i * SLOT
    char *ws_st;     // staged w-scales: 32 B per block of the wave's sequence
    uint32_t roff;   // byte offset of the wave's first block (item tile t0, group ga)
    uint32_t rjump;  // an item's last group -> the next item's first (tiles tstep apart)
};
template <int MT, int XS, int SS>
__device__ __forceinline__ RingGeom ring_geom(char *smem, int wid, int ngmax, int IPW, int M, int xwin, int pro, int t0,
                                              int tstep, int G, int ga, int ng) {
    using C = DecodeCfg<MT, XS, SS>;
    RingGeom r;
    r.ring = smem + wid * decode_wave_lds(MT, XS, SS, ngmax, ngmax * IPW, M, xwin, decode_pro_windows(pro));
    r.ws_st = r.ring + C::D * C::SLOT;
    r.roff = ((uint32_t)t0 * G + ga) * FQ_BLOCK;
    r.rjump = ((uint32_t)tstep * G - ng + 1) * FQ_BLOCK;
    return r;
}
// the w-scales of the wave's block b (item b / ng, group ga + b % ng): 16 fp16 = 32 B, lanes 2b', 2b' + 1
__device__ __forceinline__ const uint16_t *ws_stage_src(const uint16_t *wsb, int tile, int G, int ga, int j, int lane) {
    return wsb + ((long)tile * G + ga + j) * 16 + 8 * (lane & 1);
}
template <int MT>
__device__ __forceinline__ void chain_ring_ahead(uint32_t nxt_w, uint32_t nxt_p) {
    using C = DecodeCfg<MT, 0, 0>;
    constexpr int NW = decode_waves(MT), D = C::D;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    uint2 wp, pa, pb;
    asm volatile("ds_read_b64 %0, %3\n\tds_read_b64 %1, %4\n\tds_read_b64 %2, %4 offset:8\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(wp), "=&v"(pa), "=&v"(pb)
                 : "v"(nxt_w), "v"(nxt_p)
                 : "memory");
    const uint64_t wa = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(wp.x) |
                        ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(wp.y) << 32);
    const uint32_t w0 = __builtin_amdgcn_readfirstlane(pa.x), w1 = __builtin_amdgcn_readfirstlane(pa.y);
    const uint32_t w2 = __builtin_amdgcn_readfirstlane(pb.x), w3 = __builtin_amdgcn_readfirstlane(pb.y);
    const int N = w0 & 0x1fffff, xwin = w0 >> 25, K = (w1 & 0x1fff) * FQ_GROUP;
    const int IPW = w2 & 0xffff, M = w3 & 1023, ir = (w3 >> 10) & 2047, grid = w3 >> 21;
    const int G = K / FQ_GROUP, NT = (N + 15) / 16, lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), bid = blockIdx.x;
    const int nit = IPW - (ir != 0) + (bid < ir ? 1 : 0);
    const int ngmax = (G + NW - 1) / NW, ga = (wid * G) / NW, ng = ((wid + 1) * G) / NW - ga, n = ng * nit;
    if (n <= 0) return;
    // (decode_body's V2 fused plan at S = 1: t0 = the workgroup, tstep = the grid, PRO 0)
    const RingGeom rg = ring_geom<MT, 0, 0>(smem, wid, ngmax, IPW, M, xwin, 0, bid, grid, G, ga, ng);
    char *ring = rg.ring, *ws_st = rg.ws_st;
    const uint32_t *wpk = reinterpret_cast<const uint32_t *>(wa);
    const __amdgpu_buffer_rsrc_t wrs =
        __builtin_amdgcn_make_buffer_rsrc((void *)wpk, (short)0, (int)((uint32_t)NT * G * FQ_BLOCK), 0x00020000);
    const uint16_t *wsb = reinterpret_cast<const uint16_t *>(reinterpret_cast<const char *>(wpk) + (size_t)NT * G * FQ_BLOCK);
    const uint32_t wvo = lane * 16, rjump = rg.rjump;
    uint32_t roff = rg.roff;
    int rj = 0;
#pragma unroll
    for (int i = 0; i < D; i++) {
        char *dst = ring + i * C::SLOT;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, LDS_PTR(dst), 16, wvo, roff, 0, FQ_W_AUX);
        if (lane < 32) __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, LDS_PTR(dst + 1024), 16, wvo, roff + 1024, 0, FQ_W_AUX);
        if (i + 1 < n) {  // (a short sequence re-issues its last block)
            if (++rj == ng) {
                rj = 0;
                roff += rjump;
            } else {
                roff += FQ_BLOCK;
            }
        }
        if (i == 0) {  // the w-scales, 32 blocks (32 B = 2 lanes each) per instruction (decode_body's stage_all)
            for (int i0 = 0; i0 < n; i0 += 32) {
                const int b = i0 + (lane >> 1) < n ? i0 + (lane >> 1) : n - 1;
                __builtin_amdgcn_global_load_lds(ws_stage_src(wsb, bid + (b / ng) * grid, G, ga, b % ng, lane),
                                                 LDS_PTR(ws_st + i0 * 32), 16, 0, 0);
            }
        }
    }
}

// FUSE: the kernel quantizes the fp16 activations itself (fq_linear_w6ax): each wave runs the
// group quantizer (quant_group16, bit-identical to fq_quantize_act) over its own groups straight
// into the staged LDS regions, so a decode linear is one launch.  Requires XS = SS = 0.
template <int MT, int XS, int SS, bool FUSE, bool DBG, int ABL = 0, bool CH = false, int PRO = 0, bool GAT = false,
          bool CHN = false, bool CHP = false, bool QE = false>
__device__ __forceinline__ void decode_body(
    const int8_t *__restrict__ xq, const uint16_t *__restrict__ xs, const uint16_t *__restrict__ xh, int abits,
    const uint32_t *__restrict__ wpk, int Mall, int N, int K, uint16_t *__restrict__ d, int32_t *__restrict__ acc_dbg,
    float *__restrict__ slabs, uint32_t *__restrict__ tickets, int S, int IPW, int RC, int xwin, int iq, int ir,
    int NCH, const fq_gather *__restrict__ gat, const DecodePro &pro, int gridall = -1, DecodeQ qe = DecodeQ{}) {
    if (gridall < 0) gridall = (int)gridDim.x;  // (the plain kernel passes it: no hidden-argument load)
    // Every kernel argument is needed before the first DMA: make the compiler load them all in
    // ONE batch here (it would otherwise issue a second s_load batch after the index math, a
    // second serial round trip before the first DMA; tools/stamps.py).
    // (The fused producers' kernel passes the output, workspace and residual output after its
    // preloaded arguments: they are needed only after the first window, so they stay out of this batch.)
    if (PRO == 0)
        asm volatile("" ::"s"(xq), "s"(xs), "s"(xh), "s"(abits), "s"(wpk), "s"(Mall), "s"(N), "s"(K), "s"(d),
                     "s"(slabs), "s"(tickets), "s"(S), "s"(IPW), "s"(RC), "s"(xwin), "s"(iq), "s"(ir), "s"(gridall));
    else
        asm volatile("" ::"s"(xh), "s"(abits), "s"(wpk), "s"(Mall), "s"(N), "s"(K), "s"(S), "s"(IPW), "s"(RC),
                     "s"(xwin), "s"(iq), "s"(ir), "s"(gridall), "s"(pro.in), "s"(pro.gamma), "s"(pro.ldh));
    if (CH) asm volatile("" ::"s"(NCH));
    using C = DecodeCfg<MT, XS, SS>;
    constexpr int NW = decode_waves(MT), D = C::D, RG = C::RG, XSR = C::XSR;
    static_assert(!FUSE || (XS == 0 && SS == 0), "fused quantization stages into LDS");
    static_assert(PRO == 0 || (FUSE && !CH), "fused producers run in the fused quantizer's prologue");
    static_assert(!CHN || (FUSE && PRO == 0 && !GAT && !CH && !DBG), "the chain runs plain fused linears");
    static_assert(!QE || (!FUSE && PRO == 0 && !GAT && !CH && !DBG && !CHN && MT <= 16),
                  "the epilogue quantizer runs on the plain unfused decode GEMM");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    FQ_STAMP(0);
    FQ_CSTAMP(0);
    const int G = K / FQ_GROUP, NT = (N + 15) / 16;
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // All index math is 32-bit and divides at most once per launch (64-bit or per-item divisions
    // cost microseconds of scalar code before the first DMA).  The grid is a multiple of S, so a
    // WG's k-split z is fixed and its items' tiles are t0, t0 + tstep, ...
    // Row chunks (CH: NCH chunks of MT rows, 32 < M, S = 1): WG b serves rows [MT c, MT c + MT) of
    // every tile it streams, c = b % NCH, as if it were WG b / NCH of a grid of gridDim.x / NCH on
    // those rows; the x-scale stride stays the full M (ldx).  A separate instantiation: the index
    // math below costs the one-chunk kernel ~0.15 us per launch when it is not compiled out.
    const int c = CH ? (int)((unsigned)blockIdx.x % (unsigned)NCH) : 0;
    const int bid = CH ? (int)((unsigned)blockIdx.x / (unsigned)NCH) : (int)blockIdx.x;
    const int grid = CH ? (int)((unsigned)gridall / (unsigned)NCH) : gridall;
    const int M = CH ? (Mall - MT * c < MT ? Mall - MT * c : MT) : Mall, ldx = Mall;
    if (CH) {
        xq += (size_t)MT * c * K;
        xs += MT * c;
        d += (size_t)MT * c * N;
        if (DBG) acc_dbg += (size_t)MT * c * N * (K / FQ_GROUP);
    }
    const int nit = iq + (bid < ir ? 1 : 0);  // items for this WG (>= 1): host-computed quotient
    const int z = S == 1 ? 0 : (unsigned)bid % (unsigned)S;
    const int t0 = S == 1 ? bid : (unsigned)bid / (unsigned)S, tstep = S == 1 ? grid : (unsigned)grid / (unsigned)S;
    const int gz0 = S == 1 ? 0 : (unsigned)(z * G) / (unsigned)S;
    const int gz1 = S == 1 ? G : (unsigned)((z + 1) * G) / (unsigned)S;
    const int Gz = gz1 - gz0;
    const int ngmax = (Gz + NW - 1) / NW;
    const int ga = gz0 + (wid * Gz) / NW, gb = gz0 + ((wid + 1) * Gz) / NW;
    const int ng = gb - ga;  // groups per item for this wave (may be 0)
    const int n = ng * nit;  // blocks in this wave's sequence
    // blocked w-scales of the image: fp16 [NT][G][16] after the weight blocks (fq_quant.hip)
    const uint16_t *wsb = reinterpret_cast<const uint16_t *>(reinterpret_cast<const char *>(wpk) + (size_t)NT * G * FQ_BLOCK);

    const RingGeom rgeo = ring_geom<MT, XS, SS>(smem, wid, ngmax, IPW, M, FUSE ? xwin : 0, PRO, t0, tstep, G, ga, ng);
    const int wl = decode_wave_lds(MT, XS, SS, ngmax, ngmax * IPW, M, FUSE ? xwin : 0, decode_pro_windows(PRO));
    char *ring = rgeo.ring;
    char *ws_st = rgeo.ws_st;                                         // staged w-scales
    char *xs_st = ws_st + (SS ? 0 : decode_wsst_bytes(ngmax * IPW));  // staged x-scales
    char *x_st = xs_st + (SS ? 0 : decode_xsst_bytes(ngmax, MT));     // staged activations
    const int EM = M * 16;                                            // live elements of a tile
    float *red = reinterpret_cast<float *>(smem + NW * wl);           // [RC][NW][M*16]
    int *flag = reinterpret_cast<int *>(red + RC * NW * EM);          // [IPW]
    char *wsum = reinterpret_cast<char *>(flag) + ((4 * IPW + 15) & ~15);  // PRO 1: [NW], PRO 4: [2][NW] floats

    auto item_tile = [&](int it) { return t0 + it * tstep; };

    // Fused quantizer.  The fp16 activations of the wave's (group, row) pairs come in by LDS-DMA
    // (one 1 KiB instruction per 4 pairs) into a window of xwin pairs, issued ahead of the ring
    // so that waiting for them does not wait for the ring; 16 lanes quantize one pair.
    const int qsub = lane & 15;
    const int R = ng * M;  // (group, row) pairs this wave quantizes
    char *xh_st = x_st + (XS ? 0 : decode_xst_bytes(ngmax, M));  // fp16 window (FUSE)
    const int xwb = FUSE ? decode_xwin_bytes(ngmax, M, xwin) : 0;   // (PRO: the next windows)
    const long ldh = PRO ? (long)pro.ldh : (long)K;
    auto x_fetch = [&](int r0) {  // pairs [r0, r0 + xwin) -> xh_st
        if (PRO == 3) {
            // Reference bit planes (int32 [K/128][M/c][b][c][4], c = min(M, 8), k0 at bit 31;
            // engine/src/pack/bit_packing.cu:104-131): a pair's plane p is 16 contiguous bytes.
            // 8 lanes per pair (lane & 7 = plane, planes >= b re-read plane b - 1), 8 pairs per
            // instruction, window slot = 128 B per pair.
            const int ch = M < 8 ? M : 8, q = (lane & 7) < abits ? (lane & 7) : abits - 1;
            const int32_t *planes = reinterpret_cast<const int32_t *>(xh);
            for (int c = 0; c < xwin && r0 + c < R; c += 8) {
                int rg = r0 + c + (lane >> 3);
                rg = rg < R ? rg : R - 1;
                const int j = M == 1 ? rg : rg / M, row = rg - j * M;
                const long wd = (long)(ga + j) * (M * abits * 4) + (row / ch) * (abits * ch * 4) + q * (ch * 4) + (row % ch) * 4;
                __builtin_amdgcn_global_load_lds(planes + wd, LDS_PTR(xh_st + c * 128), 16, 0, 0);
            }
            if (r0 == 0) {  // x-scales: the reference's duplicated pairs (half[K/128][2 ceil4(M)],
                            // SCALE_PACKING_A) are one dword per (group, row) -> xs_st slots
                const int ld2 = (M + 3) / 4 * 4;
                const uint32_t *xsd = reinterpret_cast<const uint32_t *>(pro.in);
                for (int i0 = 0; i0 < ng; i0 += 64 / XSR) {
                    const int i = i0 + lane / XSR, row = lane % XSR;
                    __builtin_amdgcn_global_load_lds(xsd + (long)(ga + (i < ng ? i : ng - 1)) * ld2 + (row < M ? row : M - 1),
                                                     LDS_PTR(xs_st + i0 * XSR * 4), 4, 0, 0);
                }
            }
            return;
        }
        for (int c = 0; c < xwin && r0 + c < R; c += 4) {
            int rg = r0 + c + (lane >> 4);
            rg = rg < R ? rg : R - 1;
            const int j = M == 1 ? rg : rg / M, row = rg - j * M;
            const long off = (long)(ga + j) * FQ_GROUP + qsub * 8;
            __builtin_amdgcn_global_load_lds(xh + row * ldh + off, LDS_PTR(xh_st + c * 256), 16, 0, 0);
            if (PRO == 1 && pro.in && !(FQ_PRO_ABL & 2))
                __builtin_amdgcn_global_load_lds(pro.in + off, LDS_PTR(xh_st + xwb + c * 256), 16, 0, 0);
            if (PRO == 1 && !(FQ_PRO_ABL & 2))
                __builtin_amdgcn_global_load_lds(pro.gamma + off, LDS_PTR(xh_st + 2 * xwb + c * 256), 16, 0, 0);
            if (PRO == 2 && !(FQ_PRO_ABL & 8))
                __builtin_amdgcn_global_load_lds(pro.in + row * ldh + off, LDS_PTR(xh_st + xwb + c * 256), 16, 0, 0);
            if (PRO == 4) {  // (M = 1: the residual row is xh; gamma, beta, bias are per column)
                if (pro.in) __builtin_amdgcn_global_load_lds(pro.in + off, LDS_PTR(xh_st + xwb + c * 256), 16, 0, 0);
                __builtin_amdgcn_global_load_lds(pro.gamma + off, LDS_PTR(xh_st + 2 * xwb + c * 256), 16, 0, 0);
                if (pro.beta) __builtin_amdgcn_global_load_lds(pro.beta + off, LDS_PTR(xh_st + 3 * xwb + c * 256), 16, 0, 0);
                if (pro.bias) __builtin_amdgcn_global_load_lds(pro.bias + off, LDS_PTR(xh_st + 4 * xwb + c * 256), 16, 0, 0);
            }
        }
    };
    auto x_store = [&](int rg, uint2 codes, uint16_t sh) {
        if (rg < R) {
            const int j = M == 1 ? rg : rg / M, row = rg - j * M;
            ds_write_b64(lds_addr(x_st + rg * 128 + xswz(row, qsub >> 1) + (qsub & 1) * 8), codes);
            if (qsub == 0) ds_write_b32(lds_addr(xs_st + (j * XSR + row) * 4), sh);
        }
    };
    auto x_quant = [&](int r0) {  // two 4-pair chunks per step where possible (chains interleave)
        for (int c = 0; c < xwin && r0 + c < R; c += 8) {  // wave-uniform bounds
            const int rg = r0 + c + (lane >> 4);
            const bool two = c + 4 < xwin && r0 + c + 4 < R;
            v4i raw0 = ds_read_b128(lds_addr(xh_st + c * 256 + lane * 16));
            v4i raw1 = ds_read_b128(lds_addr(xh_st + (two ? c + 4 : c) * 256 + lane * 16));
            v4i up0, up1;  // PRO 2: the up window
            if (PRO == 2) {
                up0 = ds_read_b128(lds_addr(xh_st + xwb + c * 256 + lane * 16));
                up1 = ds_read_b128(lds_addr(xh_st + xwb + (two ? c + 4 : c) * 256 + lane * 16));
                asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(raw0), "+v"(raw1), "+v"(up0), "+v"(up1)::"memory");
            } else {
                // the wait redefines raw0/raw1, so no use of them can be placed above it
                asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(raw0), "+v"(raw1)::"memory");
            }
            uint4 v0 = make_uint4(raw0[0], raw0[1], raw0[2], raw0[3]);
            if (PRO == 2 && (FQ_PRO_ABL & 4)) v0 = add_residual8(v0, make_uint4(up0[0], up0[1], up0[2], up0[3]));
            else if (PRO == 2) v0 = silu_mul8(v0, make_uint4(up0[0], up0[1], up0[2], up0[3]));
            uint2 codes0;
            const uint16_t sh0 = quant_group16(v0, abits, codes0);
            x_store(rg, codes0, sh0);
            if (two) {
                uint4 v1 = make_uint4(raw1[0], raw1[1], raw1[2], raw1[3]);
                if (PRO == 2 && (FQ_PRO_ABL & 4)) v1 = add_residual8(v1, make_uint4(up1[0], up1[1], up1[2], up1[3]));
                else if (PRO == 2) v1 = silu_mul8(v1, make_uint4(up1[0], up1[1], up1[2], up1[3]));
                uint2 codes1;
                const uint16_t sh1 = quant_group16(v1, abits, codes1);
                x_store(rg + 4, codes1, sh1);
            }
        }
    };
    // PRO 3: bit planes -> int8 codes.  Lane 8 pp + q builds the 16 codes of chunk q (k = 16 q ..
    // 16 q + 15) of pair pp: per plane, bit-reverse the word (value k0 + i at bit i), then spread
    // each nibble over four bytes (x * 0x00204081 & 0x01010101) and add it in with weight 2^p, the
    // top plane with 256 - 2^(b-1) (the sign bit of a b-bit two's complement value, sign-extended
    // to the int8 byte).  The bytes never carry into each other (sum <= 255).
    auto x_unpack = [&](int r0) {
        const uint32_t sgn = 256u - (1u << (abits - 1));
        for (int c = 0; c < xwin && r0 + c < R; c += 8) {
            const int pp = c + (lane >> 3), rg = r0 + pp, q = lane & 7;
            const uint32_t pa = lds_addr(xh_st + pp * 128 + (q >> 1) * 4);
            const bool a8 = abits == 8;  // wave-uniform: planes 6 and 7 only at A8
            uint32_t w[8];
#pragma unroll
            for (int p = 0; p < 6; p++) w[p] = ds_read_b32(pa + p * 16);
            if (a8) {
                w[6] = ds_read_b32(pa + 6 * 16);
                w[7] = ds_read_b32(pa + 7 * 16);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]),
                         "+v"(w[5]), "+v"(w[6]), "+v"(w[7])::"memory");
            uint32_t o[4] = {0u, 0u, 0u, 0u};
            auto plane = [&](int p, uint32_t mul) {
                const uint32_t h = __builtin_bitreverse32(w[p]) >> (16 * (q & 1));
#pragma unroll
                for (int dd = 0; dd < 4; dd++) o[dd] += ((((h >> (4 * dd)) & 15u) * 0x00204081u) & 0x01010101u) * mul;
            };
#pragma unroll
            for (int p = 0; p < 5; p++) plane(p, 1u << p);
            plane(5, a8 ? 32u : sgn);
            if (a8) {
                plane(6, 64u);
                plane(7, sgn);
            }
            if (pp < xwin && rg < R) {
                const int j = M == 1 ? rg : rg / M, row = rg - j * M;
                ds_write_b128(lds_addr(x_st + rg * 128 + xswz(row, q)), v4i{(int)o[0], (int)o[1], (int)o[2], (int)o[3]});
            }
        }
    };

    // buffer resources of the activation codes, their scales and the image's w-scales (issue, stage_all)
    const __amdgpu_buffer_rsrc_t xqr =
        __builtin_amdgcn_make_buffer_rsrc((void *)xq, (short)0, (int)((uint32_t)M * (uint32_t)K), 0x00020000);
    const __amdgpu_buffer_rsrc_t xsr =
        __builtin_amdgcn_make_buffer_rsrc((void *)xs, (short)0, (int)((uint32_t)G * (uint32_t)ldx * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t wsr =
        __builtin_amdgcn_make_buffer_rsrc((void *)wsb, (short)0, (int)((uint32_t)NT * G * 32), 0x00020000);

    // ---- staging of the wave's scales (and unfused activation rows): issued right after the
    // first ring block (below), so that every wave's first-needed DMAs leave the CU's address unit
    // before the rest of the prologue burst; the first ring wait retires it in order.
    const int nws = (n > 0 && !SS && !(ABL & 8)) ? (n + 31) / 32 : 0;  // its instruction count
    auto stage_all = [&]() {
        if (n > 0 && !SS && !(ABL & 8)) {
            for (int i0 = 0; i0 < n; i0 += 32) {  // w-scales: 32 blocks (32 B = 2 lanes each) per instruction
                const int i = i0 + (lane >> 1) < n ? i0 + (lane >> 1) : n - 1;
                __builtin_amdgcn_global_load_lds(ws_stage_src(wsb, item_tile(i / ng), G, ga, i % ng, lane),
                                                 LDS_PTR(ws_st + i0 * 32), 16, 0, 0);
            }
            if (!FUSE) {
                for (int i0 = 0; i0 < ng; i0 += 64 / XSR) {  // x-scales: XSR per group, ushort per lane
                    const int i = i0 + lane / XSR, row = lane % XSR;
                    __builtin_amdgcn_global_load_lds(xs + (long)(ga + (i < ng ? i : ng - 1)) * ldx + (row < M ? row : M - 1),
                                                     LDS_PTR(xs_st + i0 * XSR * 4), 2, 0, 0);
                }
            }
        }
        if (n > 0 && !XS && !FUSE && !(ABL & 8)) {  // activation rows: 8 lanes x 16 B per (group, row)
            // the lane's pair rg = r0 + lane / 8 as (group j, row), stepped without a division per piece
            int j = 0, row = lane >> 3;
            while (row >= M) {
                row -= M;
                ++j;
            }
            for (int r0 = 0; r0 < R; r0 += 8) {
                const bool in = r0 + (lane >> 3) < R;  // past the last pair: a copy of pair R - 1
                const int jj = in ? j : ng - 1, rw = in ? row : M - 1;
                const int chunk = (lane & 7) ^ (rw & 7);  // lands at position lane & 7 (xswz)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(xqr, LDS_PTR(x_st + r0 * 128), 16,
                                                         (uint32_t)rw * K + (uint32_t)(ga + jj) * FQ_GROUP + chunk * 16, 0, 0, 0);
                row += 8;
                while (row >= M) {
                    row -= M;
                    ++j;
                }
            }
        }
        FQ_STAMP(7);
    };

    // ---- the ring over the wave's block sequence
    // V2 (fully staged variants): the weight DMAs address the image through a buffer resource with
    // the block's byte offset in an SGPR (advanced incrementally: +1 block per group, a jump per
    // item), so a refill is two buffer_load ... lds instructions with no per-lane 64-bit address
    // math on the path from "slot landed" to "slot refilled" (the host keeps the image < 4 GiB).
    constexpr bool V2 = FQ_DEC_V2 && XS == 0 && SS == 0;
    const __amdgpu_buffer_rsrc_t wrs =
        __builtin_amdgcn_make_buffer_rsrc((void *)wpk, (short)0, (int)((uint32_t)NT * G * FQ_BLOCK), 0x00020000);
    const uint32_t wvo = lane * 16;
    uint32_t roff = rgeo.roff;          // next block to issue
    const uint32_t rjump = rgeo.rjump;  // an item's last group -> the next item's first
    // Every DMA of the ring and the staging goes through a buffer resource with a per-lane offset fixed
    // for the launch and the block / group in an SGPR offset (never the instruction's immediate: on an
    // LDS-DMA it moves the LDS destination too), so the unfused variants' refills carry no 64-bit
    // address VALU either (the host keeps the image < 4 GiB; M x K, scales smaller still).
    uint32_t xpo[C::XP > 0 ? C::XP : 1];  // XS: the lane's activation piece offsets (row, swizzled chunk)
#pragma unroll
    for (int p = 0; p < C::XP; p++) {
        const int row = p * 8 + (lane >> 3), chunk = (lane & 7) ^ (row & 7);
        xpo[p] = (uint32_t)(row < M ? row : M - 1) * (uint32_t)K + chunk * 16;
    }
    auto issue = [&](int it, int j, int slot) {  // block (item it, group ga + j) -> slot
        const int t = item_tile(it), g = ga + j;
        char *dst = ring + slot * C::SLOT;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, LDS_PTR(dst), 16, wvo, roff, 0, FQ_W_AUX);
        if (lane < 32) __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, LDS_PTR(dst + 1024), 16, wvo, roff + 1024, 0, FQ_W_AUX);
        if constexpr (V2) return;
#pragma unroll
        for (int p = 0; p < C::XP; p++)  // activation rows [MT][128 B], swizzled chunks
            __builtin_amdgcn_raw_ptr_buffer_load_lds(xqr, LDS_PTR(dst + FQ_BLOCK + p * 1024), 16, xpo[p],
                                                     (uint32_t)g * FQ_GROUP, 0, 0);
        if (SS) {  // 16 w-scales (16 B per lane, lanes 0..1) and XSR x-scales (ushort, lanes 0..XSR-1)
            if (lane < 2)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(wsr, LDS_PTR(dst + C::WS_OFF), 16, 16 * lane,
                                                         ((uint32_t)t * G + g) * 32, 0, 0);
            if (lane < XSR)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(xsr, LDS_PTR(dst + C::XS_OFF), 2, (uint32_t)(lane < M ? lane : M - 1) * 2,
                                                         (uint32_t)g * ldx * 2, 0, 0);
        }
    };
    // Order: first activation window -> ring block 0 -> staging -> ring blocks 1 .. D-1 (exactly
    // D ring issues, unrolled; slots past a short sequence get a never-read copy of its last
    // block).  The first ring wait (vmcnt((D-1)U)) then retires block 0 and the staging, and
    // waiting for the window is vmcnt(D*U + nws).  Each wave instruction costs the CU's address
    // unit ~30 cycles whatever its size, and the prologue burst of all waves is ~60 of them: the
    // first-needed ones go first.
    // the peer-store gather kernel whose x is the previous gather's output: its wait is folded in
    // here (gather_poll), after the ring is issued; the activation window follows the poll
    const bool wfold = GAT && FUSE && pro.wgat != nullptr;
    if (FUSE && n > 0 && !wfold && !CHN) x_fetch(0);
    // the chain: lane (pair c + 4u + lane / 16, chunk lane % 16) holds 8 fp16 values of x -- as 16 bytes
    // of x itself (an input ready before the launch: gr false), or as the four 8-byte granules of the
    // previous linear's hand-off (gr)
    // A producer link reads a second source, `in` (RMSNorm: added to the residual x; SiLU: up), the same
    // way; SiLU's gate and up rows have stride ldh.
    const bool gr = CHN && pro.hx != nullptr;
    // (CHP: a chain launch whose run holds producer links -- a separate instantiation, so the plain
    // chain keeps its code)
    const int cpro = CHP ? pro.cpro : 0;
    const bool hasin = CHP && cpro != 0 && pro.in != nullptr, gin = hasin && pro.hin != nullptr;
    const uint32_t xld = CHP && cpro == 2 ? (uint32_t)pro.ldh : (uint32_t)K;  // row stride (elements)
    const uint32_t xspan = (uint32_t)(M - 1) * xld + K;                           // elements of a source
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        gr ? (void *)pro.hx : (void *)xh, (short)0, (int)(xspan * (gr ? 4 : 2)), 0x00020000);
    const __amdgpu_buffer_rsrc_t inr = __builtin_amdgcn_make_buffer_rsrc(
        gin ? (void *)pro.hin : (void *)pro.in, (short)0, (int)(xspan * (gin ? 4 : 2)), 0x00020000);
    auto chn_el = [&](int c, int u) -> uint32_t {  // element offset of the lane's 8 values
        int rg = c + 4 * u + (lane >> 4);
        rg = rg < R ? rg : R - 1;
        const int j = M == 1 ? rg : rg / M, row = rg - j * M;
        return (uint32_t)row * xld + (uint32_t)(ga + j) * FQ_GROUP + qsub * 8;
    };
    auto chn_off = [&](int c, int u) -> uint32_t { return chn_el(c, u) * (gr ? 4 : 2); };
    // a ready x's first 16 pairs are loaded ahead of the ring, so they return first.  (Granules are
    // not: a first look at the hand-off ahead of the ring made every linear slower -- the ring issue
    // behind those loads took up to 1.4 us longer)
    // A producer link that also waits for granules (its `in`) loads its ready values behind the ring
    // instead: they are not needed before the granules arrive, and ahead of the ring they delay it.
    uint4 xv0[4], gg0 = make_uint4(0, 0, 0, 0);
    const bool late = FQ_CHAIN_LATE_READY && CHP && gin;
    auto ready_loads = [&]() {
        if (CHN && !gr && n > 0) {
#pragma unroll
            for (int u = 0; u < 4; u++)
                if (4 * u < R) xv0[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, chn_off(0, u), 0, 16));
        }
        if (CHP && cpro == 1 && n > 0) gg0 = *reinterpret_cast<const uint4 *>(pro.gamma + chn_el(0, 0));  // (RMSNorm: gamma)
    };
    if (!late) ready_loads();
    int rit = 0, rj = 0;  // (item, group) of the next block to issue
    auto advance = [&]() {
        if (++rj == ng) {
            rj = 0;
            ++rit;
            roff += rjump;
        } else {
            roff += FQ_BLOCK;
        }
    };
    // (a chain linear after the first: the previous linear's tail issued these, chain_ring_ahead;
    // only the issue position advances here)
    const bool pre = CHN && FQ_CHAIN_AHEAD && pro.pre;
    if (n > 0) {
#pragma unroll
        for (int i = 0; i < D; i++) {
            if (!pre) issue(rit, rj, i);
            if (i + 1 < n) advance();  // (a short sequence re-issues its last block)
            if (i == 0 && !pre) stage_all();
        }
    }
    FQ_STAMP(1);
    FQ_CSTAMP(1);
    if (late) ready_loads();
    // a producer chain's argument block, by wave 0 of linear 0 only, issued behind its ring (needed a
    // linear later; a plain chain's smaller block was loaded as the launch started)
    typedef const uint32_t __attribute__((address_space(4))) kdword;  // (the constant address space)
    uint32_t dv[4] = {0u, 0u, 0u, 0u};
    if (CHN && CHP && pro.cwrite && wid == 0) {
        const kdword *ka = (const kdword *)(uintptr_t)pro.kargs + 4 * lane;
#pragma unroll
        for (int q = 0; q < 4; q++) dv[q] = ka[q];
    }
    if (GAT && FUSE && wfold) {
        gather_poll(pro.wgat, pro.werr, wid);
        if (n > 0) x_fetch(0);
    }
    // workgroup 0 advances the epoch around linear 1 (not in the launch whose tag wraps)
    const bool eupd = CHN && pro.link == 1 && blockIdx.x == 0 && wid == 0 && chain_late(pro.epoch) != 0x7ffffffeu;
    const uint32_t eseen = eupd ? chain_epoch_load(pro.chain) : 0u;

    // A chain wave whose wait failed -- it timed out, or the workspace's error word was set (another
    // workgroup timed out, in this launch or an earlier one) -- makes every output of its workgroup for
    // this linear fp16 NaN (its partials are NaN, so the reduction's sums are), so a caller that never
    // reads the status word cannot consume the undefined results silently.  Later
    // linears of the launch see the error word as they start and fail at once.
    bool cfail = false;
#ifndef FQ_CHAIN_NAN
#define FQ_CHAIN_NAN 1  // (development: 0 = the round-5 chain without the NaN outputs, A/B builds)
#endif
    if (CHN && !CHP && n > 0) {  // ---- the chain: activations by sc1 buffer loads to registers; from the hand-off,
        // each lane's four granules re-loaded until every tag is this launch's tag
        const uint32_t want = gr ? chain_tag(chain_late(pro.epoch)) : 0u;
        uint32_t *err = pro.chain + 32 * FQ_CHAIN_ERR;
        bool failed = gr && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
        for (int c = 0; c < R; c += 16) {  // wave-uniform
            uint4 v[4];
            uint32_t off[4];
#pragma unroll
            for (int u = 0; u < 4; u++) off[u] = chn_off(c, u);
            if (!gr && c == 0) {
#pragma unroll
                for (int u = 0; u < 4; u++) v[u] = xv0[u];
            } else if (!gr) {
#pragma unroll
                for (int u = 0; u < 4; u++)
                    if (c + 4 * u < R) v[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, off[u], 0, 16));
            } else {
                for (int spin = 0; spin < (1 << 20); spin++) {
                    // every granule load of the pass in flight at once, then the tag compares (a
                    // short-circuit && between them serialises one round trip per load pair)
                    uint4 g0[4], g1[4];
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        if (c + 4 * u < R) {
                            g0[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, off[u], 0, 16));
                            g1[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, off[u] + 16, 0, 16));
                        }
                    }
                    bool ok = true;
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        if (c + 4 * u < R) {
                            v[u] = make_uint4(g0[u].x, g0[u].z, g1[u].x, g1[u].z);
                            ok = ok & (g0[u].y == want) & (g0[u].w == want) & (g1[u].y == want) & (g1[u].w == want);
                        }
                    }
                    if (__builtin_amdgcn_ballot_w64(!ok) == 0 || failed) break;
                    __builtin_amdgcn_s_sleep(FQ_CHAIN_SLEEP);
                    if (spin == (1 << 20) - 1) {
                        failed = true;
                        if (lane == 0) chain_fail(pro.chain);
                    }
                }
                if (c == 0) FQ_CSTAMP(6);  // (development stamps: the first pass's tags all matched)
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                if (c + 4 * u >= R) break;
                uint2 codes;
                const uint16_t sh = quant_group16(v[u], abits, codes);
                x_store(c + 4 * u + (lane >> 4), codes, sh);
            }
        }
        cfail = failed;
        FQ_CSTAMP(2);
    } else if (CHP && n > 0) {  // ---- the chain with producer links (a separate instantiation): two sources
        // each lane's four granules re-loaded until every tag is this launch's tag
        const uint32_t want = (gr || gin) ? chain_tag(chain_late(pro.epoch)) : 0u;
        uint32_t *err = pro.chain + 32 * FQ_CHAIN_ERR;
        bool failed = (gr || gin) && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
        for (int c = 0; c < R; c += 16) {  // wave-uniform
            uint4 v[4], w[4];  // x (RMSNorm: the residual; SiLU: gate) and `in`
#pragma unroll
            for (int u = 0; u < 4; u++) w[u] = make_uint4(0, 0, 0, 0);
            // both sources: ready values load once, granules until their tags match -- a source whose
            // tags all matched is not loaded again (the other's re-polls do not queue behind it)
            bool dx = !gr, din = !gin;
            for (int spin = 0; spin < (1 << 20); spin++) {
                // every load of the pass in flight at once, then the tag compares (a short-circuit &&
                // between them serialises one round trip per load pair)
                uint4 gx0[4], gx1[4], gi0[4], gi1[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    if (c + 4 * u < R) {
                        const uint32_t el = chn_el(c, u);
                        if (!gr) {
                            if (spin == 0)
                                v[u] = c == 0 ? xv0[u] : __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, el * 2, 0, 16));
                        } else if (!dx) {
                            gx0[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, el * 4, 0, 16));
                            gx1[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, el * 4 + 16, 0, 16));
                        }
                        if (hasin && !gin) {
                            if (spin == 0) w[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(inr, el * 2, 0, 16));
                        } else if (gin && !din) {
                            gi0[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(inr, el * 4, 0, 16));
                            gi1[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(inr, el * 4 + 16, 0, 16));
                        }
                    }
                }
                bool okx = true, okin = true;
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    if (c + 4 * u < R) {
                        if (gr && !dx) {
                            v[u] = make_uint4(gx0[u].x, gx0[u].z, gx1[u].x, gx1[u].z);
                            okx = okx & (gx0[u].y == want) & (gx0[u].w == want) & (gx1[u].y == want) & (gx1[u].w == want);
                        }
                        if (gin && !din) {
                            w[u] = make_uint4(gi0[u].x, gi0[u].z, gi1[u].x, gi1[u].z);
                            okin = okin & (gi0[u].y == want) & (gi0[u].w == want) & (gi1[u].y == want) & (gi1[u].w == want);
                        }
                    }
                }
                dx = dx || __builtin_amdgcn_ballot_w64(!okx) == 0;  // (wave-uniform)
                din = din || __builtin_amdgcn_ballot_w64(!okin) == 0;
                if ((dx && din) || failed) break;
                __builtin_amdgcn_s_sleep(FQ_CHAIN_SLEEP);
                if (spin == (1 << 20) - 1) {
                    failed = true;
                    if (lane == 0) chain_fail(pro.chain);
                }
            }
            FQ_CSTAMP(6);
            cfail = failed;
            if (CHP && cpro == 1) {  // residual add + RMSNorm (M = 1, K = 4 x 128 x NW: lane = chunk 64 wid + lane,
                                  // as the fused producer kernel, PRO 1 above -- the same bits)
                uint4 r = v[0];
                const uint4 gg = gg0;
                if (hasin) {
                    r = add_residual8(w[0], r);
                    if (failed) r = make_uint4(0x7e007e00u, 0x7e007e00u, 0x7e007e00u, 0x7e007e00u);  // (NaN residual)
                    if (blockIdx.x == 0) {
                        *reinterpret_cast<uint4 *>(pro.res_out + chn_el(0, 0)) = r;
                        if (pro.hr) {  // the residual for a later linear of the chain: four granules
                            const uint32_t rw[4] = {r.x, r.y, r.z, r.w};
                            const uint64_t tg = (uint64_t)chain_tag(chain_late(pro.epoch)) << 32;
#pragma unroll
                            for (int q = 0; q < 4; q++)
                                __hip_atomic_store(pro.hr + chn_el(0, 0) / 2 + q, tg | rw[q], __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
                        }
                    }
                }
                float acc = wave_sum64(sumsq8(r, 0.0f));
                if (lane == 0) ds_write_b32(lds_addr(wsum) + 4 * wid, __float_as_uint(acc));
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                FQ_CSTAMP(7);
                v4i s0 = ds_read_b128(lds_addr(wsum)), s1 = ds_read_b128(lds_addr(wsum) + 16);
                asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(s0), "+v"(s1)::"memory");
                float ss = __int_as_float(s0[0]);
#pragma unroll
                for (int q = 1; q < NW; q++) ss = ss + __int_as_float(q < 4 ? s0[q] : s1[q - 4]);
                uint2 codes;
                const uint16_t sh = quant_group16(rms_apply8(r, gg, rms_scale(ss, K, pro.eps)), abits, codes);
                x_store(lane >> 4, codes, sh);
                break;  // (R = 4: one chunk)
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                if (c + 4 * u >= R) break;
                uint2 codes;
                const uint4 q = CHP && cpro == 2 ? silu_mul8(v[u], w[u]) : v[u];
                const uint16_t sh = quant_group16(q, abits, codes);
                x_store(c + 4 * u + (lane >> 4), codes, sh);
            }
        }
        FQ_CSTAMP(2);
    }
    if (CHN && pro.cwrite && wid == 0) {  // (the chain's argument copy -> LDS; landed with the inputs)
        if (CHP)
            ds_write_b128(pro.cdesc_lds + lane * 16, v4i{(int)dv[0], (int)dv[1], (int)dv[2], (int)dv[3]});
        else
            ds_write_b64(pro.cdesc_lds + lane * 8, make_uint2(pro.dvx, pro.dvy));
    }
    if (CHN) {
    } else if (FUSE && n > 0) {  // ---- codes -> x_st, scales -> xs_st
        if (GAT && wfold)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the window was issued after the ring)
        else
            wait_vm_plus<D * C::U>(nws);
        FQ_STAMP(5);
        if (PRO == 1) {  // residual add + RMSNorm over the row (R = 4 pairs: lane = chunk 64 wid + lane)
            const uint32_t xb = lds_addr(xh_st) + lane * 16;
            v4i rr = ds_read_b128(xb), ii = ds_read_b128(xb + xwb), gg = ds_read_b128(xb + 2 * xwb);
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(rr), "+v"(ii), "+v"(gg)::"memory");
            uint4 r = make_uint4(rr[0], rr[1], rr[2], rr[3]);
            if (pro.in) {
                r = add_residual8(make_uint4(ii[0], ii[1], ii[2], ii[3]), r);
                if (blockIdx.x == 0) *reinterpret_cast<uint4 *>(pro.res_out + 8 * (64 * wid + lane)) = r;
            }
            float acc = sumsq8(r, 0.0f), ss = acc;
            if (!(FQ_PRO_ABL & 1)) {
                acc = wave_sum64(acc);  // (fq_producers.hip's tree)
                if (lane == 0) ds_write_b32(lds_addr(wsum) + 4 * wid, __float_as_uint(acc));
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                v4i s0 = ds_read_b128(lds_addr(wsum)), s1 = ds_read_b128(lds_addr(wsum) + 16);
                asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(s0), "+v"(s1)::"memory");
                ss = __int_as_float(s0[0]);
#pragma unroll
                for (int w = 1; w < NW; w++) ss = ss + __int_as_float(w < 4 ? s0[w] : s1[w - 4]);
            }
            uint2 codes;
            const uint16_t sh = quant_group16(rms_apply8(r, make_uint4(gg[0], gg[1], gg[2], gg[3]), rms_scale(ss, K, pro.eps)),
                                              abits, codes);
            x_store(lane >> 4, codes, sh);
        } else if (PRO == 4) {  // bias + residual + input, LayerNorm (lane = chunk 64 wid + lane, as PRO 1)
            const uint32_t xb = lds_addr(xh_st) + lane * 16;
            v4i rr = ds_read_b128(xb), ii = ds_read_b128(xb + xwb), gg = ds_read_b128(xb + 2 * xwb);
            v4i be = ds_read_b128(xb + 3 * xwb), bi = ds_read_b128(xb + 4 * xwb);
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(rr), "+v"(ii), "+v"(gg), "+v"(be), "+v"(bi)::"memory");
            const uint4 in4 = make_uint4(ii[0], ii[1], ii[2], ii[3]), bi4 = make_uint4(bi[0], bi[1], bi[2], bi[3]);
            const uint4 be4 = make_uint4(be[0], be[1], be[2], be[3]);
            float v[8];
            ln_add8(pro.in ? &in4 : nullptr, make_uint4(rr[0], rr[1], rr[2], rr[3]), pro.bias ? &bi4 : nullptr, v);
            const uint4 h = ln_pack8(v);
            if (blockIdx.x == 0 && pro.res_out) *reinterpret_cast<uint4 *>(pro.res_out + 8 * (64 * wid + lane)) = h;
            float s = 0.0f, q = 0.0f;
            ln_sums8(v, s, q);
            s = wave_sum64(s);
            q = wave_sum64(q);
            if (lane == 0) {
                ds_write_b32(lds_addr(wsum) + 4 * wid, __float_as_uint(s));
                ds_write_b32(lds_addr(wsum) + 4 * (NW + wid), __float_as_uint(q));
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            v4i s0 = ds_read_b128(lds_addr(wsum)), s1 = ds_read_b128(lds_addr(wsum) + 16);
            v4i q0 = ds_read_b128(lds_addr(wsum) + 4 * NW), q1 = ds_read_b128(lds_addr(wsum) + 4 * NW + 16);
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(s0), "+v"(s1), "+v"(q0), "+v"(q1)::"memory");
            float S = __int_as_float(s0[0]), Q = __int_as_float(q0[0]);
#pragma unroll
            for (int w = 1; w < NW; w++) {
                S = S + __int_as_float(w < 4 ? s0[w] : s1[w - 4]);
                Q = Q + __int_as_float(w < 4 ? q0[w] : q1[w - 4]);
            }
            uint2 codes;
            const uint16_t sh = quant_group16(ln_apply8(h, ln_stats(S, Q, K, pro.eps), make_uint4(gg[0], gg[1], gg[2], gg[3]),
                                                        pro.beta ? &be4 : nullptr),
                                              abits, codes);
            x_store(lane >> 4, codes, sh);
        } else if (PRO == 3) {
            x_unpack(0);
        } else if (!(ABL & 2048)) {  // (development 2048: no quantizer, codes left undefined)
            x_quant(0);
        }
        FQ_STAMP(6);
        if (ABL & 32) {  // development: the same code once more (instruction cache now warm);
            if (!(ABL & 64)) x_quant(0);  // with 64: nothing, i.e. the cost of a stamp itself
            FQ_STAMP(4);
        }
        for (int r0 = xwin; r0 < R; r0 += xwin) {  // M > 4 or long K: later windows
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the previous window was read
            x_fetch(r0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (PRO == 3)
                x_unpack(r0);
            else
                x_quant(r0);
        }
    }

    const uint32_t otag = CHN ? chain_tag(chain_late(pro.epoch)) : 0u;  // (the chain's output granules)
    int arow[RG];  // A-operand rows (rows >= M mirror row M-1, never stored)
#pragma unroll
    for (int rg = 0; rg < RG; rg++) arow[rg] = 16 * rg + (lane & 15) < M ? 16 * rg + (lane & 15) : M - 1;
    if (ABL & 4096) {  // (development: every lane reads activation row 0 -- the M = 1 LDS access pattern)
#pragma unroll
        for (int rg = 0; rg < RG; rg++) arow[rg] = 0;
    }
    const int Npad = NT * 16;
    int i = 0;     // position in the wave's block sequence
    int rslot = 0;  // its ring slot (V2: counted, no i % D)
    for (int it = 0; it < nit; it++) {
        const int t = item_tile(it);
        const int col = 16 * t + (lane & 15);
        float cur[RG][4];
#pragma unroll
        for (int rg = 0; rg < RG; rg++)
#pragma unroll
            for (int r = 0; r < 4; r++) cur[rg][r] = 0.f;
        // V2: block j's dequant runs after block j + 1's MFMAs are issued (same item), so the wave
        // does not stall on the MFMA result between a refill and the next ring wait
        v4i pacc[RG];
        __half2 pp01[RG], pp23[RG];
        for (int j = 0; j < ng; j++, i++) {
            const int g = ga + j, slot = V2 ? rslot : i % D;
            if (V2 && i + D <= n) {
                wait_ring_steady<C::U, D>();  // D - 1 younger blocks in flight: the common case
            } else {
                const int later = (n - 1 - i) < (D - 1) ? (n - 1 - i) : (D - 1);
                wait_ring<C::U, D>(later);  // this slot (and every older DMA, the staging included) landed
            }
            if (i == 0) {
                FQ_STAMP(2);
                FQ_CSTAMP(3);
            }
            const uint32_t sp = lds_addr(ring + slot * C::SLOT);
            v2u p0 = ds_read_b64(sp + lane * 8);
            v2u p1 = ds_read_b64(sp + 512 + lane * 8);
            v2u p2 = ds_read_b64(sp + 1024 + lane * 8);
            v4i a[RG][2];
#pragma unroll
            for (int rg = 0; rg < RG; rg++) {
                const uint32_t xrow = XS ? sp + FQ_BLOCK + arow[rg] * FQ_GROUP
                                         : lds_addr(x_st + (j * M + arow[rg]) * FQ_GROUP);
#pragma unroll
                for (int s = 0; s < 2; s++) a[rg][s] = ds_read_b128(xrow + xswz(arow[rg], 4 * s + (lane >> 4)));
            }
            const uint32_t wsa = (SS ? sp + C::WS_OFF : lds_addr(ws_st) + i * 32) + 2 * (lane & 15);
            uint32_t wsv = ds_read_u16(wsa);
            v4i xd[RG];  // x-scales of rows 16rg + 4(lane>>4) .. +3, one per dword
            const uint32_t xsa = SS ? sp + C::XS_OFF : lds_addr(xs_st + j * XSR * 4);
#pragma unroll
            for (int rg = 0; rg < RG; rg++) xd[rg] = ds_read_b128(xsa + 4 * (16 * rg + 4 * (lane >> 4)));
            if constexpr (V2) {
                // LDS reads return in order: once the three plane reads (the only bytes read from
                // the slot; activations and scales are staged elsewhere) have landed, refill the
                // slot, then wait for the rest
                asm volatile("s_waitcnt lgkmcnt(%3)" : "+v"(p0), "+v"(p1), "+v"(p2) : "i"(3 * RG + 1) : "memory");
                __builtin_amdgcn_sched_barrier(0);
                if (i + D < n) {  // refill: block i + D
                    issue(rit, rj, slot);
                    advance();
                }
                rslot = rslot + 1 == D ? 0 : rslot + 1;
                asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(wsv)::"memory");
#pragma unroll
                for (int rg = 0; rg < RG; rg++) asm volatile("" : "+v"(a[rg][0]), "+v"(a[rg][1]), "+v"(xd[rg]));
                __builtin_amdgcn_sched_barrier(0);
            } else {
                // every read has landed, and the slot's bytes are in registers before its refill
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_sched_barrier(0);
                if (i + D < n) {  // refill: block i + D
                    issue(rit, rj, slot);
                    advance();
                }
            }

            if (ABL & 2) {
                cur[0][0] += (float)(p0[0] ^ p1[1] ^ p2[0] ^ a[0][1][0]) + (float)wsv + (float)xd[0][0];
                continue;
            }
            v4i b0, b1;
            if (ABL & 256) {  // (development: no unpack -- the raw plane words as operands)
                b0 = v4i{(int)p0[0], (int)p1[0], (int)p2[0], (int)p0[1]};
                b1 = v4i{(int)p1[1], (int)p2[1], (int)p0[0], (int)p1[0]};
            } else {
                b0 = unpack_fq6(p0[0], p1[0], p2[0]);
                b1 = unpack_fq6(p0[1], p1[1], p2[1]);
            }
            const __half2 w2 = __half2half2(__ushort_as_half((uint16_t)wsv));
#pragma unroll
            for (int rg = 0; rg < RG; rg++) {
                v4i acc;
                if (ABL & 512) {  // (development: no MFMA)
                    acc = v4i{a[rg][0][0] ^ b0[0], a[rg][0][1] ^ b0[1], a[rg][1][2] ^ b1[2], a[rg][1][3] ^ b1[3]};
                } else {
                    acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[rg][0], b0, v4i{0, 0, 0, 0}, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[rg][1], b1, acc, 0, 0, 0);
                }
                const uint32_t x01 = __builtin_amdgcn_perm((uint32_t)xd[rg][1], (uint32_t)xd[rg][0], 0x05040100u);
                const uint32_t x23 = __builtin_amdgcn_perm((uint32_t)xd[rg][3], (uint32_t)xd[rg][2], 0x05040100u);
                const __half2 p01 = __hmul2(*reinterpret_cast<const __half2 *>(&x01), w2);  // fp16-rounded
                const __half2 p23 = __hmul2(*reinterpret_cast<const __half2 *>(&x23), w2);  // scale product
                if (V2) {
                    if (j > 0) dequant4<ABL>(cur[rg], pacc[rg], pp01[rg], pp23[rg]);
                    pacc[rg] = acc;
                    pp01[rg] = p01;
                    pp23[rg] = p23;
                } else {
                    dequant4<ABL>(cur[rg], acc, p01, p23);
                }
                if (DBG) {
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const int row = 16 * rg + 4 * (lane >> 4) + r;
                        if (row < M && col < N) acc_dbg[((long)row * N + col) * G + g] = acc[r] >> 2;
                    }
                }
            }
        }
        if (V2 && ng > 0 && !(ABL & 2)) {  // the item's last block
#pragma unroll
            for (int rg = 0; rg < RG; rg++) dequant4<ABL>(cur[rg], pacc[rg], pp01[rg], pp23[rg]);
        }

        // ---- item end: the wave's partial tile goes to reduction slot it % RC; every RC items
        // (RC = IPW when LDS allows: once, after the stream) the WG sums the slots' NW partials
        // in a fixed order.  Raw s_barriers: the ring's DMA for later items stays in flight.
        if (ABL & 4) {
            if (lane < 16 && col < N) d[col] = f2h(cur[0][0]);
            continue;
        }
        const int rs = it % RC;
#pragma unroll
        for (int rg = 0; rg < RG; rg++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int row = 16 * rg + 4 * (lane >> 4) + r;
                if (row < M) red[(rs * NW + wid) * EM + row * 16 + (lane & 15)] = cur[rg][r] * 0.25f;
            }
        // the chain's failed wait: NaN partials, overwritten in LDS (a branch that leaves cur alone: one that
        // set cur to NaN changed the register allocation enough to add a vmcnt(0) -- the next linear's whole
        // ring -- at the chain's link loop head, 1.7 % per step)
        if (CHN && FQ_CHAIN_NAN && cfail) {  // (wave-uniform)
            const uint32_t nan = 0x7fc00000u;
#pragma unroll
            for (int rg = 0; rg < RG; rg++)
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int row = 16 * rg + 4 * (lane >> 4) + r;
                    if (row < M) ds_write_b32(lds_addr(red + (rs * NW + wid) * EM + row * 16 + (lane & 15)), nan);
                }
        }
        if (rs == RC - 1 || it == nit - 1) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
            // (k = e / EM by a multiply-high with ceil(2^32 / EM): exact while e * EM < 2^32 -- e < IPW * EM
            // with IPW <= 4096 and EM <= 512 -- instead of a per-element integer division)
            const uint32_t emi = (uint32_t)(0xffffffffu / (uint32_t)EM) + 1u;
            if ((GAT || CHN || QE) && S == 1) {  // peer-store gather / chain / QE: two adjacent columns per thread
                for (int e = 2 * threadIdx.x; e < (rs + 1) * EM; e += 2 * NW * 64) {
                    const int k = (int)(((uint64_t)(uint32_t)e * emi) >> 32), ee = e - k * EM;
                    float v0 = 0.f, v1 = 0.f;
#pragma unroll
                    for (int w = 0; w < NW; w++) {
                        v0 += red[(k * NW + w) * EM + ee];
                        v1 += red[(k * NW + w) * EM + ee + 1];
                    }
                    if (QE)  // (sc1: the group's last arriver re-loads it; N % 128 == 0, so the pair is in range)
                        __hip_atomic_store(reinterpret_cast<uint32_t *>(d + (long)(ee >> 4) * N + 16 * item_tile(it - rs + k) + (ee & 15)),
                                           (uint32_t)f2h(v0) | ((uint32_t)f2h(v1) << 16), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    else if (CHN)
                        chain_store2(d, pro.hd, otag, N, ee >> 4,
                                     16 * item_tile(it - rs + k) + (ee & 15), v0, v1);
                    else
                        gather_store2(gat, gat->P, ee >> 4, 16 * item_tile(it - rs + k) + (ee & 15), v0, v1);
                }
            } else
            for (int e = threadIdx.x; e < (rs + 1) * EM; e += NW * 64) {
                const int k = (int)(((uint64_t)(uint32_t)e * emi) >> 32), ee = e - k * EM;
                float v = 0.f;
#pragma unroll
                for (int w = 0; w < NW; w++) v += red[(k * NW + w) * EM + ee];
                const int row = ee >> 4, nn = 16 * item_tile(it - rs + k) + (ee & 15);
                if (S == 1) {
                    if (nn < N) d[(long)row * N + nn] = f2h(v);
                } else {
                    __hip_atomic_store(&slabs[((long)z * M + row) * Npad + nn], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            if (it + 1 < nit) {  // the slots are reused by the next items
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
    FQ_STAMP(3);
    FQ_CSTAMP(4);
    if constexpr (QE) {  // (S = 1)
        decode_qe_epilogue<NW>(nit, M, N, t0, tstep, tickets, d, flag, qe);
        return;
    }
    if constexpr (CHN) {  // (S = 1)
        if (eupd) chain_epoch_update(pro.chain, chain_late(pro.epoch), eseen, gridall);
        // the next linear's prologue reuses the LDS: every wave is past this one's
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        FQ_CSTAMP(5);
        if (FQ_CHAIN_AHEAD && pro.nxt_w) {
            chain_ring_ahead<MT>(pro.nxt_w, pro.nxt_p);
            if (!CHP) FQ_CSTAMP(7);  // (development stamps: the next linear's ring issued)
        }
        return;
    }
    // GAT is a separate instantiation: the gather's branches and publish step cost the plain
    // kernel ~3.5 % per launch when they are only runtime-dead (A/B over round 3's builds,
    // tools/ab_bisect.sh)
    if (!GAT) {
        if (S == 1 || (ABL & 4)) return;
        decode_splitk_fixup<NW, false>(nit, S, M, N, Npad, EM, t0, tstep, slabs, tickets, d, flag, nullptr);
        FQ_STAMP(4);
        return;
    }
    if (S > 1 && !(ABL & 4)) decode_splitk_fixup<NW, true>(nit, S, M, N, Npad, EM, t0, tstep, slabs, tickets, d, flag, gat);
    gather_publish(gat);
}

// The kernels around decode_body.  The plain one keeps the short argument list: its explicit
// arguments and the hidden block count it reads stay within the first 128 bytes of the kernarg
// segment -- 40 more bytes of (unused) arguments cost the plain launch ~2.5 % (A/B/A/B,
// tools/ab_karg.sh).  The peer-store gather and the fused producers have kernels of their own with
// lists of the same length.
#define FQ_DECODE_ARGS                                                                                              \
    const int8_t *__restrict__ xq, const uint16_t *__restrict__ xs, const uint16_t *__restrict__ xh, int abits,      \
        const uint32_t *__restrict__ wpk, int Mall, int N, int K, uint16_t *__restrict__ d,                          \
        int32_t *__restrict__ acc_dbg, float *__restrict__ slabs, uint32_t *__restrict__ tickets, int S, int IPW,    \
        int RC, int xwin, int iq, int ir, int NCH
#define FQ_DECODE_PASS xq, xs, xh, abits, wpk, Mall, N, K, d, acc_dbg, slabs, tickets, S, IPW, RC, xwin, iq, ir, NCH
// The plain kernel (the headline launch) takes 56 bytes of arguments -- five pointers and four
// dwords of bit fields (decode_pack) -- which fq_gemm.hip's build preloads into SGPRs
// (-amdgpu-kernarg-preload-count, Makefile): the launch reads no kernarg memory before its first
// DMA (A/B x 3: 0.6-1 % per step, tools/ab_preload.sh).  The debug accumulator output takes the long
// list (fq_gemm_decode_dbg_kernel).
struct DecodePacked {
    uint32_t w0, w1, w2, w3;
};
// w0 = N (21 bits) | abits << 21 (4) | xwin << 25 (6); w1 = G (13) | S << 13 (10) | NCH << 23 (4);
// w2 = IPW (16) | RC << 16 (16); w3 = Mall (10) | ir << 10 (11) | grid << 21 (11)
static bool decode_pack(int N, int K, int abits, int xwin, int S, int NCH, int IPW, int RC, int Mall, int ir,
                        int grid, DecodePacked *p) {
    const int G = K / FQ_GROUP;
    if (N >= (1 << 21) || abits > 15 || xwin > 63 || G >= (1 << 13) || S >= (1 << 10) || NCH > 15 ||
        IPW > 0xffff || RC > 0xffff || Mall >= (1 << 10) || ir >= (1 << 11) || grid >= (1 << 11))
        return false;
    p->w0 = (uint32_t)N | ((uint32_t)abits << 21) | ((uint32_t)xwin << 25);
    p->w1 = (uint32_t)G | ((uint32_t)S << 13) | ((uint32_t)NCH << 23);
    p->w2 = (uint32_t)IPW | ((uint32_t)RC << 16);
    p->w3 = (uint32_t)Mall | ((uint32_t)ir << 10) | ((uint32_t)grid << 21);
    return true;
}
template <int MT, int XS, int SS, bool FUSE, int ABL = 0, bool CH = false>
__global__ __launch_bounds__(decode_waves(MT) * 64) void fq_gemm_decode_kernel(
    const void *__restrict__ x, const uint16_t *__restrict__ xs, const uint32_t *__restrict__ wpk,
    uint16_t *__restrict__ d, char *__restrict__ ws, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
    const int N = w0 & 0x1fffff, abits = (w0 >> 21) & 15, xwin = w0 >> 25;
    const int K = (w1 & 0x1fff) * FQ_GROUP, S = (w1 >> 13) & 1023, NCH = w1 >> 23;
    const int IPW = w2 & 0xffff, RC = w2 >> 16;
    const int Mall = w3 & 1023, ir = (w3 >> 10) & 2047, grid = w3 >> 21;
    const int iq = IPW - (ir != 0);  // items per WG: IPW = ceil, iq = floor (decode_plan)
    decode_body<MT, XS, SS, FUSE, false, ABL, CH, 0, false>(
        FUSE ? nullptr : reinterpret_cast<const int8_t *>(x), xs, FUSE ? reinterpret_cast<const uint16_t *>(x) : nullptr,
        abits, wpk, Mall, N, K, d, nullptr, reinterpret_cast<float *>(ws + FQ_TICKET_BYTES),
        reinterpret_cast<uint32_t *>(ws), S, IPW, RC, xwin, iq, ir, NCH, nullptr, DecodePro{}, grid);
}
// The plain kernel with the next linear's codes in its epilogue (decode_qe_epilogue): the same preloaded
// fields, then the quantizer's outputs (needed only at the end, read from kernarg memory).
template <int MT, int XS, int SS>
__global__ __launch_bounds__(decode_waves(MT) * 64) void fq_gemm_decode_q_kernel(
    const int8_t *__restrict__ xq, const uint16_t *__restrict__ xs, const uint32_t *__restrict__ wpk,
    uint16_t *__restrict__ d, char *__restrict__ ws, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3,
    int8_t *__restrict__ qxq, uint16_t *__restrict__ qxs, int qM, int qK, int qbits) {
    const int N = w0 & 0x1fffff, abits = (w0 >> 21) & 15, xwin = w0 >> 25;
    const int K = (w1 & 0x1fff) * FQ_GROUP;
    const int IPW = w2 & 0xffff, RC = w2 >> 16;
    const int Mall = w3 & 1023, ir = (w3 >> 10) & 2047, grid = w3 >> 21;
    decode_body<MT, XS, SS, false, false, 0, false, 0, false, false, false, true>(
        xq, xs, nullptr, abits, wpk, Mall, N, K, d, nullptr, nullptr, reinterpret_cast<uint32_t *>(ws), 1, IPW, RC,
        xwin, IPW - (ir != 0), ir, 1, nullptr, DecodePro{}, grid, DecodeQ{qxq, qxs, qM, qK, qbits});
}
template <int MT, int XS, int SS, bool FUSE, bool CH>
__global__ __launch_bounds__(decode_waves(MT) * 64) void fq_gemm_decode_dbg_kernel(FQ_DECODE_ARGS) {
    decode_body<MT, XS, SS, FUSE, true, 0, CH, 0, false>(FQ_DECODE_PASS, nullptr, DecodePro{});
}
// The peer-store gather's kernel: the same list with the gather descriptor in the debug output's
// place (no debug output with a gather).
template <int MT, int XS, int SS, bool FUSE>
__global__ __launch_bounds__(decode_waves(MT) * 64) void fq_gemm_decode_gather_kernel(
    const int8_t *__restrict__ xq, const uint16_t *__restrict__ xs, const uint16_t *__restrict__ xh, int abits,
    const uint32_t *__restrict__ wpk, int Mall, int N, int K, uint16_t *__restrict__ d,
    const fq_gather *__restrict__ gat, float *__restrict__ slabs, uint32_t *__restrict__ tickets, int S, int IPW,
    int RC, int xwin, int iq, int ir, int NCH, const fq_gather *__restrict__ wgat, uint32_t *__restrict__ werr) {
    DecodePro pro{};
    pro.wgat = wgat;
    pro.werr = werr;
    decode_body<MT, XS, SS, FUSE, false, 0, false, 0, true>(xq, xs, xh, abits, wpk, Mall, N, K, d, nullptr, slabs,
                                                            tickets, S, IPW, RC, xwin, iq, ir, NCH, gat, pro);
}
#undef FQ_DECODE_ARGS
#undef FQ_DECODE_PASS
// The fused producers' kernel: what the first DMA needs -- the window sources and the packed
// fields -- in the 56 preloaded bytes, the output, workspace and residual output after them (loaded
// at entry, first waited on after the window has arrived).
template <int MT, int PRO>
__global__ __launch_bounds__(decode_waves(MT) * 64) void fq_gemm_decode_pro_kernel(
    const uint16_t *__restrict__ xh, const uint32_t *__restrict__ wpk, const uint16_t *__restrict__ pin,
    const uint16_t *__restrict__ gamma, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, int ldh, float eps,
    uint16_t *__restrict__ d, char *__restrict__ ws, uint16_t *__restrict__ res_out) {
    const int N = w0 & 0x1fffff, abits = (w0 >> 21) & 15, xwin = w0 >> 25;
    const int K = (w1 & 0x1fff) * FQ_GROUP, S = (w1 >> 13) & 1023;
    const int IPW = w2 & 0xffff, RC = w2 >> 16;
    const int Mall = w3 & 1023, ir = (w3 >> 10) & 2047, grid = w3 >> 21;
    const DecodePro pro = {pin, gamma, res_out, eps, ldh, nullptr, nullptr};
    decode_body<MT, 0, 0, true, false, 0, false, PRO, false>(
        nullptr, nullptr, xh, abits, wpk, Mall, N, K, d, nullptr, reinterpret_cast<float *>(ws + FQ_TICKET_BYTES),
        reinterpret_cast<uint32_t *>(ws), S, IPW, RC, xwin, IPW - (ir != 0), ir, 1, nullptr, pro, grid);
}

// The fused LayerNorm producer's kernel (PRO 4, M = 1): the pro kernel's list with beta and bias
// after the packed fields.
template <int MT>
__global__ __launch_bounds__(decode_waves(MT) * 64) void fq_gemm_decode_ln_kernel(
    const uint16_t *__restrict__ xh, const uint32_t *__restrict__ wpk, const uint16_t *__restrict__ pin,
    const uint16_t *__restrict__ gamma, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3,
    const uint16_t *__restrict__ beta, const uint16_t *__restrict__ bias, float eps, uint16_t *__restrict__ d,
    char *__restrict__ ws, uint16_t *__restrict__ res_out) {
    const int N = w0 & 0x1fffff, abits = (w0 >> 21) & 15, xwin = w0 >> 25;
    const int K = (w1 & 0x1fff) * FQ_GROUP, S = (w1 >> 13) & 1023;
    const int IPW = w2 & 0xffff, RC = w2 >> 16;
    const int Mall = w3 & 1023, ir = (w3 >> 10) & 2047, grid = w3 >> 21;
    const DecodePro pro = {pin, gamma, res_out, eps, K, beta, bias};
    decode_body<MT, 0, 0, true, false, 0, false, 4, false>(
        nullptr, nullptr, xh, abits, wpk, Mall, N, K, d, nullptr, reinterpret_cast<float *>(ws + FQ_TICKET_BYTES),
        reinterpret_cast<uint32_t *>(ws), S, IPW, RC, xwin, IPW - (ir != 0), ir, 1, nullptr, pro, grid);
}

// The launch whose tag would wrap (workgroup 0 left the epoch alone): the last workgroup to arrive clears
// every granule (all the others are done reading), the start counter and the epoch.
__device__ __forceinline__ void chain_wrap_end(uint32_t *__restrict__ sync, uint32_t epoch, uint4 *hand,
                                               uint32_t hand_bytes) {
    if (chain_late(epoch) != 0x7ffffffeu) return;
    __syncthreads();
    __shared__ uint32_t last;
    if (threadIdx.x == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this workgroup's start arrival has been performed
        last = __hip_atomic_fetch_add(sync + 32 * FQ_CHAIN_DONE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
               gridDim.x - 1;
    }
    __syncthreads();
    if (last) {
        for (uint32_t i = threadIdx.x; i < hand_bytes / 16; i += blockDim.x) hand[i] = make_uint4(0, 0, 0, 0);
        if (threadIdx.x < 8) __hip_atomic_store(sync + 32 * threadIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (threadIdx.x == 0) {
            __hip_atomic_store(sync + 32 * FQ_CHAIN_DONE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(sync + 32 * FQ_CHAIN_EPOCH, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// The decode chain's kernel: the links' packed fields (decode_pack) by value in the kernel
// arguments (read from LDS as each linear starts); every linear runs the fused plan fq_linear_w6ax
// would run for it (S = 1, the same grid), so the bits are the same.  Two argument layouts: a plain
// chain's links (56 B) and a producer chain's (ChainLinkP, 104 B: the producer's operands too).
struct ChainLinkP {
    const uint16_t *x;       // plain: x; RMSNorm: the residual; SiLU: gate
    const uint32_t *w;
    uint16_t *d;
    const uint64_t *hx;      // x's granules (the previous link's hand-off + offset, or an earlier RMSNorm
                             // link's residual output), or null: x is ready
    uint64_t *hd;            // this link's hand-off granules, or null
    const uint16_t *in;      // RMSNorm: added to the residual (or null); SiLU: up
    const uint64_t *hin;     // in's granules (the previous link's hand-off + offset), or null: ready
    const uint16_t *gamma;   // RMSNorm
    uint16_t *res_out;       // RMSNorm with in
    uint64_t *hr;            // RMSNorm: granules of res_out for a later link, or null
    uint32_t w0, w1, w2, w3;
    float eps;
    uint32_t ldh_pro;        // SiLU row stride (24 bits) | producer << 24
};
struct ChainLinkPlain {
    const uint16_t *x;
    const uint32_t *w;
    uint16_t *d;
    const uint64_t *hx;
    uint64_t *hd;
    uint32_t w0, w1, w2, w3;
};
// The sync pointer and link 0 (a plain linear) lead the arguments as scalars (the first 48 bytes
// preloaded into SGPRs at wave start -- an aggregate argument is not --, link 0's hand-off pointer
// after them: it is read at the epilogue); the other links follow in a struct.  A copy of the
// argument block reaches VGPRs in linear 0 (plain: 512 B, two dwords per lane as every wave starts;
// producer: 1 KiB, four dwords per lane of wave 0, behind its ring), wave 0 writes it to LDS once
// linear 0's input has arrived (so nothing waits for it), and every later linear reads its link from
// LDS (no wait on the memory counter, which would also wait for the previous linear's stores).
template <class LINK, int PAD>
struct ChainTail {
    LINK l[FQ_CHAIN_MAX - 1];  // links 1 ..
    uint4 *hand;               // the hand-off region (cleared when the tag wraps)
    uint32_t hand_bytes;
    int n;                     // >= 2
    uint32_t pad[PAD];         // (producer: the argument block is >= 1 KiB, the copy reads 1 KiB)
};
typedef ChainTail<ChainLinkPlain, 13> ChainTailPlain;
typedef ChainTail<ChainLinkP, 56> ChainTailP;
constexpr int FQ_CHAIN_TAIL_OFF = 56;  // the tail's byte offset in the arguments
// each copy reads exactly the explicit arguments (never past them into hidden arguments): the pads
// make the argument block at least as long as the copy
static_assert(sizeof(ChainLinkP) == 104 && FQ_CHAIN_TAIL_OFF + sizeof(ChainTailP) >= 1024 &&
              FQ_CHAIN_TAIL_OFF + offsetof(ChainTailP, pad) <= 1024, "the producer copy is 64 lanes x 16 bytes");
static_assert(sizeof(ChainLinkPlain) == 56 && FQ_CHAIN_TAIL_OFF + sizeof(ChainTailPlain) >= 512 &&
              FQ_CHAIN_TAIL_OFF + offsetof(ChainTailPlain, pad) <= 512, "the plain copy is 64 lanes x 8 bytes");
template <int MT, bool CHP>
__device__ __forceinline__ void chain_link(uint32_t *sync, int l, const ChainLinkP &L, uint32_t epoch, DecodePro pro) {
    const int N = L.w0 & 0x1fffff, abits = (L.w0 >> 21) & 15, xwin = L.w0 >> 25;
    const int K = (L.w1 & 0x1fff) * FQ_GROUP;
    const int IPW = L.w2 & 0xffff, RC = L.w2 >> 16;
    const int Mall = L.w3 & 1023, ir = (L.w3 >> 10) & 2047, grid = L.w3 >> 21;
    pro.chain = sync;
    pro.link = l;
    pro.epoch = epoch;
    pro.hx = L.hx;
    pro.hd = L.hd;
    if (CHP) {
        pro.in = L.in;
        pro.hin = L.hin;
        pro.gamma = L.gamma;
        pro.res_out = L.res_out;
        pro.hr = L.hr;
        pro.eps = L.eps;
        pro.ldh = (int)(L.ldh_pro & 0xffffff);
        pro.cpro = (int)(L.ldh_pro >> 24);
    }
    decode_body<MT, 0, 0, true, false, 0, false, 0, false, true, CHP>(
        nullptr, nullptr, L.x, abits, L.w, Mall, N, K, L.d, nullptr, nullptr, nullptr, 1, IPW, RC, xwin,
        IPW - (ir != 0), ir, 1, nullptr, pro, grid);
}
template <int MT, bool CHP>
__global__ __launch_bounds__(decode_waves(MT) * 64) void fq_gemm_decode_chain_kernel(
    uint32_t *__restrict__ sync, const uint16_t *x0, const uint32_t *w0p, uint16_t *d0, uint32_t p0, uint32_t p1,
    uint32_t p2, uint32_t p3, uint64_t *hd0, const std::conditional_t<CHP, ChainTailP, ChainTailPlain> t) {
    typedef std::conditional_t<CHP, ChainLinkP, ChainLinkPlain> LINK;
    __shared__ __attribute__((aligned(16))) uint32_t cdesc[CHP ? 256 : 128];
    DecodePro p0r{};
    p0r.kargs = (uint64_t)(uintptr_t)__builtin_amdgcn_kernarg_segment_ptr();
    if (!CHP) {
        typedef const uint32_t __attribute__((address_space(4))) kdword;  // (the constant address space)
        const kdword *ka = (const kdword *)__builtin_amdgcn_kernarg_segment_ptr();
        const int lane = threadIdx.x & 63;
        p0r.dvx = ka[2 * lane];
        p0r.dvy = ka[2 * lane + 1];
    }
    p0r.cwrite = true;
    p0r.cdesc_lds = lds_addr(cdesc);
    // link 1's descriptor (the tail's first link; a run has >= 2 links), for linear 0's tail
    p0r.nxt_w = lds_addr(cdesc) + FQ_CHAIN_TAIL_OFF + offsetof(LINK, w);
    p0r.nxt_p = lds_addr(cdesc) + FQ_CHAIN_TAIL_OFF + offsetof(LINK, w0);
    // the launch's epoch (used through chain_late, a linear later)
    const uint32_t epoch = __hip_atomic_load(sync + 32 * FQ_CHAIN_EPOCH, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ChainLinkP L0{};
    L0.x = x0;
    L0.w = w0p;
    L0.d = d0;
    L0.hd = hd0;
    L0.w0 = p0;
    L0.w1 = p1;
    L0.w2 = p2;
    L0.w3 = p3;
    chain_link<MT, CHP>(sync, 0, L0, epoch, p0r);
    // this workgroup has read the epoch (its tags were stored): arrive on the start counter
    if (threadIdx.x == 0)
        __hip_atomic_fetch_add(sync + 32 * (blockIdx.x & 7), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t cb = lds_addr(cdesc);
    auto rd2 = [&](int k) -> uint2 {  // dwords k, k + 1 of the arguments (k even), from LDS
        uint2 v;
        asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(cb + 4 * k) : "memory");
        return make_uint2(__builtin_amdgcn_readfirstlane(v.x), __builtin_amdgcn_readfirstlane(v.y));
    };
    typedef std::conditional_t<CHP, ChainTailP, ChainTailPlain> TAIL;
    constexpr int T0 = FQ_CHAIN_TAIL_OFF / 4, LW = sizeof(LINK) / 4;
    static_assert(T0 % 2 == 0 && LW % 2 == 0 && offsetof(TAIL, n) % 8 == 4, "ds_read_b64 pairs");
    const int n = (int)rd2(T0 + offsetof(TAIL, n) / 4 - 1).y;
    // a link's descriptor: its LW / 2 dword pairs read back to back, one wait (a wait per pair cost
    // ~0.35 us between two linears: seven serial LDS round trips)
    auto rdlink = [&](int b, uint2 *v) {
        if constexpr (LW == 14) {
            asm volatile(
                "ds_read_b64 %0, %7\n\tds_read_b64 %1, %7 offset:8\n\tds_read_b64 %2, %7 offset:16\n\t"
                "ds_read_b64 %3, %7 offset:24\n\tds_read_b64 %4, %7 offset:32\n\tds_read_b64 %5, %7 offset:40\n\t"
                "ds_read_b64 %6, %7 offset:48\n\ts_waitcnt lgkmcnt(0)"
                : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6])
                : "v"(cb + 4 * b)
                : "memory");
        } else {
            static_assert(LW == 26, "descriptor layouts");
            asm volatile(
                "ds_read_b64 %0, %13\n\tds_read_b64 %1, %13 offset:8\n\tds_read_b64 %2, %13 offset:16\n\t"
                "ds_read_b64 %3, %13 offset:24\n\tds_read_b64 %4, %13 offset:32\n\tds_read_b64 %5, %13 offset:40\n\t"
                "ds_read_b64 %6, %13 offset:48\n\tds_read_b64 %7, %13 offset:56\n\tds_read_b64 %8, %13 offset:64\n\t"
                "ds_read_b64 %9, %13 offset:72\n\tds_read_b64 %10, %13 offset:80\n\tds_read_b64 %11, %13 offset:88\n\t"
                "ds_read_b64 %12, %13 offset:96\n\ts_waitcnt lgkmcnt(0)"
                : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7]),
                  "=&v"(v[8]), "=&v"(v[9]), "=&v"(v[10]), "=&v"(v[11]), "=&v"(v[12])
                : "v"(cb + 4 * b)
                : "memory");
        }
#pragma unroll
        for (int k = 0; k < LW / 2; k++)
            v[k] = make_uint2(__builtin_amdgcn_readfirstlane(v[k].x), __builtin_amdgcn_readfirstlane(v[k].y));
    };
    auto p64 = [](uint2 a) -> uint64_t { return (uint64_t)a.x | ((uint64_t)a.y << 32); };
    for (int l = 1; l < n; l++) {
        uint2 v[LW / 2];
        rdlink(T0 + (l - 1) * LW, v);
        ChainLinkP L{};
        L.x = reinterpret_cast<const uint16_t *>(p64(v[0]));
        L.w = reinterpret_cast<const uint32_t *>(p64(v[1]));
        L.d = reinterpret_cast<uint16_t *>(p64(v[2]));
        L.hx = reinterpret_cast<const uint64_t *>(p64(v[3]));
        L.hd = reinterpret_cast<uint64_t *>(p64(v[4]));
        constexpr int WO = offsetof(LINK, w0) / 8;
        if constexpr (CHP) {
            L.in = reinterpret_cast<const uint16_t *>(p64(v[5]));
            L.hin = reinterpret_cast<const uint64_t *>(p64(v[6]));
            L.gamma = reinterpret_cast<const uint16_t *>(p64(v[7]));
            L.res_out = reinterpret_cast<uint16_t *>(p64(v[8]));
            L.hr = reinterpret_cast<uint64_t *>(p64(v[9]));
            L.eps = __uint_as_float(v[WO + 2].x);
            L.ldh_pro = v[WO + 2].y;
        }
        L.w0 = v[WO].x;
        L.w1 = v[WO].y;
        L.w2 = v[WO + 1].x;
        L.w3 = v[WO + 1].y;
        DecodePro pr{};
        pr.pre = true;  // (linear l - 1's tail issued this linear's ring)
        if (l + 1 < n) {
            pr.nxt_w = cb + 4 * (T0 + l * LW) + offsetof(LINK, w);
            pr.nxt_p = cb + 4 * (T0 + l * LW) + offsetof(LINK, w0);
        }
        chain_link<MT, CHP>(sync, l, L, epoch, pr);
    }
    chain_wrap_end(sync, epoch, t.hand, t.hand_bytes);
}

// Wait until every rank of a peer-store gather has published this generation (one workgroup; lane q
// polls rank q's flag with system-scope loads, sleeping between polls), then acquire and advance
// the generation.  Bounded: after ~1 s the error word is set and the kernel returns (results are
// then undefined, never a hang); once the error word is set every later wait returns at once, so a
// broken peer path costs one timeout, not one per call.
__global__ __launch_bounds__(64) void fq_gather_wait_kernel(const fq_gather *__restrict__ gat, uint32_t *__restrict__ err) {
    const int lane = threadIdx.x;
    if (err && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) return;
    const uint32_t target = __hip_atomic_load(gat->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // (publish advanced it)
    const uint32_t *mine = gat->flags[gat->rank];
    bool ok = lane >= gat->P;
    for (int spin = 0; spin < (1 << 20); spin++) {  // ~1 s at ~1 us per poll
        if (!ok) ok = __hip_atomic_load(mine + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= target;
        if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;
        __builtin_amdgcn_s_sleep(8);
    }
    if (__builtin_amdgcn_ballot_w64(!ok) != 0) {
        if (lane == 0 && err) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope
}

// =============================================================================================
// Prefill kernel (M > 32): int8-MFMA bound.  WG tile 128 (M) x 128 (N), 4 waves as 2 x 2, each
// wave 64 x 64 = 4 x 4 tiles of 16x16; one k-step per 128-wide group; two WGs per CU, so that one
// WG's barrier / LDS-latency chain overlaps the other's MFMAs.
//
// What bounds it (rocprofv3 + tools/prefill_ablate.py): the VALU beside the MFMAs and the serial
// latency chain of each group step, not LDS or HBM bandwidth.  So:
//   * the fq6 weights are unpacked ONCE per WG and group: each wave DMAs the three planes of two
//     tiles (16 B per lane and plane = two block lanes, two groups ahead) into its own small LDS
//     buffer, unpacks both k-steps at the start of the step before and writes the int8 B operands
//     to LDS; every wave then reads ready MFMA operands;
//   * A (128 rows x 128 B, 16-byte chunks XOR-swizzled by row & 7, xswz) and the group's scales
//     arrive by LDS-DMA (global_load_lds, 16 B per lane), one group ahead, two stages;
//   * the MFMA takes the weights as its A operand and the activations as B, so each lane ends with
//     4 consecutive output columns of one row: 8-byte output stores, and the w-scales of those
//     columns are one 8-byte LDS read;
//   * dequant per element and group: one v_cvt_f32_i32 and one v_fma_mix_f32 with the fp16 scale
//     product (half(xs * ws), two per v_pk_mul_f16) -- the reference's rounding.
// One raw barrier per group.  Every wave issues 8 DMA instructions per group (4 of A, one of
// scales or a filler, 3 weight planes).  All LDS accesses are inline asm: the compiler cannot
// tell them from the DMA still landing and would drain it with vmcnt(0); waits are counted here.
// =============================================================================================
constexpr int PF_BM = 128, PF_BN = 128, PF_TILES = PF_BN / 16, PF_WAVES = 4;
constexpr int PF_XS_OFF = PF_BM * FQ_GROUP;        // A: 16 KiB, then the x-scales, one per dword
constexpr int PF_WS_OFF = PF_XS_OFF + PF_BM * 4;   // w-scales of the 8 tiles (fp16 [8][16])
constexpr int PF_PAD_OFF = PF_WS_OFF + PF_BN * 2;  // filler DMA target (never read)
constexpr int PF_ASTAGE = PF_PAD_OFF + 16;         // 17168 B, two stages
constexpr int PF_BSTAGE = PF_TILES * 2 * 1024;     // unpacked B: [tile][k-step][lane][16 B], two stages
constexpr int PF_VM_A = 5, PF_VM_W = 3;            // per wave and group: A + scale DMAs, weight planes
// s_waitcnt immediate (gfx9 encoding) that waits for vmcnt <= n only
constexpr int vmcnt_only(int n) { return (n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8); }

// ABL (development ablations, FQ_DEV_ABLATION builds only): 1 = no dequant (accumulators kept
// alive, no VALU), 2 = no MFMA (operands kept alive), 4 = no compute-side LDS reads, 8 = no
// global loads / DMA, 16 = no output stores, 32 = no A DMA, 64 = no weight loads.
// U8: the weights arrive already unpacked (fq_unpack_w8_kernel: the int8 B operands of every
// (tile, group) exactly as unpack_w writes them to LDS, [NT][G][k-step][lane][16 B]), by LDS-DMA
// with A into the same B stage: no plane buffer, no unpack VALU, no ds_write, one DMA stream.
template <bool DBG, int ABL = 0, bool U8 = false>
__global__ __launch_bounds__(PF_WAVES * 64, 2) void fq_gemm_prefill_kernel(
    const int8_t *__restrict__ xq, const uint16_t *__restrict__ xs, const uint32_t *__restrict__ wpk, int M,
    int N, int K, uint16_t *__restrict__ d, int32_t *__restrict__ acc_dbg, const char *__restrict__ wu, int S,
    float *__restrict__ slabs) {
    __shared__ __attribute__((aligned(16))) char sa[2 * PF_ASTAGE];
    __shared__ __attribute__((aligned(16))) char sbu[2 * PF_BSTAGE];
    __shared__ __attribute__((aligned(16))) char sraw[U8 ? 16 : PF_WAVES * 3072];
    const int G = K / FQ_GROUP, NT = (N + 15) / 16;
    const uint16_t *wsb = reinterpret_cast<const uint16_t *>(reinterpret_cast<const char *>(wpk) + (size_t)NT * G * FQ_BLOCK);
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wid >> 1, wn = wid & 1;

    // Block order: the bijective XCD remap (consecutive logical tiles run on one XCD), then groups
    // of 8 M-panels walked M-fastest, so the WGs resident on an XCD share A and B k-slices in L2.
    const int nbm = (M + PF_BM - 1) / PF_BM, nbn = (NT + PF_TILES - 1) / PF_TILES, nwg = nbm * nbn;
    // split-K (S > 1, few tiles): WG b takes tile b / S and groups [g0, g1) of split z = b % S
    const int bid = S == 1 ? (int)blockIdx.x : (int)((unsigned)blockIdx.x / (unsigned)S);
    const int z = (int)blockIdx.x - bid * S;
    const int g0 = (int)((unsigned)(z * G) / (unsigned)S), g1 = (int)((unsigned)((z + 1) * G) / (unsigned)S);
    const int xcd = bid % 8, q = nwg / 8, rr = nwg % 8;
    const int lid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / 8;
    const int span = 8 * nbn, first = (lid / span) * 8;
    const int gsz = nbm - first < 8 ? nbm - first : 8;
    const int bm = first + (lid % span) % gsz, bn = (lid % span) / gsz;
    const int m0 = bm * PF_BM, t0 = bn * PF_TILES;

    // ---- per-lane sources at group 0 (a group adds 128 B to A, 1536 B to B, M or 16 to scales)
    const int8_t *asrc[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int row = 32 * wid + 8 * i + (lane >> 3);
        const int m = m0 + row < M ? m0 + row : M - 1;  // rows past M are computed, never stored
        asrc[i] = xq + (size_t)m * K + ((lane & 7) ^ (row & 7)) * 16;
    }
    const int srow = 64 * (wid & 1) + lane;  // waves 0-1: x-scales of rows 64w .. 64w + 63
    const uint16_t *xsrc = xs + (m0 + srow < M ? m0 + srow : M - 1);
    const int wt = t0 + (lane >> 1) < NT ? t0 + (lane >> 1) : NT - 1;  // wave 2: the w-scales
    const uint16_t *wsrc = wsb + (size_t)wt * G * 16 + 8 * (lane & 1);
    const int btile = 2 * wid + (lane >> 5);  // tiles 2w, 2w + 1; block lanes 2j, 2j + 1
    const int bt = t0 + btile < NT ? t0 + btile : NT - 1;
    const char *bsrc = reinterpret_cast<const char *>(wpk) + (size_t)bt * G * FQ_BLOCK + (lane & 31) * 16;
    const char *usrc[2];  // U8: tiles 2w, 2w + 1 of the unpacked operands, this lane's 16 B
#pragma unroll
    for (int t = 0; t < 2; t++) {
        const int ut = t0 + 2 * wid + t < NT ? t0 + 2 * wid + t : NT - 1;
        usrc[t] = wu + (size_t)ut * G * 2048 + lane * 16;
    }

    const uint32_t la = lds_addr(sa), lbu = lds_addr(sbu);
    auto stage = [&](int g, int slot) {  // A + scales of group g -> A stage `slot` (PF_VM_A)
        if (ABL & 8) return;
        char *buf = sa + slot * PF_ASTAGE;
#pragma unroll
        for (int i = 0; i < 4; i++)
            if (!(ABL & 32))
                __builtin_amdgcn_global_load_lds(asrc[i] + g * FQ_GROUP, LDS_PTR(buf + (32 * wid + 8 * i) * FQ_GROUP), 16, 0, 0);
        if (wid < 2)
            __builtin_amdgcn_global_load_lds(xsrc + (size_t)g * M, LDS_PTR(buf + PF_XS_OFF + 64 * wid * 4), 2, 0, 0);
        else if (lane < (wid == 2 ? 16 : 1))
            __builtin_amdgcn_global_load_lds(wsrc + (wid == 2 ? g * 16 : 0), LDS_PTR(buf + (wid == 2 ? PF_WS_OFF : PF_PAD_OFF)), 16, 0, 0);
        if (U8 && !(ABL & 64)) {
            char *bdst = sbu + slot * PF_BSTAGE + 2 * wid * 2048;
#pragma unroll
            for (int t = 0; t < 2; t++)
#pragma unroll
                for (int k = 0; k < 2; k++)
                    __builtin_amdgcn_global_load_lds(usrc[t] + (size_t)g * 2048 + k * 1024, LDS_PTR(bdst + t * 2048 + k * 1024), 16, 0, 0);
        }
    };
    // The weight planes go through a small per-wave LDS buffer (DMA like A): values loaded into
    // VGPRs by inline asm a whole step before their use would be invisible to the register
    // allocator's notion of time, so a copy or re-use of those registers could race the load.
    // Wave w's buffer is [plane][tile 2w, 2w + 1][512 B] (the DMA is lane-linear, 16 B = block
    // lanes 2j, 2j + 1 per lane); each lane then reads back the 8-byte pieces of ITS block lane in
    // both tiles, so that the unpacked operands are written lane-linearly (no bank conflicts).
    const uint32_t lraw = lds_addr(sraw) + wid * 3072 + lane * 8;
    auto load_w = [&](int g) {  // three planes of group g -> the wave's raw buffer (PF_VM_W)
        if (ABL & (8 | 64)) return;
#pragma unroll
        for (int r = 0; r < 3; r++)
            __builtin_amdgcn_global_load_lds(bsrc + (size_t)g * FQ_BLOCK + r * 512, LDS_PTR(sraw + wid * 3072 + r * 1024), 16, 0, 0);
    };
    v2u raw[2][3];  // [tile 2w + t][plane]
    auto read_w = [&]() {  // the wave's raw buffer (landed) -> registers
        raw[0][0] = ds_read_b64_at<0>(lraw);
        raw[0][1] = ds_read_b64_at<1024>(lraw);
        raw[0][2] = ds_read_b64_at<2048>(lraw);
        raw[1][0] = ds_read_b64_at<512>(lraw);
        raw[1][1] = ds_read_b64_at<1536>(lraw);
        raw[1][2] = ds_read_b64_at<2560>(lraw);
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(raw[0][0]), "+v"(raw[0][1]), "+v"(raw[0][2]), "+v"(raw[1][0]), "+v"(raw[1][1]), "+v"(raw[1][2])::"memory");
    };
    auto unpack_w = [&](int bslot) {  // raw -> int8 B operands of tiles 2w, 2w + 1, both k-steps
        const uint32_t wa = lbu + bslot * PF_BSTAGE + 2 * wid * 2048 + lane * 16;
#pragma unroll
        for (int t = 0; t < 2; t++) {
            ds_write_b128(wa + t * 2048, unpack_fq6(raw[t][0][0], raw[t][1][0], raw[t][2][0]));
            ds_write_b128(wa + t * 2048 + 1024, unpack_fq6(raw[t][0][1], raw[t][1][1], raw[t][2][1]));
        }
    };

    // LDS read offsets: the wave's A rows (xswz: row & 7 == lane & 7 for every 16-row tile), the
    // x-scale of the lane's row per tile, its B operands and the w-scales of its 4 columns per tile
    const int arow = wm * 64 + (lane & 15);
    const uint32_t a_off0 = arow * FQ_GROUP + xswz(arow, lane >> 4), a_off1 = arow * FQ_GROUP + xswz(arow, 4 + (lane >> 4));
    const uint32_t x_off = PF_XS_OFF + arow * 4;
    const uint32_t w_off = PF_WS_OFF + (wn * 64 + 4 * (lane >> 4)) * 2;
    const uint32_t b_off = wn * 4 * 2048 + lane * 16;

    float out[4][4][4];  // [mi][ni][r]: row 16 mi + (lane & 15), column 16 ni + 4 (lane >> 4) + r
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 4; j++)
#pragma unroll
            for (int r = 0; r < 4; r++) out[i][j][r] = 0.f;

    // prologue: A stage 0 and the weights of group 0; unpack them; weights of group 1
    stage(g0, 0);
    if (!U8) {
        load_w(g0);
        __builtin_amdgcn_s_waitcnt(vmcnt_only(0));
        read_w();
        load_w(g1 > g0 + 1 ? g0 + 1 : g0);
        unpack_w(0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    } else {
        __builtin_amdgcn_s_waitcnt(vmcnt_only(0));
    }

    // Step g: barrier (A stage g, B operands g in LDS; every wave done with step g - 1) -> issue A
    // stage g + 1 -> the weights of group g + 1 (loaded a step ago) to registers, their buffer
    // refilled with group g + 2, unpacked to LDS -> MFMAs on group g -> wait for A stage g + 1.
    for (int g = g0; g < g1; g++) {
        const int gl = g - g0;  // stage parity
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        stage(g + 1 < g1 ? g + 1 : g1 - 1, (gl + 1) & 1);  // past the last group: never-read copies,
        if (!U8) {                                          // so every path issues the same count
            __builtin_amdgcn_s_waitcnt(vmcnt_only(PF_VM_A));
            read_w();
            load_w(g + 2 < g1 ? g + 2 : g1 - 1);
            unpack_w((gl + 1) & 1);
        }

        const uint32_t ab = la + (gl & 1) * PF_ASTAGE, bb = lbu + (gl & 1) * PF_BSTAGE + b_off;
        v4i b[4][2];
        v2u wv[4];
        v4i a[4][2];
        uint32_t xv[4];
        if (ABL & 4) {
#pragma unroll
            for (int i = 0; i < 4; i++) {
                b[i][0] = b[i][1] = a[i][0] = a[i][1] = v4i{(int)ab, (int)bb, g, i};
                wv[i] = v2u{ab + i, bb};
                xv[i] = bb + i;
            }
        } else {
#define FQ_PF_B(ni)                                                \
        b[ni][0] = ds_read_b128_at<(ni) * 2048>(bb);                \
        b[ni][1] = ds_read_b128_at<(ni) * 2048 + 1024>(bb);         \
        wv[ni] = ds_read_b64_at<(ni) * 32>(ab + w_off);
        FQ_PF_B(0) FQ_PF_B(1) FQ_PF_B(2) FQ_PF_B(3)
#undef FQ_PF_B
#define FQ_PF_A(mi)                                                    \
        a[mi][0] = ds_read_b128_at<(mi) * 16 * FQ_GROUP>(ab + a_off0); \
        a[mi][1] = ds_read_b128_at<(mi) * 16 * FQ_GROUP>(ab + a_off1); \
        xv[mi] = ds_read_b32_at<(mi) * 64>(ab + x_off);
        FQ_PF_A(0) FQ_PF_A(1) FQ_PF_A(2) FQ_PF_A(3)
#undef FQ_PF_A
        }
        // (the 4 unpack writes are older than these reads: the counts below cover them)
        asm volatile("s_waitcnt lgkmcnt(12)"
                     : "+v"(b[0][0]), "+v"(b[0][1]), "+v"(b[1][0]), "+v"(b[1][1]), "+v"(b[2][0]), "+v"(b[2][1]),
                       "+v"(b[3][0]), "+v"(b[3][1]), "+v"(wv[0]), "+v"(wv[1]), "+v"(wv[2]), "+v"(wv[3]));
        // Blocks j = (mi, ni) in order, the dequant of block j - 1 pinned after the MFMAs of block j
        // (as in fq_gemm_prefill_big_kernel: the accumulators' latency is covered by those MFMAs)
        v4i accq[2];
        auto dequant = [&](const v4i acc, int mi, int ni) {
            // the fp16-rounded scale products w * xs (v_pk_mul_f16, xs broadcast by op_sel_hi)
            const uint32_t q01 = pk_mul_f16_lo(wv[ni][0], xv[mi]), q23 = pk_mul_f16_lo(wv[ni][1], xv[mi]);
            const __half2 p01 = __builtin_bit_cast(__half2, q01), p23 = __builtin_bit_cast(__half2, q23);
            float *o = out[mi][ni];
            o[0] = fmaf((float)acc[0], __low2float(p01), o[0]);
            o[1] = fmaf((float)acc[1], __high2float(p01), o[1]);
            o[2] = fmaf((float)acc[2], __low2float(p23), o[2]);
            o[3] = fmaf((float)acc[3], __high2float(p23), o[3]);
            if (DBG) {
                const int m = m0 + arow + mi * 16;
                const int n = (t0 + wn * 4 + ni) * 16 + 4 * (lane >> 4);
#pragma unroll
                for (int r = 0; r < 4; r++)
                    if (m < M && n + r < N) acc_dbg[((size_t)m * N + n + r) * G + g] = acc[r] >> 2;
            }
        };
#pragma unroll
        for (int j = 0; j <= 16; j++) {
            if (j < 16) {
                const int mi = j >> 2, ni = j & 3;
                if (ni == 0) {
                    if (mi == 0) asm volatile("s_waitcnt lgkmcnt(9)" : "+v"(a[0][0]), "+v"(a[0][1]), "+v"(xv[0]));
                    if (mi == 1) asm volatile("s_waitcnt lgkmcnt(6)" : "+v"(a[1][0]), "+v"(a[1][1]), "+v"(xv[1]));
                    if (mi == 2) asm volatile("s_waitcnt lgkmcnt(3)" : "+v"(a[2][0]), "+v"(a[2][1]), "+v"(xv[2]));
                    if (mi == 3) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[3][0]), "+v"(a[3][1]), "+v"(xv[3]));
                }
                if (ABL & 2) {
                    asm volatile("" ::"v"(a[mi][0]), "v"(a[mi][1]), "v"(b[ni][0]), "v"(b[ni][1]), "v"(xv[mi]), "v"(wv[ni]));
                } else {
                    // weights as the A operand: acc[r] = column 4 (lane >> 4) + r, row lane & 15
                    v4i acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[ni][0], a[mi][0], v4i{0, 0, 0, 0}, 0, 0, 0);
                    accq[j & 1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[ni][1], a[mi][1], acc, 0, 0, 0);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            if (j > 0 && !(ABL & 2)) {
                const int pj = j - 1;
                if (ABL & 1)
                    asm volatile("" ::"v"(accq[pj & 1]), "v"(xv[pj >> 2]), "v"(wv[pj & 3]));
                else
                    dequant(accq[pj & 1], pj >> 2, pj & 3);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        // A stage g + 1 landed (the weights of group g + 2 may stay in flight); the unpack writes
        // retired with the reads above.  (sched_barrier: keep the wait below the MFMA block.)
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_waitcnt(vmcnt_only(U8 ? 0 : PF_VM_W));
    }
    // the copies past the last group are still landing: LDS must be quiet before the WG retires
    __builtin_amdgcn_s_waitcnt(vmcnt_only(0));

    if (S > 1) {  // fp32 partial tile -> split z's slab [z][M][Npad]; fq_splitk_reduce_kernel sums them
        const size_t Npad = (size_t)NT * 16;
#pragma unroll
        for (int mi = 0; mi < 4; mi++) {
            const int m = m0 + arow + mi * 16;
#pragma unroll
            for (int ni = 0; ni < 4; ni++) {
                const int tn = t0 + wn * 4 + ni;
                const float *o = out[mi][ni];
                if (!(ABL & 16) && m < M && tn < NT)
                    *reinterpret_cast<float4 *>(slabs + ((size_t)z * M + m) * Npad + tn * 16 + 4 * (lane >> 4)) =
                        make_float4(o[0] * 0.25f, o[1] * 0.25f, o[2] * 0.25f, o[3] * 0.25f);
            }
        }
        return;
    }
    // 4 consecutive columns per lane: one 8-byte store when N keeps them 8-byte aligned
    const bool vec = (N & 3) == 0;
#pragma unroll
    for (int mi = 0; mi < 4; mi++) {
        const int m = m0 + arow + mi * 16;
#pragma unroll
        for (int ni = 0; ni < 4; ni++) {
            const int n = (t0 + wn * 4 + ni) * 16 + 4 * (lane >> 4);
            const float *o = out[mi][ni];
            if (ABL & 16) {
                asm volatile("" ::"v"(o[0]), "v"(o[1]), "v"(o[2]), "v"(o[3]));
            } else if (m < M) {
                uint16_t *dst = d + (size_t)m * N + n;
                if (vec && n + 3 < N) {
                    const uint32_t lo = (uint32_t)f2h(o[0] * 0.25f) | ((uint32_t)f2h(o[1] * 0.25f) << 16);
                    const uint32_t hi = (uint32_t)f2h(o[2] * 0.25f) | ((uint32_t)f2h(o[3] * 0.25f) << 16);
                    *reinterpret_cast<uint2 *>(dst) = make_uint2(lo, hi);
                } else {
#pragma unroll
                    for (int r = 0; r < 4; r++)
                        if (n + r < N) dst[r] = f2h(o[r] * 0.25f);
                }
            }
        }
    }
}

// Split-K finish: d = fp16(sum over z = 0 .. S-1 of slab z), in z order (deterministic), four
// columns per thread.  Traffic: 4 S M Npad bytes read, 2 M N written.
__global__ __launch_bounds__(256) void fq_splitk_reduce_kernel(const float *__restrict__ slabs, int S, int M, int N,
                                                                uint16_t *__restrict__ d) {
    const int NT = (N + 15) / 16, q4 = NT * 4;  // float4 columns per row
    const long idx = (long)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (long)M * q4) return;
    const int m = (int)(idx / q4), c = (int)(idx - (long)m * q4);
    const size_t stride = (size_t)M * NT * 16;
    const float4 *src = reinterpret_cast<const float4 *>(slabs + (size_t)m * NT * 16) + c;
    float4 v = src[0];
    for (int zz = 1; zz < S; zz++) {
        const float4 w = *reinterpret_cast<const float4 *>(reinterpret_cast<const float *>(src) + zz * stride);
        v.x += w.x;
        v.y += w.y;
        v.z += w.z;
        v.w += w.w;
    }
    const int n = 4 * c;
    uint16_t *dst = d + (size_t)m * N + n;
    const uint16_t h[4] = {f2h(v.x), f2h(v.y), f2h(v.z), f2h(v.w)};
    if ((N & 3) == 0 && n + 3 < N) {
        *reinterpret_cast<uint2 *>(dst) = make_uint2(h[0] | ((uint32_t)h[1] << 16), h[2] | ((uint32_t)h[3] << 16));
    } else {
#pragma unroll
        for (int r = 0; r < 4; r++)
            if (n + r < N) dst[r] = h[r];
    }
}

// Large-M prefill on 256 x 256 workgroup tiles (the U8 path, M >= PF_U8_MIN_M).  Measured on the
// 128 x 128 kernel above (tools/prefill_ablate.py, M = 16384): its data-movement skeleton alone --
// no MFMA, no dequant -- takes 47 % of the launch, and per CU and group step it moves 72 LDS-DMA
// pieces (TA-issued at ~30 cycles each) and reads 128 KiB of fragments from LDS (1024 cycles at
// 128 B/clk) for 4.2 M MACs (1031 MFMA cycles at peak): the LDS and the address unit, not the
// MFMA, bound it.  Here one workgroup of 8 waves per CU owns 256 rows x 256 columns; each wave a
// 128 x 64 tile (8 x 4 blocks of 16 x 16, the same MFMA core, dequant, operand layouts and
// epilogue as fq_gemm_prefill_kernel): per group step 66 DMA pieces and 192 KiB of fragment
// reads for 8.4 M MACs -- half the DMA and three quarters of the LDS reads per MAC.  Two stages
// of 65.5 KiB (A 32 KiB + scales, unpacked B 32 KiB).  Bit-identical to the 128 x 128 kernels.
constexpr int PB_BM = 256, PB_TILES = 16, PB_WAVES = 8;
constexpr int PB_XS_OFF = PB_BM * FQ_GROUP;          // A: 32 KiB, then the x-scales, one per dword
constexpr int PB_WS_OFF = PB_XS_OFF + PB_BM * 4;     // w-scales of the 16 tiles (fp16 [16][16])
constexpr int PB_ASTAGE = PB_WS_OFF + PB_TILES * 32; // 33.5 KiB
constexpr int PB_BSTAGE = PB_TILES * 2 * 1024;       // unpacked B: [tile][k-step][lane][16 B]

#ifdef FQ_DEV_ABLATION
// development (ABL & 32): per-wave cycle sums of the group-step segments (barrier wait, stage DMA
// issue, compute, trailing DMA wait) for the first 256 workgroups, tools/pb_stamps.py
__device__ unsigned long long g_pb_stamps[256 * PB_WAVES * 4];
#define PB_STAMP(k)                                                                          \
    if (ABL & 32) {                                                                          \
        __builtin_amdgcn_sched_barrier(0);                                                   \
        unsigned long long t_;                                                               \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");            \
        __builtin_amdgcn_sched_barrier(0);                                                   \
        if ((k) >= 0) pb_seg[(k) < 0 ? 0 : (k)] += t_ - pb_t;                                \
        pb_t = t_;                                                                           \
    }
#else
#define PB_STAMP(k)
#endif

// ABL: development ablations as in fq_gemm_prefill_kernel (1, 2, 4, 8, 16; 32 stamps; 64 no priority).  XSF (M % 256 == 0:
// every row tile full, its x-scales 16-byte aligned): the 256 x-scales of a group arrive packed in
// one 512-byte DMA piece instead of four 64-lane ushort pieces into dword slots.
// QO: the epilogue also quantizes the fp16 output for the next linear (PbQ; N % 128 == 0): a tile
// row's 256 columns are two whole 128-column groups, each held by a pair of waves (wn 0-1, 2-3).
struct PbQ {
    int8_t *qx;    // int8 [qM][qK]: the output's leading qM * qK values, read row-major as qM x qK
    uint16_t *qs;  // fp16 [qK / 128][qM]
    int qM, qK, qbits;
};
template <bool DBG, int ABL = 0, bool XSF = false, bool QO = false>
__global__ __launch_bounds__(PB_WAVES * 64, 1) void fq_gemm_prefill_big_kernel(
    const int8_t *__restrict__ xq, const uint16_t *__restrict__ xs, const uint32_t *__restrict__ wpk, int M,
    int N, int K, uint16_t *__restrict__ d, int32_t *__restrict__ acc_dbg, const char *__restrict__ wu, PbQ qo) {
    extern __shared__ __attribute__((aligned(16))) char pb_smem[];
    char *sa = pb_smem, *sbu = pb_smem + 2 * PB_ASTAGE;
    const int G = K / FQ_GROUP, NT = (N + 15) / 16;
    const uint16_t *wsb = reinterpret_cast<const uint16_t *>(reinterpret_cast<const char *>(wpk) + (size_t)NT * G * FQ_BLOCK);
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wid >> 2, wn = wid & 3;  // 2 x 4 waves of 128 rows x 64 columns

    // Block order as in fq_gemm_prefill_kernel: XCD remap, then groups of 8 M-panels
    const int nbm = (M + PB_BM - 1) / PB_BM, nbn = (NT + PB_TILES - 1) / PB_TILES, nwg = nbm * nbn;
    const int bid = blockIdx.x, xcd = bid % 8, q = nwg / 8, rr = nwg % 8;
    const int lid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / 8;
    const int span = 8 * nbn, first = (lid / span) * 8;
    const int gsz = nbm - first < 8 ? nbm - first : 8;
    const int bm = first + (lid % span) % gsz, bn = (lid % span) / gsz;
    const int m0 = bm * PB_BM, t0 = bn * PB_TILES;

    // DMA: waves 4-7 issue all of it (wave 4 + v: A rows 64 v .. 64 v + 63 in 8 pieces, the unpacked
    // B of tiles 4 v .. 4 v + 3 in 8, the x-scales (one packed piece from wave 5, XSF; otherwise 64
    // rows per wave), wave 4 the w-scales); waves 0-3 issue none.  Waves w and w + 4 share a SIMD
    // and otherwise run in lockstep (MI355X_MICROARCH.md, two waves per SIMD): this way waves 0-3
    // reach their LDS reads and MFMAs while their partners are still issuing the next stage.
    const bool dmaw = wid >= 4;
    // Static priority for the DMA waves (measured: -2..-5 % against none or waves 0-3 prioritised):
    // their next stage leaves earlier, and they are the later-dispatched, arbitration-losing half.
    if (dmaw && !(ABL & 64)) __builtin_amdgcn_s_setprio(1);  // (ABL & 64: development, no priority)
    const int v4 = wid & 3;
    const int swz = ((lane & 7) ^ ((lane >> 3) & 7)) * 16;  // (row & 7 == (lane >> 3) & 7 for all 8 pieces)
    const int srow = 64 * v4 + lane;
    const int wt = t0 + (lane >> 1) < NT ? t0 + (lane >> 1) : NT - 1;
    // Buffer-addressed DMA (the host keeps every operand below 4 GiB for this kernel): each piece's
    // lane offset is fixed for the whole K loop and the group moves only the SGPR offset, so a stage
    // costs no per-piece 64-bit address VALU (those are the DMA waves' extra VALU, which the
    // dequant-bound loop cannot hide).  Rows past M read row M - 1 (computed, never stored).
    const __amdgpu_buffer_rsrc_t xqr = __builtin_amdgcn_make_buffer_rsrc((void *)xq, (short)0, (int)((uint32_t)M * (uint32_t)K), 0x00020000);
    const __amdgpu_buffer_rsrc_t xsr = __builtin_amdgcn_make_buffer_rsrc((void *)xs, (short)0, (int)((uint32_t)M * G * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t wsr = __builtin_amdgcn_make_buffer_rsrc((void *)wsb, (short)0, (int)((uint32_t)NT * G * 32), 0x00020000);
    const __amdgpu_buffer_rsrc_t wur = __builtin_amdgcn_make_buffer_rsrc((void *)wu, (short)0, (int)((uint32_t)NT * G * 2048), 0x00020000);
    uint32_t aoff[8], boff[4];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const int row = 64 * v4 + 8 * i + (lane >> 3);
        aoff[i] = (uint32_t)(m0 + row < M ? m0 + row : M - 1) * (uint32_t)K + swz;
    }
#pragma unroll
    for (int t = 0; t < 4; t++) {
        const int ut = t0 + 4 * v4 + t < NT ? t0 + 4 * v4 + t : NT - 1;
        boff[t] = (uint32_t)ut * G * 2048 + lane * 16;
    }
    const uint32_t xsoff = XSF ? (uint32_t)(m0 + 8 * lane) * 2 : (uint32_t)(m0 + srow < M ? m0 + srow : M - 1) * 2;
    const uint32_t wsoff = ((uint32_t)wt * G * 16 + 8 * (lane & 1)) * 2;
    auto stage = [&](int g, int slot) {
        if (ABL & 8) return;
        if (!dmaw) return;
        char *buf = sa + slot * PB_ASTAGE;
#pragma unroll
        for (int i = 0; i < 8; i++)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(xqr, LDS_PTR(buf + (64 * v4 + 8 * i) * FQ_GROUP), 16, aoff[i],
                                                     g * FQ_GROUP, 0, 0);
        if (XSF) {
            if (wid == 5 && lane < 32)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(xsr, LDS_PTR(buf + PB_XS_OFF), 16, xsoff, g * M * 2, 0, 0);
        } else {
            __builtin_amdgcn_raw_ptr_buffer_load_lds(xsr, LDS_PTR(buf + PB_XS_OFF + 64 * v4 * 4), 2, xsoff, g * M * 2, 0, 0);
        }
        if (wid == 4 && lane < 32)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(wsr, LDS_PTR(buf + PB_WS_OFF), 16, wsoff, g * 32, 0, 0);
        char *bdst = sbu + slot * PB_BSTAGE + 4 * v4 * 2048;
#pragma unroll
        for (int t = 0; t < 4; t++) {
            __builtin_amdgcn_raw_ptr_buffer_load_lds(wur, LDS_PTR(bdst + t * 2048), 16, boff[t], g * 2048, 0, 0);
            // (the immediate offset would move the LDS destination too: the +1024 goes in the SGPR offset)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(wur, LDS_PTR(bdst + t * 2048 + 1024), 16, boff[t], g * 2048 + 1024, 0, 0);
        }
    };

    const uint32_t la = lds_addr(sa), lbu = lds_addr(sbu);
    const int arow = wm * 128 + (lane & 15);
    const uint32_t a_off0 = arow * FQ_GROUP + xswz(arow, lane >> 4), a_off1 = arow * FQ_GROUP + xswz(arow, 4 + (lane >> 4));
    const uint32_t x_off = PB_XS_OFF + arow * (XSF ? 2 : 4);
    const uint32_t w_off = PB_WS_OFF + (wn * 64 + 4 * (lane >> 4)) * 2;
    const uint32_t b_off = wn * 4 * 2048 + lane * 16;

    float out[8][4][4];  // [mi][ni][r]: row 16 mi + (lane & 15), column 16 ni + 4 (lane >> 4) + r
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
        for (int j = 0; j < 4; j++)
#pragma unroll
            for (int r = 0; r < 4; r++) out[i][j][r] = 0.f;

    stage(0, 0);
    __builtin_amdgcn_s_waitcnt(vmcnt_only(0));
    unsigned long long pb_seg[4] = {0, 0, 0, 0}, pb_t = 0;
    (void)pb_seg;
    (void)pb_t;
    PB_STAMP(-1);
    for (int g = 0; g < G; g++) {
        PB_STAMP(3);
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        PB_STAMP(0);
        stage(g + 1 < G ? g + 1 : G - 1, (g + 1) & 1);  // (past the last group: a never-read copy)
        PB_STAMP(1);
        const uint32_t ab = la + (g & 1) * PB_ASTAGE, bb = lbu + (g & 1) * PB_BSTAGE + b_off;
        v4i b[4][2];
        v2u wv[4];
        v4i a[3][2];  // row blocks mi, mi + 1 and mi + 2 in flight
        uint32_t xv[4];  // their x-scales; slot mi % 4 lives until the dequant of (mi, 3), one block
                         // into row mi + 1 (after row mi + 3's reads were issued into slot (mi + 3) % 4)
        if (ABL & 4) {
#pragma unroll
            for (int i = 0; i < 4; i++) {
                b[i][0] = b[i][1] = v4i{(int)ab, (int)bb, g, i};
                wv[i] = v2u{ab + i, bb};
            }
#pragma unroll
            for (int i = 0; i < 3; i++) a[i][0] = a[i][1] = v4i{(int)bb, (int)ab, i, g};
#pragma unroll
            for (int i = 0; i < 4; i++) xv[i] = ab + 3 * i;
        } else {
#define FQ_PB_B(ni)                                                \
        b[ni][0] = ds_read_b128_at<(ni) * 2048>(bb);                \
        b[ni][1] = ds_read_b128_at<(ni) * 2048 + 1024>(bb);         \
        wv[ni] = ds_read_b64_at<(ni) * 32>(ab + w_off);
        FQ_PB_B(0) FQ_PB_B(1) FQ_PB_B(2) FQ_PB_B(3)
#undef FQ_PB_B
#define FQ_PB_A(mi)                                                                  \
        a[(mi) % 3][0] = ds_read_b128_at<(mi) * 16 * FQ_GROUP>(ab + a_off0);          \
        a[(mi) % 3][1] = ds_read_b128_at<(mi) * 16 * FQ_GROUP>(ab + a_off1);          \
        xv[(mi) % 4] = XSF ? ds_read_u16_at<(mi) * 32>(ab + x_off) : ds_read_b32_at<(mi) * 64>(ab + x_off);
        FQ_PB_A(0) FQ_PB_A(1)
        // in flight: B (8) + w-scales (4) + rows 0, 1 (3 each); each row block's reads are waited
        // for with the next-but-one block's (3) and the next one's (3) still outstanding
        asm volatile("s_waitcnt lgkmcnt(3)"
                     : "+v"(b[0][0]), "+v"(b[0][1]), "+v"(b[1][0]), "+v"(b[1][1]), "+v"(b[2][0]), "+v"(b[2][1]),
                       "+v"(b[3][0]), "+v"(b[3][1]), "+v"(wv[0]), "+v"(wv[1]), "+v"(wv[2]), "+v"(wv[3]),
                       "+v"(a[0][0]), "+v"(a[0][1]), "+v"(xv[0]));
            // (DBG: the debug output's register pressure makes the compiler spill, and a spill or copy of
            // a read still in flight would take the old register contents: no read stays in flight)
            if constexpr (DBG) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[1][0]), "+v"(a[1][1]), "+v"(xv[1]));
        }
        const uint32_t ab0 = ab + a_off0, ab1 = ab + a_off1, abx = ab + x_off;  // row block reads: immediate offsets
        // Blocks j = (mi, ni) in order, the dequant of block j - 1 after the MFMAs of block j: the
        // accumulators' MFMA latency is covered by the next block's MFMAs instead of s_nops.
        v4i accq[2];
        auto dequant = [&](const v4i acc, int mi, int ni) {
            // the fp16-rounded scale products w * xs (v_pk_mul_f16, xs broadcast by op_sel_hi)
            const uint32_t q01 = pk_mul_f16_lo(wv[ni][0], xv[mi % 4]), q23 = pk_mul_f16_lo(wv[ni][1], xv[mi % 4]);
            const __half2 p01 = __builtin_bit_cast(__half2, q01), p23 = __builtin_bit_cast(__half2, q23);
            float *o = out[mi][ni];
            o[0] = fmaf((float)acc[0], __low2float(p01), o[0]);
            o[1] = fmaf((float)acc[1], __high2float(p01), o[1]);
            o[2] = fmaf((float)acc[2], __low2float(p23), o[2]);
            o[3] = fmaf((float)acc[3], __high2float(p23), o[3]);
            if (DBG) {
                const int m = m0 + arow + mi * 16;
                const int n = (t0 + wn * 4 + ni) * 16 + 4 * (lane >> 4);
#pragma unroll
                for (int r = 0; r < 4; r++)
                    if (m < M && n + r < N) acc_dbg[((size_t)m * N + n + r) * G + g] = acc[r] >> 2;
            }
        };
#pragma unroll
        for (int j = 0; j <= 32; j++) {
            if (j < 32) {
                const int mi = j >> 2, ni = j & 3, c = mi % 3;
                if (ni == 0) {
                    if (mi > 0) {  // row block mi landed; mi + 1 may still be in flight
                        if (mi + 1 < 8)
                            asm volatile("s_waitcnt lgkmcnt(3)" : "+v"(a[c][0]), "+v"(a[c][1]), "+v"(xv[mi % 4]));
                        else
                            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[c][0]), "+v"(a[c][1]), "+v"(xv[mi % 4]));
                    }
                    // issue row block mi + 2 into the slot row block mi - 1 used (its MFMAs are issued)
                    if (mi + 2 < 8 && !(ABL & 4)) {
                        const int c2 = (mi + 2) % 3;
                        if constexpr (DBG) {  // (this loop is not unrolled in the debug variant: one
                                              // register-addressed read each, no switch to merge)
                            const uint32_t ro = (mi + 2) * 16 * FQ_GROUP;
                            a[c2][0] = ds_read_b128(ab0 + ro);
                            a[c2][1] = ds_read_b128(ab1 + ro);
                            xv[(mi + 2) % 4] = XSF ? ds_read_u16(abx + (mi + 2) * 32) : ds_read_b32(abx + (mi + 2) * 64);
                            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[c2][0]), "+v"(a[c2][1]), "+v"(xv[(mi + 2) % 4]));
                        } else {
                            a[c2][0] = ds_read_b128_k<16 * FQ_GROUP>(ab0, mi + 2);
                            a[c2][1] = ds_read_b128_k<16 * FQ_GROUP>(ab1, mi + 2);
                            xv[(mi + 2) % 4] = XSF ? ds_read_u16_k<32>(abx, mi + 2) : ds_read_b32_k<64>(abx, mi + 2);
                        }
                    }
                }
                v4i acc;
                if (ABL & 2) {  // (development: operands kept alive, no MFMA)
                    acc = b[ni][0] ^ a[c][1];
                    asm volatile("" : "+v"(acc) : "v"(b[ni][1]), "v"(a[c][0]));
                } else {
                    acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[ni][0], a[c][0], v4i{0, 0, 0, 0}, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[ni][1], a[c][1], acc, 0, 0, 0);
                }
                accq[j & 1] = acc;
            }
            // pinned order: this block's MFMAs, then the previous block's dequant (hipcc would hoist
            // the dequant above the MFMAs and stall on the accumulators; measured 2-5 % faster)
            __builtin_amdgcn_sched_barrier(0);
            if (j > 0) {
                const int pj = j - 1;
                if (ABL & 1)  // (development: accumulators kept alive, no dequant)
                    asm volatile("" ::"v"(accq[pj & 1]), "v"(xv[(pj >> 2) % 4]), "v"(wv[pj & 3]));
                else
                    dequant(accq[pj & 1], pj >> 2, pj & 3);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        PB_STAMP(2);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_waitcnt(vmcnt_only(0));  // stage g + 1 landed
    }
    PB_STAMP(3);
#ifdef FQ_DEV_ABLATION
    if ((ABL & 32) && lane == 0 && blockIdx.x < 256)
        for (int k = 0; k < 4; k++) g_pb_stamps[(blockIdx.x * PB_WAVES + wid) * 4 + k] = pb_seg[k];
#endif

    // Epilogue: a lane holds 4 consecutive columns of each 16 x 16 block; one v_permlane16_swap per
    // dword over the block pairs (0, 1), (2, 3) gives every lane 8 consecutive columns of one block
    // (even 16-lane rows: block np, columns 8 (h >> 1) ..; odd rows: block np + 1), so the output
    // leaves in 16-byte stores: 16 instead of 32 per lane.  The store tail of a one-WG-per-CU
    // kernel is issue-bound (cdna_hip_programming.md T21), and every CU hits it at once.
    const bool vec8 = (N & 7) == 0;
    const int hrow = lane >> 4;
#pragma unroll
    for (int mi = 0; mi < 8; mi++) {
        const int m = m0 + arow + mi * 16;
#pragma unroll
        for (int np = 0; np < 4; np += 2) {
            uint32_t pk[2][2];  // [block np + q][dword]: fp16 x 2, this lane's columns in order
#pragma unroll
            for (int q = 0; q < 2; q++) {
                const float *o = out[mi][np + q];
                pk[q][0] = (uint32_t)f2h(o[0] * 0.25f) | ((uint32_t)f2h(o[1] * 0.25f) << 16);
                pk[q][1] = (uint32_t)f2h(o[2] * 0.25f) | ((uint32_t)f2h(o[3] * 0.25f) << 16);
            }
#pragma unroll
            for (int w = 0; w < 2; w++) {
                const auto r = __builtin_amdgcn_permlane16_swap(pk[0][w], pk[1][w], false, false);
                pk[0][w] = r[0];
                pk[1][w] = r[1];
            }
            const int n = (t0 + wn * 4 + np + (hrow & 1)) * 16 + 8 * (hrow >> 1);
            if (ABL & 16) {
                asm volatile("" ::"v"(pk[0][0]), "v"(pk[0][1]), "v"(pk[1][0]), "v"(pk[1][1]));
            } else if (m < M) {
                uint16_t *dst = d + (size_t)m * N + n;
                if (vec8 && n + 7 < N) {
                    *reinterpret_cast<uint4 *>(dst) = make_uint4(pk[0][0], pk[0][1], pk[1][0], pk[1][1]);
                } else {
#pragma unroll
                    for (int r = 0; r < 8; r++)
                        if (n + r < N) dst[r] = (uint16_t)(pk[r >> 2][(r >> 1) & 1] >> (16 * (r & 1)));
                }
            }
        }
    }
    if constexpr (QO) {
        // The next linear's activation codes, as fq_quantize_act computes them from the fp16 output:
        // per (row, 128-column group) the absmax of the fp16 values -- this lane's 16 (4 blocks x 4
        // columns), the row's 4 lanes (lane ^ 16, ^ 32), then the partner wave's half through LDS
        // (the stage buffers are idle: every wave is past its last fragment read and DMA wait) --
        // then quant_scale / quant_code on each value.
        const int hi = (1 << (qo.qbits - 1)) - 1, lo = -(1 << (qo.qbits - 1));
        float *amx = reinterpret_cast<float *>(pb_smem);  // [wave][mi][16 rows]
        typedef _Float16 h2v __attribute__((ext_vector_type(2)));
        auto halves = [&](int mi, int ni, int k) {  // the output's fp16 values of columns 16 ni + 4 h + 2k, +1
            return __builtin_bit_cast(h2v, pack_h2(out[mi][ni][2 * k] * 0.25f, out[mi][ni][2 * k + 1] * 0.25f));
        };
        float mx[8];
#pragma unroll
        for (int mi = 0; mi < 8; mi++) {
            // packed |.| max (v_pk_max_f16: maxNum skips NaN, as fmaxf) over the lane's 16 values
            h2v a = __builtin_elementwise_abs(halves(mi, 0, 0));
#pragma unroll
            for (int j = 1; j < 8; j++) a = __builtin_elementwise_max(a, __builtin_elementwise_abs(halves(mi, j >> 1, j & 1)));
            float m = fmaxf(-1.0f, fmaxf((float)a.x, (float)a.y));  // (the reference's seed -1)
            m = fmaxf(m, __shfl_xor(m, 16));
            mx[mi] = fmaxf(m, __shfl_xor(m, 32));
        }
        __syncthreads();
        if (lane < 16) {
#pragma unroll
            for (int mi = 0; mi < 8; mi++) amx[(wid * 8 + mi) * 16 + lane] = mx[mi];
        }
        __syncthreads();
        const size_t lim = (size_t)qo.qM * qo.qK;
        const int gcol = t0 * 16 + (wn >> 1) * FQ_GROUP;  // the group's first column
#pragma unroll
        for (int mi = 0; mi < 8; mi++) {
            const int m = m0 + arow + mi * 16;
            const float gm = fmaxf(mx[mi], amx[((wid ^ 1) * 8 + mi) * 16 + (lane & 15)]);
            float rcb;
            const uint16_t sh = quant_scale(gm, qo.qbits, rcb);
            const size_t f0 = (size_t)m * N + gcol;  // the group's flat index
            if (m >= M || gcol >= N || f0 >= lim) continue;
            if (lane < 16 && (wn & 1) == 0)
                qo.qs[(f0 % qo.qK) / FQ_GROUP * (size_t)qo.qM + f0 / qo.qK] = sh;
            uint32_t w[4];  // block ni's 4 codes of this lane's columns 16 ni + 4 h ..
#pragma unroll
            for (int ni = 0; ni < 4; ni++) {
                int c[4];
#pragma unroll
                for (int k = 0; k < 2; k++) {  // the element step on the fp16 values (v_fma_mix_f32)
                    const h2v v = halves(mi, ni, k);
                    const uint32_t b = __builtin_bit_cast(uint32_t, v);
                    const float hs0 = __uint_as_float(((b << 16) & 0x80000000u) | 0x3f000000u);  // copysign(0.5, x)
                    const float hs1 = __uint_as_float((b & 0x80000000u) | 0x3f000000u);
                    c[2 * k] = med3_i32(cvt_i32_sat(fmaf((float)v.x, rcb, hs0)), lo, hi);
                    c[2 * k + 1] = med3_i32(cvt_i32_sat(fmaf((float)v.y, rcb, hs1)), lo, hi);
                }
                const uint32_t p01 = __builtin_amdgcn_perm((uint32_t)c[1], (uint32_t)c[0], 0x0c0c0400u);
                const uint32_t p23 = __builtin_amdgcn_perm((uint32_t)c[3], (uint32_t)c[2], 0x0c0c0400u);
                w[ni] = __builtin_amdgcn_perm(p23, p01, 0x05040100u);
            }
            // 4 x 4 transpose over (16-lane row h, block ni): permlane32 swaps, then permlane16 swaps
            // leave row h with block h's 16 consecutive codes -- one 16-byte store instead of four
#pragma unroll
            for (int k = 0; k < 2; k++) {
                const auto t = __builtin_amdgcn_permlane32_swap(w[k], w[k + 2], false, false);
                w[k] = t[0];
                w[k + 2] = t[1];
            }
#pragma unroll
            for (int k = 0; k < 4; k += 2) {
                const auto t = __builtin_amdgcn_permlane16_swap(w[k], w[k + 1], false, false);
                w[k] = t[0];
                w[k + 1] = t[1];
            }
            const int n = (t0 + wn * 4 + (lane >> 4)) * 16;
            *reinterpret_cast<uint4 *>(qo.qx + (size_t)m * N + n) = make_uint4(w[0], w[1], w[2], w[3]);
        }
    }
}

// =============================================================================================
// Host side: plan + launch
// =============================================================================================
struct DecodePlan {
    int MT, S, grid, IPW, RC, XS, SS, xwin;  // xwin: fused fp16 window (0 = not fused)
    int NCH;                                 // row chunks of MT rows (M > 32), else 1
    int NT;                                  // 16-column tiles
    int cost4;                               // modelled time, quarter-blocks per wave (see decode_plan)
    int pro;                                 // fused producer (DecodePro): 0, 1 (RMSNorm) or 2 (SiLU)
    bool fits;
};
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
    if (p.NCH > 1) M = p.MT;  // a WG holds one row chunk
    const int NW = decode_waves(p.MT);
    const int Gz = (K / FQ_GROUP + p.S - 1) / p.S;
    const int ngmax = (Gz + NW - 1) / NW;
    const int wm = decode_pro_windows(p.pro);
    return (size_t)NW * decode_wave_lds(p.MT, p.XS, p.SS, ngmax, ngmax * p.IPW, M, p.xwin, wm) +
           (size_t)p.RC * NW * M * 16 * 4 + ((4 * (size_t)p.IPW + 15) & ~(size_t)15) + 8 * NW + 16;
}

// Cost model, in quarter-blocks of one wave's stream (one 1.5 KiB block per wave at the
// whole-chip rate is ~0.7 us for the 7B shapes; tools/fuse_bench.py, tools/stamps.py):
//   stream   4 x items per WG x groups per wave
//   k-split  24 (the fix-up: slab drain, ticket and slab round trips, ~2.5 us; fitted to a forced-S
//            sweep of the TP shard shapes, tools/ksplit_sweep.sh) + the slab bytes each WG moves
//   fused    1 per (group, row) pair a wave quantizes (~0.17 us each, measured M = 1..16)
//   split    12 for the separate quantize launch (~2.2 us incl. its launch)
static const int kSplitQuantCost4 = 12;

// fused: only the fully staged variant (the quantizer writes straight into the staged regions);
// `fits` is false when that does not fit LDS and the caller must quantize separately.
static DecodePlan decode_plan(int M, int N, int K, bool fused, int pro = 0) {
    DecodePlan p;
    p.pro = fused ? pro : 0;
    p.MT = M <= 4 ? 4 : (M <= 8 ? 8 : (M <= 16 ? 16 : (M <= 32 ? 32 : 64)));
    const int NT = (N + 15) / 16, G = K / FQ_GROUP;
    p.NT = NT;
    p.NCH = 1;
    const int cus = device_cus();
    const int NW = decode_waves(p.MT);
    if (M > 32) {  // row chunks of 64: every chunk streams the whole weight image, no k-split
        p.NCH = (M + 63) / 64;
        p.S = 1;
        p.xwin = 0;
        const int items = NT * p.NCH;
        p.grid = (items < cus ? items : cus) / p.NCH * p.NCH;
        if (p.grid < p.NCH) p.grid = p.NCH;
        const int gw = p.grid / p.NCH;  // WGs per chunk
        p.IPW = (NT + gw - 1) / gw;
        p.cost4 = 4 * p.IPW * ((G + NW - 1) / NW) + kSplitQuantCost4;
        const int modes[3][2] = {{0, 0}, {1, 0}, {1, 1}};
        p.fits = false;
        for (int m = 0; m < 3 && !p.fits; m++) {
            p.XS = modes[m][0];
            p.SS = modes[m][1];
            for (p.RC = p.IPW; p.RC >= 1 && !p.fits; p.RC--) p.fits = decode_lds_bytes(p, M, N, K) <= kLdsMax;
            if (p.fits) p.RC++;
        }
        return p;
    }
    // k-split S minimises the modelled GEMM cost; S divides the grid so that z = blockIdx % S is
    // fixed per WG; ties keep the smaller S.  S (hence the summation order) is the same fused or
    // not, so fq_linear_w6ax gives the same bits whichever way it runs.
    long best = -1;
    p.S = 1;
    for (int S = 1; S <= G && S <= cus; S++) {
        const int items = NT * S;
        const int grid = items < cus ? items : cus;
        if (grid % S) continue;
        const long ipw = (items + grid - 1) / grid;
        const long ngw = ((G + S - 1) / S + NW - 1) / NW;
        long cost = 4 * ipw * ngw;
        if (S > 1) cost += 24 + 4 * ipw * M * 128 / (NW * FQ_BLOCK);
        if (best < 0 || cost < best) {
            best = cost;
            p.S = S;
        }
    }
#ifdef FQ_DEV_ABLATION
    if (const char *fs = getenv("FQ_DEV_S")) {  // development: force the k-split (tools/shape_sweep.py)
        const int S = atoi(fs), items = NT * S, grid = items < cus ? items : cus;
        if (S >= 1 && S <= G && grid % S == 0) p.S = S;
    }
#endif
    const int ngw = ((G + p.S - 1) / p.S + NW - 1) / NW;
    // (pro 3, bit planes: the unpack costs about half the quantizer per pair -- M = 2..16 A/B of the
    // forced-fuse variant against import + GEMM)
    p.cost4 = (int)best + (fused ? (pro == 3 ? (ngw * M + 1) / 2 : ngw * M) : kSplitQuantCost4);
    const int items = NT * p.S;
    p.grid = items < cus ? items : cus;
    p.IPW = (items + p.grid - 1) / p.grid;
    // staging: the most staged variant that fits LDS, then as many reduction slots as fit
    // (RC = IPW: one reduction after the whole stream)
    // (fused: the fully staged variant with the largest fp16 window that fits)
    const int modes[3][2] = {{0, 0}, {1, 0}, {1, 1}};
    const int nm = fused ? 1 : 3;
    // One item per workgroup at 5-16 rows: the activation rows ride in the ring slots (XS = 1) -- the
    // same bytes as the up-front staging, but no LDS-DMA burst before the first block (M = 16, 4096 x
    // 4096: 5.17 vs 5.74 us per launch; M = 8: 4.88 vs 5.29, 4096 x 11008 8.75 vs 9.67).  Not with more
    // items (the rows would be fetched once per item: M = 16, 12288 x 4096, 3 items 9.88 vs 9.56; 22016
    // 18.0 vs 15.4), nor for 16-row tiles over long K, whose slots carry 16 rows whatever M (M = 12, 4096 x
    // 11008: 9.7 vs 9.0).  profiles/r06_m16_xs_ab.txt, r06_m8_xs_ab.txt.  Same bits: XS moves the rows, not
    // the summation.
    int m0 = !fused && p.IPW == 1 && (p.MT == 8 || (p.MT == 16 && K <= 8192)) ? 1 : 0;
#ifdef FQ_DEV_ABLATION
    if (const char *e = getenv("FQ_DEV_XS"); e && !fused) m0 = atoi(e) == 1 ? 1 : 0;  // development: force either
#endif
    p.fits = false;
    for (int m = m0; m < nm && !p.fits; m++) {
        p.XS = modes[m][0];
        p.SS = modes[m][1];
        for (p.xwin = fused ? 32 : 0; !p.fits && p.xwin >= (fused ? 4 : 0); p.xwin = p.xwin ? p.xwin / 2 : -1) {
            for (p.RC = p.IPW; p.RC >= 1 && !p.fits; p.RC--) p.fits = decode_lds_bytes(p, M, N, K) <= kLdsMax;
            if (p.fits) {
                p.RC++;
                break;
            }
        }
    }
    return p;
}

static const size_t kTicketBytes = FQ_TICKET_BYTES;  // tickets for up to 65536 16-column tiles

// Large-M prefill unpacks the weight image once per call into int8 B operands in the workspace
// (0.75 B read + 1 B written per weight: ~1 % of the GEMM at M = 16384) so that the GEMM's B
// path is a plain LDS-DMA stream (fq_gemm_prefill_kernel<U8>).
constexpr int PF_U8_MIN_M = 2048;  // below, the unpack pass costs more than it saves (measured)
static size_t prefill_u8_bytes(int N, int K) { return (size_t)((N + 15) / 16) * (K / FQ_GROUP) * 2048; }

// One thread per (tile, group, block lane): its 8 bytes of each plane -> the two 16-byte int8
// B operands (k-steps 0 and 1) that unpack_w writes for that lane.
__global__ __launch_bounds__(256) void fq_unpack_w8_kernel(const char *__restrict__ img, long nblk,
                                                          char *__restrict__ wu) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= nblk * 64) return;
    const long blk = i >> 6;
    const int lane = (int)(i & 63);
    const char *src = img + blk * FQ_BLOCK + lane * 8;
    const uint2 p0 = *reinterpret_cast<const uint2 *>(src);
    const uint2 p1 = *reinterpret_cast<const uint2 *>(src + 512);
    const uint2 p2 = *reinterpret_cast<const uint2 *>(src + 1024);
    char *dst = wu + blk * 2048 + lane * 16;
    *reinterpret_cast<v4i *>(dst) = unpack_fq6(p0.x, p1.x, p2.x);
    *reinterpret_cast<v4i *>(dst + 1024) = unpack_fq6(p0.y, p1.y, p2.y);
}

// Split-K for the 128 x 128 prefill kernel when its tiles leave the chip under-filled (32 < M <
// PF_U8_MIN_M with few row x column tiles, e.g. M = 64, N = 4096: 32 WGs on 256 CUs).  Modelled
// time in us: rounds of two WGs per CU (its occupancy) x groups per split x PF_STEP_US per group
// step, plus for S > 1 the reduce launch and the fp32 slab bytes (written once, read once) at an
// effective 3 TB/s.  Constants fitted to a forced-S sweep on MI355X (tools/psplit_sweep.sh: M = 33
// .. 1024 on four LLaMA-2-7B shapes, 120 runs): the plan is within 2.1 us of the best S in every
// case (5.2 us summed over 24; the first guess, one WG per CU at 1.3 us and 5 TB/s, lost 36).
static const double PF_STEP_US = 1.4, PF_RED_US = 1.0, PF_SLAB_BPUS = 3e6;
static int prefill_split(int M, int N, int K) {
    if (M <= 32 || M >= PF_U8_MIN_M) return 1;
    const int G = K / FQ_GROUP, NT = (N + 15) / 16;
    const double nwg = (double)((M + PF_BM - 1) / PF_BM) * ((NT + PF_TILES - 1) / PF_TILES), slots = 2.0 * device_cus();
    int bs = 1;
    double best = 0;
    for (int S = 1; S <= 16 && S <= G; S *= 2) {  // the calibrated splits: 1, 2, 4, 8, 16
        const double t = ceil(nwg * S / slots) * ceil((double)G / S) * PF_STEP_US +
                         (S > 1 ? PF_RED_US + 2.0 * S * M * NT * 16 * sizeof(float) / PF_SLAB_BPUS : 0.0);
        if (S == 1 || t < best) {
            best = t;
            bs = S;
        }
    }
#ifdef FQ_DEV_ABLATION
    if (const char *fs = getenv("FQ_DEV_PS")) {  // development: force S (tools/psplit_sweep.sh)
        const int f = atoi(fs);
        if (f >= 1 && f <= G) bs = f;
    }
#endif
    return bs;
}
// 32 < M <= 128: the decode kernel with 64-row tiles (each weight block streamed once for all 64 rows;
// beyond 64 rows, row chunks of 64, each streaming the weights) or the 128 x 128 prefill kernel (split-K
// when its tiles are few).  Measured (tools/midm_sweep.py, profiles/r06_midm_sweep.txt, us per GEMM launch,
// decode / prefill): M = 33 .. 64 -- 4096 x 4096 8.9-9.3 / 13.6-15.7, 12288 x 4096 18.7-21.2 / 21.9-23.6,
// 4096 x 11008 16.7-18.6 / 21.7-23.2, but 22016 x 4096 33.6-40.4 / 32.6-34.1 (5.4 tiles per CU: the
// activation rows re-staged per tile); M = 96 .. 128 (two chunks) only 4096 x 4096 wins, 15.5 / 18.3-20.5.
// (The round-5 rule, row chunks of 32, won only on 4096 x 4096: 11.2-11.5 us.)
static bool midm_decode(int M, int N, int K) {
    if (M <= 32 || M > 128) return false;
    const int NT = (N + 15) / 16;
    bool use = M <= 64 ? NT <= 3 * device_cus() : (NT <= device_cus() && K <= 4096);
#ifdef FQ_DEV_ABLATION
    if (const char *e = getenv("FQ_DEV_MIDM")) use = atoi(e) != 0;  // development: force either
#endif
    return use;
}
static size_t prefill_slab_bytes(int M, int N, int S) { return (size_t)S * M * ((N + 15) / 16) * 16 * sizeof(float); }

extern "C" size_t fq_gemm_workspace_bytes(int M, int N, int K) {
    if (M <= 0 || N <= 0 || K <= 0 || K % FQ_GROUP) return 0;
    if (M >= PF_U8_MIN_M) return kTicketBytes + prefill_u8_bytes(N, K);  // tickets left untouched
    if (M > 32 && !midm_decode(M, N, K)) {
        const int S = prefill_split(M, N, K);
        return S > 1 ? kTicketBytes + prefill_slab_bytes(M, N, S) : 0;
    }
    const int S = decode_plan(M, N, K, false).S;  // the same for every staging variant and fused
    if (S == 1) return 0;
    const size_t Npad = (size_t)((N + 15) / 16) * 16;
    return kTicketBytes + (size_t)S * M * Npad * sizeof(float);
}

extern "C" fq_status fq_workspace_init(void *workspace, size_t bytes, fq_stream_t stream) {
    if (!bytes) return FQ_OK;
    if (!workspace) return FQ_ERR_NULL;
    if (hipMemsetAsync(workspace, 0, bytes < kTicketBytes ? bytes : kTicketBytes, (hipStream_t)stream) != hipSuccess)
        return FQ_ERR_HIP;
    return FQ_OK;
}

#ifdef FQ_DEV_ABLATION
extern "C" int fq_dev_stamps(unsigned long long *host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_fq_stamps), sizeof(unsigned long long) * n) == hipSuccess ? 0 : 1;
}
extern "C" int fq_dev_chain_stamps(unsigned long long *host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_fq_cstamps), (size_t)n * 8) == hipSuccess ? 0 : 1;
}
extern "C" int fq_dev_pb_stamps(unsigned long long *host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_pb_stamps), sizeof(unsigned long long) * n) == hipSuccess ? 0 : 1;
}
static int dev_ablation() {
    const char *e = getenv("FQ_DEV_ABLATION");
    return e ? atoi(e) : 0;
}
#endif

struct DecodeArgs {
    const int8_t *xq;
    const uint16_t *xs, *xh;
    int abits;
    const void *wpk;
    int M, N, K;
    uint16_t *d;
    int32_t *acc_dbg;
    void *workspace;
    const fq_gather *gat;  // peer-store gather (device memory), or nullptr
    DecodePro pro;         // fused producer arguments (PRO > 0)
};

template <int MT, int XS, int SS, bool FUSE, bool DBG, bool CH = false, int PRO = 0>
static fq_status launch_decode(const DecodePlan &p, const DecodeArgs &a, hipStream_t stream) {
    uint32_t *tickets = p.S > 1 ? (uint32_t *)a.workspace : nullptr;
    float *slabs = p.S > 1 ? (float *)((char *)a.workspace + kTicketBytes) : nullptr;
    const size_t lds = decode_lds_bytes(p, a.M, a.N, a.K);
    const dim3 grid(p.grid), block(decode_waves(MT) * 64);
    if ((size_t)p.NT * (a.K / FQ_GROUP) * FQ_BLOCK >= ((size_t)1 << 32)) return FQ_ERR_SHAPE;  // (buffer offsets)
    DecodePacked pk;
    const int gw = p.grid / p.NCH, items = p.NT * p.S;
    if (items / gw != p.IPW - (items % gw != 0) ||
        !decode_pack(a.N, a.K, a.abits, p.xwin, p.S, p.NCH, p.IPW, p.RC, a.M, items % gw, p.grid, &pk))
        return FQ_ERR_SHAPE;  // (never for the planner's decode plans; the packing's bounds)
    const void *xarg = FUSE ? (const void *)a.xh : (const void *)a.xq;
#ifdef FQ_DEV_ABLATION
    if (!DBG && !CH && (MT == 4 || MT == 16) && XS == 0 && SS == 0) {  // (the fused and the unfused kernel)
        const int abl = dev_ablation();
#define FQ_ABL(v)                                                                                           \
    if (abl == v) {                                                                                           \
        hipLaunchKernelGGL((fq_gemm_decode_kernel<MT, XS, SS, FUSE, v>), grid, block, lds, stream, xarg, a.xs, \
                           (const uint32_t *)a.wpk, a.d, (char *)a.workspace, pk.w0, pk.w1, pk.w2, pk.w3);      \
        FQ_LAUNCH_CHECK();                                                                                    \
        return FQ_OK;                                                                                         \
    }
        FQ_ABL(2) FQ_ABL(4) FQ_ABL(6) FQ_ABL(8) FQ_ABL(14) FQ_ABL(16) FQ_ABL(48) FQ_ABL(112)
        FQ_ABL(256) FQ_ABL(512) FQ_ABL(1024) FQ_ABL(768) FQ_ABL(1536) FQ_ABL(1792) FQ_ABL(2048) FQ_ABL(2052)
        FQ_ABL(4096)
#undef FQ_ABL
    }
#endif
    if constexpr (PRO == 4) {  // the fused LayerNorm (M = 1, S = 1)
        if (p.NCH != 1) return FQ_ERR_SHAPE;
        hipLaunchKernelGGL((fq_gemm_decode_ln_kernel<MT>), grid, block, lds, stream, a.xh, (const uint32_t *)a.wpk,
                           a.pro.in, a.pro.gamma, pk.w0, pk.w1, pk.w2, pk.w3, a.pro.beta, a.pro.bias, a.pro.eps, a.d,
                           (char *)a.workspace, a.pro.res_out);
        FQ_LAUNCH_CHECK();
        return FQ_OK;
    }
    if constexpr (PRO != 0 && PRO != 4) {  // the fused producers (FUSE, S as planned, no debug output, no gather)
        if (p.NCH != 1) return FQ_ERR_SHAPE;  // (the producer plans have one row chunk)
        hipLaunchKernelGGL((fq_gemm_decode_pro_kernel<MT, PRO>), grid, block, lds, stream, a.xh,
                           (const uint32_t *)a.wpk, a.pro.in, a.pro.gamma, pk.w0, pk.w1, pk.w2, pk.w3, a.pro.ldh,
                           a.pro.eps, a.d, (char *)a.workspace, a.pro.res_out);
        FQ_LAUNCH_CHECK();
        return FQ_OK;
    }
    if constexpr (!CH && !DBG) {
        if (a.gat) {  // the peer-store gather
            hipLaunchKernelGGL((fq_gemm_decode_gather_kernel<MT, XS, SS, FUSE>), grid, block, lds, stream, a.xq, a.xs,
                               a.xh, a.abits, (const uint32_t *)a.wpk, a.M, a.N, a.K, a.d, a.gat, slabs, tickets, p.S,
                               p.IPW, p.RC, p.xwin, p.NT * p.S / (p.grid / p.NCH), p.NT * p.S % (p.grid / p.NCH),
                               p.NCH, FUSE ? a.pro.wgat : nullptr, a.pro.werr);
            FQ_LAUNCH_CHECK();
            return FQ_OK;
        }
    }
    if (a.gat) return FQ_ERR_SHAPE;  // (no gather with the debug output or row chunks)
    if constexpr (DBG) {
        hipLaunchKernelGGL((fq_gemm_decode_dbg_kernel<MT, XS, SS, FUSE, CH>), grid, block, lds, stream, a.xq, a.xs,
                           a.xh, a.abits, (const uint32_t *)a.wpk, a.M, a.N, a.K, a.d, a.acc_dbg, slabs, tickets, p.S,
                           p.IPW, p.RC, p.xwin, p.NT * p.S / (p.grid / p.NCH), p.NT * p.S % (p.grid / p.NCH), p.NCH);
    } else {
        hipLaunchKernelGGL((fq_gemm_decode_kernel<MT, XS, SS, FUSE, 0, CH>), grid, block, lds, stream, xarg, a.xs,
                           (const uint32_t *)a.wpk, a.d, (char *)a.workspace, pk.w0, pk.w1, pk.w2, pk.w3);
    }
    FQ_LAUNCH_CHECK();
    return FQ_OK;
}

template <int MT, bool FUSE, bool DBG>
static fq_status dispatch_modes(const DecodePlan &p, const DecodeArgs &a, hipStream_t stream) {
    if constexpr (MT == 64) {  // 32 < M: never fused; row chunks of 64 beyond 64 rows
        if (FUSE) return FQ_ERR_SHAPE;
        if (p.NCH > 1) {
            if (p.XS == 0) return launch_decode<MT, 0, 0, false, DBG, true>(p, a, stream);
            if (p.SS == 0) return launch_decode<MT, 1, 0, false, DBG, true>(p, a, stream);
            return launch_decode<MT, 1, 1, false, DBG, true>(p, a, stream);
        }
    } else {
        if (FUSE) return launch_decode<MT, 0, 0, true, DBG>(p, a, stream);
    }
    if (p.XS == 0) return launch_decode<MT, 0, 0, false, DBG>(p, a, stream);
    if (p.SS == 0) return launch_decode<MT, 1, 0, false, DBG>(p, a, stream);
    return launch_decode<MT, 1, 1, false, DBG>(p, a, stream);
}

template <bool FUSE, bool DBG>
static fq_status dispatch_decode(const DecodePlan &p, const DecodeArgs &a, hipStream_t stream) {
    if (!p.fits) return FQ_ERR_SHAPE;  // the unfused plan always fits for K <= 2^20
    switch (p.MT) {
        case 4: return dispatch_modes<4, FUSE, DBG>(p, a, stream);
        case 8: return dispatch_modes<8, FUSE, DBG>(p, a, stream);
        case 16: return dispatch_modes<16, FUSE, DBG>(p, a, stream);
        case 32: return dispatch_modes<32, FUSE, DBG>(p, a, stream);
        default: return dispatch_modes<64, FUSE, DBG>(p, a, stream);
    }
}

// The fused one-launch linear is taken when it fits and its modelled cost (in-kernel quantizer
// redundant across WGs) does not exceed the split plan's (quantize launch + GEMM).
#ifndef FQ_FUSE_FORCE_M
#define FQ_FUSE_FORCE_M 0  // (development: fuse whenever it fits for M <= this, A/B tooling)
#endif
static bool decode_fuse(int M, int N, int K, DecodePlan *out, int pro = 0) {
    if (M > 32) return false;
    const DecodePlan f = decode_plan(M, N, K, true, pro);
    if (!f.fits || (M > FQ_FUSE_FORCE_M && f.cost4 > decode_plan(M, N, K, false).cost4)) return false;
    if (out) *out = f;
    return true;
}

extern "C" size_t fq_linear_act_scratch_bytes(int M, int N, int K) {
    if (M <= 0 || N <= 0 || K <= 0 || K % FQ_GROUP) return 0;
    if (decode_fuse(M, N, K, nullptr)) return 0;
    return (size_t)M * K + (size_t)M * (K / FQ_GROUP) * 2;
}

// One-launch decode linear (quantize + GEMM) when the staged plan fits; FQ_ERR_SHAPE otherwise.
fq_status fq_decode_linear_fused(const uint16_t *x, int M, int N, int K, int abits, const void *w_packed,
                                 uint16_t *d, int32_t *acc_dbg, void *workspace, size_t workspace_bytes,
                                 hipStream_t s, bool *launched, const fq_gather *gat, const fq_gather *wgat,
                                 uint32_t *werr) {
    *launched = false;
    DecodePlan p;
    if (!decode_fuse(M, N, K, &p)) return FQ_OK;
    const size_t need = fq_gemm_workspace_bytes(M, N, K);
    if (need && (!workspace || workspace_bytes < need)) return FQ_ERR_WORKSPACE;
    DecodeArgs a = {nullptr, nullptr, x, abits, w_packed, M, N, K, d, acc_dbg, workspace, gat, DecodePro{}};
    if (wgat && (!gat || acc_dbg)) return FQ_ERR_SHAPE;  // (the folded wait exists in the gather kernel only)
    a.pro.wgat = wgat;
    a.pro.werr = werr;
    *launched = true;
    return acc_dbg ? dispatch_decode<true, true>(p, a, s) : dispatch_decode<true, false>(p, a, s);
}

// ---- decode chain: the links that can run in one persistent launch are those whose fused plan
// is one 4-row tile set over the whole chip with no k-split (every LLaMA / OPT decode shape at
// M <= 4 with N >= 16 x CUs), outputs in 16-column multiples, 16-byte aligned activations; a
// producer link as its one-launch entry point requires (RMSNorm: M = 1, K = 4096; SiLU: any M <= 4).
static bool ranges_overlap(const void *a, size_t na, const void *b, size_t nb) {
    return a && b && (uintptr_t)a < (uintptr_t)b + nb && (uintptr_t)b < (uintptr_t)a + na;
}
static bool in_range(const void *a, size_t na, const void *b, size_t nb) {  // [a, a+na) inside [b, b+nb)
    return (uintptr_t)a >= (uintptr_t)b && (uintptr_t)a + na <= (uintptr_t)b + nb;
}
static size_t chain_xspan(int M, const fq_chain_link &L) {  // bytes of x (and in): SiLU rows have stride ldh
    const size_t ld = L.pro == 2 ? (size_t)L.ldh : (size_t)L.K;
    return ((size_t)(M - 1) * ld + L.K) * 2;
}
static bool chain_plan(int M, const fq_chain_link &L, DecodePlan *p) {
    if (M > 4 || L.N % 16 || ((uintptr_t)L.x & 15) || ((uintptr_t)L.d & 3) || L.pro < 0 || L.pro > 2) return false;
    if (L.pro == 1) {  // as fq_rmsnorm_linear_w6ax's one-launch form
        const size_t rb = (size_t)L.K * 2;
        if (M != 1 || L.K != 4 * FQ_GROUP * decode_waves(4) || !L.gamma || (L.in && !L.res_out) ||
            (((uintptr_t)L.gamma | (uintptr_t)L.in | (uintptr_t)L.res_out) & 15))
            return false;
        if (L.in && (ranges_overlap(L.res_out, rb, L.x, rb) || ranges_overlap(L.res_out, rb, L.in, rb) ||
                     ranges_overlap(L.res_out, rb, L.gamma, rb)))
            return false;
    }
    if (L.pro == 2 && (!L.in || L.ldh < L.K || L.ldh % 8 || ((uintptr_t)L.in & 15))) return false;
    *p = decode_plan(M, L.N, L.K, true);
    return p->fits && p->MT == 4 && p->S == 1 && p->NCH == 1 && p->grid == device_cus() &&
           decode_lds_bytes(*p, M, L.N, L.K) + 2048 <= kLdsMax &&  // (+ the chain kernel's static LDS)
           (size_t)p->NT * (L.K / FQ_GROUP) * FQ_BLOCK < ((size_t)1 << 32);
}
static size_t chain_handoff_bytes(int M, int N) { return ((size_t)M * N * 4 + 255) & ~(size_t)255; }

extern "C" size_t fq_chain_workspace_bytes(const fq_chain_link *links, int n, int M) {
    size_t b = FQ_CHAIN_SYNC_BYTES;
    for (int l = 0; links && l < n; l++) {
        if (l + 1 < n) b += chain_handoff_bytes(M, links[l].N);
        if (links[l].pro == 1 && links[l].in) b += chain_handoff_bytes(M, links[l].K);  // its residual output
    }
    return b;
}

extern "C" fq_status fq_chain_workspace_init(void *chain_ws, size_t bytes, fq_stream_t stream) {
    if (!bytes) return FQ_OK;
    if (!chain_ws) return FQ_ERR_NULL;
    return hipMemsetAsync(chain_ws, 0, bytes, (hipStream_t)stream) == hipSuccess ? FQ_OK : FQ_ERR_HIP;
}

// ---- host-visible chain status: chain workspace -> the caller's pinned host word (host side), and the
// word's device address in the workspace's sync area (device side, read by chain_fail)
static std::mutex g_chain_mu;
static std::unordered_map<const void *, volatile uint32_t *> g_chain_status;

__global__ void fq_chain_bind_kernel(uint32_t *__restrict__ sync, uint64_t host_dev) {
    if (threadIdx.x == 0)
        __hip_atomic_store(reinterpret_cast<uint64_t *>(sync + 32 * FQ_CHAIN_HOST), host_dev, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

static fq_status chain_bind(void *chain_ws, uint32_t *host_status, hipStream_t s) {
    void *dev = nullptr;
    if (hipHostGetDevicePointer(&dev, host_status, 0) != hipSuccess || !dev) {
        (void)hipGetLastError();  // (not device-mapped memory: clear the sticky error)
        return FQ_ERR_NULL;
    }
    *(volatile uint32_t *)host_status = 0u;  // (a word that starts nonzero would read as a timeout)
    hipLaunchKernelGGL(fq_chain_bind_kernel, dim3(1), dim3(64), 0, s, (uint32_t *)chain_ws, (uint64_t)(uintptr_t)dev);
    FQ_LAUNCH_CHECK();
    std::lock_guard<std::mutex> lk(g_chain_mu);
    g_chain_status[chain_ws] = host_status;
    return FQ_OK;
}

extern "C" fq_status fq_chain_bind_status(void *chain_ws, size_t chain_ws_bytes, uint32_t *host_status,
                                          fq_stream_t stream) {
    if (!chain_ws || !host_status) return FQ_ERR_NULL;
    // (the bind kernel writes the word's address at byte 32 * 4 * FQ_CHAIN_HOST of the sync area)
    if (((uintptr_t)chain_ws & 255) || chain_ws_bytes < FQ_CHAIN_SYNC_BYTES) return FQ_ERR_WORKSPACE;
    return chain_bind(chain_ws, host_status, (hipStream_t)stream);
}

extern "C" fq_status fq_chain_status(const void *chain_ws) {
    std::lock_guard<std::mutex> lk(g_chain_mu);
    const auto it = g_chain_status.find(chain_ws);
    return it != g_chain_status.end() && *it->second != 0u ? FQ_ERR_TIMEOUT : FQ_OK;
}

extern "C" fq_status fq_chain_reset(void *chain_ws, size_t bytes, fq_stream_t stream) {
    if (!chain_ws) return FQ_ERR_NULL;
    const fq_status st = fq_chain_workspace_init(chain_ws, bytes, stream);
    if (st != FQ_OK) return st;
    uint32_t *h = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_chain_mu);
        const auto it = g_chain_status.find(chain_ws);
        if (it != g_chain_status.end()) h = const_cast<uint32_t *>(it->second);
    }
    if (!h) return FQ_OK;
    *(volatile uint32_t *)h = 0u;  // (no launch on chain_ws is in flight: the caller synchronised)
    return chain_bind(chain_ws, h, (hipStream_t)stream);
}

// Every workgroup of a chain launch waits on others of the same launch: the kernel must hold one
// workgroup per CU at the run's LDS size (the grid is the CU count).  Cached per (kernel, LDS bytes).
template <bool CHP>
static bool chain_coresident(size_t lds) {
    static std::mutex mu;
    static std::unordered_map<size_t, bool> cache;
    std::lock_guard<std::mutex> lk(mu);
    const auto it = cache.find(lds);
    if (it != cache.end()) return it->second;
    int nb = 0;
    const bool ok = hipOccupancyMaxActiveBlocksPerMultiprocessor(
                        &nb, reinterpret_cast<const void *>(fq_gemm_decode_chain_kernel<4, CHP>),
                        decode_waves(4) * 64, lds) == hipSuccess && nb >= 1;
    if (!ok) (void)hipGetLastError();
    cache[lds] = ok;
    return ok;
}

// one link as its own entry point (the chain's fallback; the same bits)
static fq_status chain_link_alone(const fq_chain_link &L, int M, int8_t *xq_buf, uint16_t *xs_buf, void *workspace,
                                  size_t workspace_bytes, fq_stream_t stream) {
    if (L.pro == 1)
        return fq_rmsnorm_linear_w6ax(L.in, L.x, L.res_out, L.gamma, L.eps, M, L.N, L.K, L.abits, L.w_packed, L.d,
                                      xq_buf, xs_buf, workspace, workspace_bytes, stream);
    if (L.pro == 2)
        return fq_silu_linear_w6ax(L.x, L.in, L.ldh, M, L.N, L.K, L.abits, L.w_packed, L.d, xq_buf, xs_buf, workspace,
                                   workspace_bytes, stream);
    return fq_linear_w6ax(L.x, M, L.N, L.K, L.abits, L.w_packed, L.d, xq_buf, xs_buf, workspace, workspace_bytes,
                          stream);
}

extern "C" fq_status fq_linear_chain_w6ax(const fq_chain_link *links, int n, int M, void *chain_ws,
                                          size_t chain_ws_bytes, int8_t *xq_buf, uint16_t *xs_buf, void *workspace,
                                          size_t workspace_bytes, fq_stream_t stream) {
    if (!links || n <= 0) return FQ_ERR_NULL;
    if (M <= 0 || M > 32) return FQ_ERR_SHAPE;
    for (int l = 0; l < n; l++) {
        const fq_chain_link &L = links[l];
        if (!L.x || !L.w_packed || !L.d) return FQ_ERR_NULL;
        if (L.N <= 0 || L.K <= 0 || L.K % FQ_GROUP) return FQ_ERR_SHAPE;
        if (L.abits != 6 && L.abits != 8) return FQ_ERR_BITS;
        if (L.pro < 0 || L.pro > 2) return FQ_ERR_SHAPE;
    }
    const hipStream_t s = (hipStream_t)stream;
    if (chain_ws && fq_chain_status(chain_ws) != FQ_OK) return FQ_ERR_TIMEOUT;  // (until fq_chain_reset)
    const bool ws_ok = chain_ws && chain_ws_bytes >= FQ_CHAIN_SYNC_BYTES && ((uintptr_t)chain_ws & 255) == 0;
    char *hand = (char *)chain_ws + FQ_CHAIN_SYNC_BYTES;  // the hand-off granules of a run
    const size_t hand_bytes = ws_ok ? (chain_ws_bytes - FQ_CHAIN_SYNC_BYTES) / 16 * 16 : 0;
    if (hand_bytes >= ((size_t)1 << 32)) return FQ_ERR_WORKSPACE;
    int l = 0;
    while (l < n) {
        // The longest run from l (at most FQ_CHAIN_MAX links, the first a plain linear) in which every
        // link is chainable, no output (d, res_out) overlaps another output or any input (x, in, gamma)
        // of the run, except that a link's x / in may lie inside the previous link's d (read from its
        // hand-off granules) and an RMSNorm link's residual x may be an earlier RMSNorm link's res_out
        // (read from that link's residual granules); every other input is ready before the launch.
        DecodePlan plans[FQ_CHAIN_MAX];
        int xsrc[FQ_CHAIN_MAX], insrc[FQ_CHAIN_MAX];  // -1 ready; j >= 0: link j's d (x, in) or res_out (x, RMSNorm)
        bool needd[FQ_CHAIN_MAX] = {}, needr[FQ_CHAIN_MAX] = {};
        size_t used = 0;
        int r = 0;
        while (ws_ok && l + r < n && r < FQ_CHAIN_MAX && (r > 0 || links[l].pro == 0) &&
               chain_plan(M, links[l + r], &plans[r])) {
            const fq_chain_link &L = links[l + r];
            const size_t xb = chain_xspan(M, L), db = (size_t)M * L.N * 2, gb = (size_t)L.K * 2;
            const size_t rb = (L.pro == 1 && L.in) ? (size_t)M * L.K * 2 : 0;  // res_out
            int xs = -1, is = -1;
            size_t extra = 0;
            if (r > 0) {
                const fq_chain_link &P = links[l + r - 1];
                const size_t pb = (size_t)M * P.N * 2;
                if (in_range(L.x, xb, P.d, pb) && (((uintptr_t)L.x - (uintptr_t)P.d) & 3) == 0) xs = r - 1;
                if (L.pro != 0 && L.in && in_range(L.in, xb, P.d, pb) && (((uintptr_t)L.in - (uintptr_t)P.d) & 3) == 0)
                    is = r - 1;
                if ((xs >= 0 || is >= 0) && !needd[r - 1]) extra += chain_handoff_bytes(M, P.N);
            }
            if (xs < 0 && L.pro == 1)
                for (int j = 0; j < r; j++)
                    if (links[l + j].pro == 1 && links[l + j].in && links[l + j].res_out == L.x) {
                        xs = FQ_CHAIN_MAX + j;  // (an earlier link's residual output)
                        if (!needr[j]) extra += chain_handoff_bytes(M, links[l + j].K);
                    }
            bool ok = used + extra <= hand_bytes;
            for (int j = 0; ok && j <= r; j++) {
                const fq_chain_link &Q = links[l + j];
                const size_t qd = (size_t)M * Q.N * 2, qr = (Q.pro == 1 && Q.in) ? (size_t)M * Q.K * 2 : 0;
                const size_t qx = chain_xspan(M, Q);
                // this link's outputs against every output and input of the run so far (itself included:
                // its own res_out was checked by chain_plan)
                if (j < r && (ranges_overlap(L.d, db, Q.d, qd) || ranges_overlap(L.d, db, Q.res_out, qr) ||
                              ranges_overlap(L.res_out, rb, Q.d, qd) || ranges_overlap(L.res_out, rb, Q.res_out, qr)))
                    ok = false;
                if (ranges_overlap(L.d, db, Q.x, qx) || ranges_overlap(L.d, db, Q.in, Q.pro ? qx : 0) ||
                    ranges_overlap(L.d, db, Q.gamma, Q.pro == 1 ? (size_t)Q.K * 2 : 0))
                    ok = false;
                if (j < r && (ranges_overlap(L.res_out, rb, Q.x, qx) || ranges_overlap(L.res_out, rb, Q.in, Q.pro ? qx : 0) ||
                              ranges_overlap(L.res_out, rb, Q.gamma, Q.pro == 1 ? (size_t)Q.K * 2 : 0)))
                    ok = false;
                // this link's ready inputs against the run's outputs (its own included)
                const bool xfrom = (xs == r - 1 && j == r - 1) || (xs == FQ_CHAIN_MAX + j);
                if (!xfrom && (ranges_overlap(L.x, xb, Q.d, qd) || ranges_overlap(L.x, xb, Q.res_out, qr))) ok = false;
                if (L.pro != 0 && !(is == r - 1 && j == r - 1) &&
                    (ranges_overlap(L.in, xb, Q.d, qd) || ranges_overlap(L.in, xb, Q.res_out, qr)))
                    ok = false;
                if (L.pro == 1 && (ranges_overlap(L.gamma, gb, Q.d, qd) || ranges_overlap(L.gamma, gb, Q.res_out, qr)))
                    ok = false;
            }
            if (!ok) break;
            xsrc[r] = xs;
            insrc[r] = is;
            if (xs >= 0 && xs < FQ_CHAIN_MAX) needd[xs] = true;
            if (is >= 0) needd[is] = true;
            if (xs >= FQ_CHAIN_MAX) needr[xs - FQ_CHAIN_MAX] = true;
            used += extra;
            r++;
        }
        if (r < 2) {  // a run of one: the link's own entry point
            const fq_status st = chain_link_alone(links[l], M, xq_buf, xs_buf, workspace, workspace_bytes, stream);
            if (st != FQ_OK) return st;
            l++;
            continue;
        }
        // hand-off regions: link i's output granules (when the next link reads its d), its residual
        // granules (when a later RMSNorm link reads its res_out)
        uint64_t *hd[FQ_CHAIN_MAX] = {}, *hr[FQ_CHAIN_MAX] = {};
        size_t off = 0;
        for (int i = 0; i < r; i++) {
            if (needd[i]) {
                hd[i] = reinterpret_cast<uint64_t *>(hand + off);
                off += chain_handoff_bytes(M, links[l + i].N);
            }
            if (needr[i]) {
                hr[i] = reinterpret_cast<uint64_t *>(hand + off);
                off += chain_handoff_bytes(M, links[l + i].K);
            }
        }
        ChainLinkP cl[FQ_CHAIN_MAX];
        size_t lds = 0;
        for (int i = 0; i < r; i++) {
            const fq_chain_link &L = links[l + i];
            const DecodePlan &p = plans[i];
            DecodePacked pk;
            const int items = p.NT;
            if (items / p.grid != p.IPW - (items % p.grid != 0) ||
                !decode_pack(L.N, L.K, L.abits, p.xwin, 1, 1, p.IPW, p.RC, M, items % p.grid, p.grid, &pk))
                return FQ_ERR_SHAPE;
            const uint64_t *hx = nullptr, *hin = nullptr;
            if (xsrc[i] >= FQ_CHAIN_MAX) {
                hx = hr[xsrc[i] - FQ_CHAIN_MAX];
            } else if (xsrc[i] >= 0) {
                hx = hd[i - 1] + ((uintptr_t)L.x - (uintptr_t)links[l + i - 1].d) / 4;
            }
            if (insrc[i] >= 0) hin = hd[i - 1] + ((uintptr_t)L.in - (uintptr_t)links[l + i - 1].d) / 4;
            cl[i] = ChainLinkP{L.x, (const uint32_t *)L.w_packed, L.d, hx, hd[i], L.pro ? L.in : nullptr, hin,
                              L.pro == 1 ? L.gamma : nullptr, (L.pro == 1 && L.in) ? L.res_out : nullptr, hr[i],
                              pk.w0, pk.w1, pk.w2, pk.w3, L.eps,
                              (uint32_t)(L.pro == 2 ? L.ldh : 0) | ((uint32_t)L.pro << 24)};
            const size_t b = decode_lds_bytes(p, M, L.N, L.K);
            lds = b > lds ? b : lds;
        }
        bool prod = false;
        for (int i = 0; i < r; i++) prod = prod || links[l + i].pro != 0;
        if (!(prod ? chain_coresident<true>(lds) : chain_coresident<false>(lds))) {
            for (int i = 0; i < r; i++) {  // not one workgroup per CU: the links as their entry points
                const fq_status st = chain_link_alone(links[l + i], M, xq_buf, xs_buf, workspace, workspace_bytes, stream);
                if (st != FQ_OK) return st;
            }
            l += r;
            continue;
        }
        if (prod) {
            ChainTailP t{};
            for (int i = 1; i < r; i++) t.l[i - 1] = cl[i];
            t.n = r;
            t.hand = (uint4 *)hand;
            t.hand_bytes = (uint32_t)hand_bytes;
            hipLaunchKernelGGL((fq_gemm_decode_chain_kernel<4, true>), dim3(plans[0].grid), dim3(decode_waves(4) * 64),
                               lds, s, (uint32_t *)chain_ws, cl[0].x, cl[0].w, cl[0].d, cl[0].w0, cl[0].w1, cl[0].w2,
                               cl[0].w3, cl[0].hd, t);
        } else {
            ChainTailPlain t{};
            for (int i = 1; i < r; i++) {
                const ChainLinkP &c = cl[i];
                t.l[i - 1] = ChainLinkPlain{c.x, c.w, c.d, c.hx, c.hd, c.w0, c.w1, c.w2, c.w3};
            }
            t.n = r;
            t.hand = (uint4 *)hand;
            t.hand_bytes = (uint32_t)hand_bytes;
            hipLaunchKernelGGL((fq_gemm_decode_chain_kernel<4, false>), dim3(plans[0].grid), dim3(decode_waves(4) * 64),
                               lds, s, (uint32_t *)chain_ws, cl[0].x, cl[0].w, cl[0].d, cl[0].w0, cl[0].w1, cl[0].w2,
                               cl[0].w3, cl[0].hd, t);
        }
        FQ_LAUNCH_CHECK();
        l += r;
    }
    return FQ_OK;
}

extern "C" size_t fq_chain_error_offset(void) { return 4 * 32 * FQ_CHAIN_ERR; }

// A producer fused into the one-launch decode linear (DecodePro): pro = 1, residual add + RMSNorm
// (xh = the residual; M = 1, K = 4 * 128 * waves, no k-split), pro = 2, SiLU(xh) * in (M <= 32).
// Launches only when the fused plan is taken; *launched tells the caller to run the producer
// kernel and the GEMM instead.
static bool pro_fuse(int pro, int M, int N, int K, DecodePlan *p) {
    if (!decode_fuse(M, N, K, p, pro)) return false;
    return (pro != 1 && pro != 4) || (M == 1 && p->MT == 4 && p->S == 1 && K == 4 * FQ_GROUP * decode_waves(4));
}
extern "C" size_t fq_layernorm_linear_scratch_bytes(int M, int N, int K) {
    DecodePlan p;
    if (M <= 0 || N <= 0 || K <= 0 || K % FQ_GROUP || pro_fuse(4, M, N, K, &p)) return 0;
    return (size_t)M * K + (size_t)M * (K / FQ_GROUP) * 2;
}
extern "C" size_t fq_rmsnorm_linear_scratch_bytes(int M, int N, int K) {
    DecodePlan p;
    if (M <= 0 || N <= 0 || K <= 0 || K % FQ_GROUP || pro_fuse(1, M, N, K, &p)) return 0;
    return (size_t)M * K + (size_t)M * (K / FQ_GROUP) * 2;
}
extern "C" size_t fq_silu_linear_scratch_bytes(int M, int N, int K) {
    DecodePlan p;
    if (M <= 0 || N <= 0 || K <= 0 || K % FQ_GROUP || pro_fuse(2, M, N, K, &p)) return 0;
    return (size_t)M * K + (size_t)M * (K / FQ_GROUP) * 2;
}

fq_status fq_decode_linear_pro(int pro, const uint16_t *xh, const DecodePro &prod, int M, int N, int K, int abits,
                               const void *w_packed, uint16_t *d, void *workspace, size_t workspace_bytes,
                               hipStream_t s, bool *launched) {
    *launched = false;
    if (pro != 1 && pro != 2 && pro != 4) return FQ_ERR_SHAPE;
    DecodePlan p;
    if (!pro_fuse(pro, M, N, K, &p)) return FQ_OK;
    const size_t need = fq_gemm_workspace_bytes(M, N, K);
    if (need && (!workspace || workspace_bytes < need)) return FQ_ERR_WORKSPACE;
    DecodeArgs a = {nullptr, nullptr, xh, abits, w_packed, M, N, K, d, nullptr, workspace, nullptr, prod};
    *launched = true;
    if (pro == 1) return launch_decode<4, 0, 0, true, false, false, 1>(p, a, s);
    if (pro == 4) return launch_decode<4, 0, 0, true, false, false, 4>(p, a, s);
    switch (p.MT) {
        case 4: return launch_decode<4, 0, 0, true, false, false, 2>(p, a, s);
        case 8: return launch_decode<8, 0, 0, true, false, false, 2>(p, a, s);
        case 16: return launch_decode<16, 0, 0, true, false, false, 2>(p, a, s);
        default: return launch_decode<32, 0, 0, true, false, false, 2>(p, a, s);
    }
}

// The reference's bit-plane activations (FQBMMAExecFn_t's X + duplicated X_SCALE, the wrapper's
// gemm(const int* A ...)) unpacked inside the decode GEMM's prologue (PRO 3): one launch wherever
// fq_linear_w6ax would fuse its quantizer; otherwise fq_import_ref_x into the caller's buffers,
// then fq_gemm_w6ax.  Bit-identical either way (the same plan, S and reduction order).
#ifndef FQ_PLANES_FORCE_FUSE
#define FQ_PLANES_FORCE_FUSE 0  // (development: 1 = unpack in the prologue whenever it fits, A/B tooling)
#endif
static bool planes_fuse(int M, int N, int K, DecodePlan *p) {
    if (!(M <= 8 || M % 8 == 0)) return false;
    if (FQ_PLANES_FORCE_FUSE) {
        if (M > 32) return false;
        *p = decode_plan(M, N, K, true, 3);
        return p->fits;
    }
    return decode_fuse(M, N, K, p, 3);
}
extern "C" size_t fq_planes_act_scratch_bytes(int M, int N, int K) {
    DecodePlan p;
    if (M <= 0 || N <= 0 || K <= 0 || K % FQ_GROUP || planes_fuse(M, N, K, &p)) return 0;
    return (size_t)M * K + (size_t)M * (K / FQ_GROUP) * 2;
}
extern "C" fq_status fq_gemm_w6ax_planes(const int32_t *x_bitplanes, const uint16_t *x_scale_dup, const void *w_packed,
                                         int M, int N, int K, int abits, uint16_t *d, int8_t *xq_buf, uint16_t *xs_buf,
                                         void *workspace, size_t workspace_bytes, fq_stream_t stream) {
    if (!x_bitplanes || !x_scale_dup || !w_packed || !d) return FQ_ERR_NULL;
    if (M <= 0 || N <= 0 || K <= 0 || K % FQ_GROUP || (M > 8 && M % 8)) return FQ_ERR_SHAPE;
    if ((size_t)((N + 15) / 16) > kTicketBytes / 4) return FQ_ERR_SHAPE;
    if (abits != 6 && abits != 8) return FQ_ERR_BITS;
    DecodePlan p;
    if (planes_fuse(M, N, K, &p)) {
        const size_t need = fq_gemm_workspace_bytes(M, N, K);
        if (need && (!workspace || workspace_bytes < need)) return FQ_ERR_WORKSPACE;
        const DecodePro pro = {x_scale_dup, nullptr, nullptr, 0.f, K};
        DecodeArgs a = {nullptr, nullptr, reinterpret_cast<const uint16_t *>(x_bitplanes), abits, w_packed, M, N, K,
                        d, nullptr, workspace, nullptr, pro};
        hipStream_t s = (hipStream_t)stream;
        switch (p.MT) {
            case 4: return launch_decode<4, 0, 0, true, false, false, 3>(p, a, s);
            case 8: return launch_decode<8, 0, 0, true, false, false, 3>(p, a, s);
            case 16: return launch_decode<16, 0, 0, true, false, false, 3>(p, a, s);
            default: return launch_decode<32, 0, 0, true, false, false, 3>(p, a, s);
        }
    }
    if (!xq_buf || !xs_buf) return FQ_ERR_NULL;
    const fq_status st = fq_import_ref_x(x_bitplanes, x_scale_dup, M, K, abits, xq_buf, xs_buf, stream);
    if (st != FQ_OK) return st;
    return fq_gemm_w6ax(xq_buf, xs_buf, w_packed, M, N, K, abits, d, nullptr, workspace, workspace_bytes, stream);
}

fq_status fq_gemm_w6ax_impl(const int8_t *xq, const uint16_t *xs, const void *w_packed, int M, int N, int K,
                            int abits, uint16_t *d, int32_t *acc_dbg, void *workspace, size_t workspace_bytes,
                            fq_stream_t stream, const fq_gather *gat);
extern "C" fq_status fq_gemm_w6ax(const int8_t *xq, const uint16_t *xs, const void *w_packed, int M, int N,
                                  int K, int abits, uint16_t *d, int32_t *acc_dbg, void *workspace,
                                  size_t workspace_bytes, fq_stream_t stream) {
    return fq_gemm_w6ax_impl(xq, xs, w_packed, M, N, K, abits, d, acc_dbg, workspace, workspace_bytes, stream, nullptr);
}

// The prefill GEMM over once-unpacked int8 B operands wu ([NT][G][k-step][lane][16 B], written by
// fq_unpack_w8_kernel): the 256 x 256 tile kernel, or the 128 x 128 one when its last-round fill is
// better (M >= PF_U8_MIN_M).
static fq_status launch_prefill_u8(const int8_t *xq, const uint16_t *xs, const void *w_packed, const char *wu, int M,
                                   int N, int K, uint16_t *d, int32_t *acc_dbg, hipStream_t s, const PbQ *q = nullptr) {
    const int NT = (N + 15) / 16;
    const long nwg = (long)((M + PF_BM - 1) / PF_BM) * ((NT + PF_TILES - 1) / PF_TILES);
    const unsigned nbig = (unsigned)(((M + PB_BM - 1) / PB_BM) * ((NT + PB_TILES - 1) / PB_TILES));
    const size_t lds_big = 2 * (size_t)(PB_ASTAGE + PB_BSTAGE);
    const bool xsf = M % PB_BM == 0;
    // 256 x 256 or 128 x 128 tiles over the unpacked weights: the larger tile is ~13 % cheaper
    // per MAC on a full chip, the smaller one fills it in finer steps (one WG per CU for 256 x
    // 256, two for 128 x 128).  Take the 128 x 128 kernel when its last-round fill beats the
    // 256 x 256 one's by more than that (tools/ab_pfm.sh, M = 2048 .. 8192 on the LLaMA-3-8B
    // shapes: e.g. M = 2048, N = 4096: 128 WGs of 256 x 256 = half the CUs, 91 -> 69 us).
    const double slots = device_cus();
    const double fill_big = nbig / (ceil(nbig / slots) * slots), fill_128 = nwg / (ceil(nwg / (2 * slots)) * 2 * slots);
    bool small_tiles = fill_big * 1.15 < fill_128;
#ifdef FQ_DEV_ABLATION
    if (const char *e = getenv("FQ_DEV_PF128")) small_tiles = atoi(e) != 0;  // development: force either
#endif
    // the 256 x 256 kernel addresses its operands by 32-bit buffer offsets (the activations and the
    // unpacked weights each below 4 GiB; every LLaMA / OPT prefill shape is far below)
    if ((uint64_t)M * K >= (1ull << 32) || (uint64_t)NT * (K / FQ_GROUP) * 2048 >= (1ull << 32)) small_tiles = true;
    if (small_tiles) {
        if (acc_dbg)
            hipLaunchKernelGGL((fq_gemm_prefill_kernel<true, 0, true>), dim3((unsigned)nwg), dim3(PF_WAVES * 64), 0, s,
                               xq, xs, (const uint32_t *)w_packed, M, N, K, d, acc_dbg, (const char *)wu, 1, nullptr);
        else
            hipLaunchKernelGGL((fq_gemm_prefill_kernel<false, 0, true>), dim3((unsigned)nwg), dim3(PF_WAVES * 64), 0, s,
                               xq, xs, (const uint32_t *)w_packed, M, N, K, d, acc_dbg, (const char *)wu, 1, nullptr);
        FQ_LAUNCH_CHECK();
        // (the 128 x 128 tile holds one group per row only across two WGs: its output is quantized apart)
        if (q) return fq_quantize_act(d, q->qM, q->qK, q->qbits, q->qx, q->qs, s);
        return FQ_OK;
    }
#define FQ_BIG(dbg, xf, qo)                                                                                  \
    hipLaunchKernelGGL((fq_gemm_prefill_big_kernel<dbg, 0, xf, qo>), dim3(nbig), dim3(PB_WAVES * 64), lds_big, s, \
                       xq, xs, (const uint32_t *)w_packed, M, N, K, d, acc_dbg, (const char *)wu, qo ? *q : PbQ{})
    if (acc_dbg) {
        if (xsf) FQ_BIG(true, true, false); else FQ_BIG(true, false, false);
    } else if (q) {
        if (xsf) FQ_BIG(false, true, true); else FQ_BIG(false, false, true);
    } else {
        if (xsf) FQ_BIG(false, true, false); else FQ_BIG(false, false, false);
    }
#undef FQ_BIG
    FQ_LAUNCH_CHECK();
    return FQ_OK;
}

fq_status fq_gemm_w6ax_impl(const int8_t *xq, const uint16_t *xs, const void *w_packed, int M, int N, int K,
                            int abits, uint16_t *d, int32_t *acc_dbg, void *workspace, size_t workspace_bytes,
                            fq_stream_t stream, const fq_gather *gat) {
    if (!xq || !xs || !w_packed || (!d && !gat)) return FQ_ERR_NULL;
    if (gat && (M > 32 || N % 16)) return FQ_ERR_SHAPE;  // peer-store gather: decode sizes, whole tiles
    if (M <= 0 || N <= 0 || K <= 0 || K % FQ_GROUP) return FQ_ERR_SHAPE;
    if ((size_t)((N + 15) / 16) > kTicketBytes / 4) return FQ_ERR_SHAPE;
    if (abits != 6 && abits != 8) return FQ_ERR_BITS;
    // The kernels are bit-width agnostic (int8 activations, values bounded by abits); abits is
    // validated for API parity with FLEXQGEMMWrapper(X_BITS, W_BITS, SIGNED).
    hipStream_t s = (hipStream_t)stream;
    if (M <= 32 || (!gat && midm_decode(M, N, K))) {
        DecodePlan p = decode_plan(M, N, K, false);
        const size_t need = fq_gemm_workspace_bytes(M, N, K);
        if (need && (!workspace || workspace_bytes < need)) return FQ_ERR_WORKSPACE;
        DecodeArgs a = {xq, xs, nullptr, abits, w_packed, M, N, K, d, acc_dbg, workspace, gat};
        return acc_dbg ? dispatch_decode<false, true>(p, a, s) : dispatch_decode<false, false>(p, a, s);
    }
    const int NT = (N + 15) / 16;
    const long nwg = (long)((M + PF_BM - 1) / PF_BM) * ((NT + PF_TILES - 1) / PF_TILES);
    if (nwg > 0x7fffffffL) return FQ_ERR_SHAPE;
#ifdef FQ_DEV_ABLATION
    if (!acc_dbg && dev_ablation() >= 1 && dev_ablation() <= 127) {
        const int abl = dev_ablation();
        const bool u8 = M >= PF_U8_MIN_M && workspace && workspace_bytes >= kTicketBytes + prefill_u8_bytes(N, K);
        char *wu = u8 ? (char *)workspace + kTicketBytes : nullptr;
        if (u8) {
            const long nblk = (long)NT * (K / FQ_GROUP);
            hipLaunchKernelGGL(fq_unpack_w8_kernel, dim3((unsigned)((nblk * 64 + 255) / 256)), dim3(256), 0, s,
                               (const char *)w_packed, nblk, wu);
        }
#define FQ_PABL(v)                                                                                         \
        if (abl == v && u8)                                                                                  \
            hipLaunchKernelGGL((fq_gemm_prefill_kernel<false, v, true>), dim3((unsigned)nwg), dim3(PF_WAVES * 64), 0, s, \
                               xq, xs, (const uint32_t *)w_packed, M, N, K, d, acc_dbg, (const char *)wu, 1, nullptr); \
        if (abl == v && !u8)                                                                                 \
            hipLaunchKernelGGL((fq_gemm_prefill_kernel<false, v>), dim3((unsigned)nwg), dim3(PF_WAVES * 64), 0, s, xq, xs, \
                               (const uint32_t *)w_packed, M, N, K, d, acc_dbg, nullptr, 1, nullptr);
        FQ_PABL(1) FQ_PABL(2) FQ_PABL(3) FQ_PABL(4) FQ_PABL(5) FQ_PABL(7) FQ_PABL(8) FQ_PABL(11) FQ_PABL(15)
        FQ_PABL(16) FQ_PABL(31) FQ_PABL(35) FQ_PABL(67) FQ_PABL(99) FQ_PABL(6) FQ_PABL(12) FQ_PABL(17) FQ_PABL(19)
#undef FQ_PABL
        FQ_LAUNCH_CHECK();
        return FQ_OK;
    }
    if (!acc_dbg && dev_ablation() >= 128 && dev_ablation() <= 255 && M >= PF_U8_MIN_M && workspace &&
        workspace_bytes >= kTicketBytes + prefill_u8_bytes(N, K)) {  // the 256 x 256 kernel, ABL = value - 128
        const int abl = dev_ablation() - 128;
        char *wu = (char *)workspace + kTicketBytes;
        const long nblk = (long)NT * (K / FQ_GROUP);
        hipLaunchKernelGGL(fq_unpack_w8_kernel, dim3((unsigned)((nblk * 64 + 255) / 256)), dim3(256), 0, s,
                           (const char *)w_packed, nblk, wu);
        const unsigned nbig = (unsigned)(((M + PB_BM - 1) / PB_BM) * ((NT + PB_TILES - 1) / PB_TILES));
        const size_t lds_big = 2 * (size_t)(PB_ASTAGE + PB_BSTAGE);
#define FQ_BABL(v)                                                                                         \
        if (abl == v)                                                                                        \
            hipLaunchKernelGGL((fq_gemm_prefill_big_kernel<false, v>), dim3(nbig), dim3(PB_WAVES * 64), lds_big, s, \
                               xq, xs, (const uint32_t *)w_packed, M, N, K, d, acc_dbg, (const char *)wu, PbQ{});
        FQ_BABL(0) FQ_BABL(1) FQ_BABL(2) FQ_BABL(3) FQ_BABL(4) FQ_BABL(8) FQ_BABL(12) FQ_BABL(16) FQ_BABL(7) FQ_BABL(15) FQ_BABL(32) \
        FQ_BABL(33) FQ_BABL(34) FQ_BABL(35) FQ_BABL(36) FQ_BABL(40) FQ_BABL(64) FQ_BABL(96) FQ_BABL(104)
#undef FQ_BABL
        FQ_LAUNCH_CHECK();
        return FQ_OK;
    }
#endif
    // Large M with room in the workspace: unpack once, then the U8 kernel (without a workspace the
    // GEMM unpacks per WG; both are bit-identical)
    if (M >= PF_U8_MIN_M && workspace && workspace_bytes >= kTicketBytes + prefill_u8_bytes(N, K)) {
        const long nblk = (long)NT * (K / FQ_GROUP);
        // after the ticket region: one workspace serves both this and the split-K decode, whose
        // tickets must stay zero between launches
        char *wu = (char *)workspace + kTicketBytes;
        hipLaunchKernelGGL(fq_unpack_w8_kernel, dim3((unsigned)((nblk * 64 + 255) / 256)), dim3(256), 0, s,
                           (const char *)w_packed, nblk, wu);
        FQ_LAUNCH_CHECK();
        return launch_prefill_u8(xq, xs, w_packed, wu, M, N, K, d, acc_dbg, s);
    }
    // Few tiles (narrow N, modest M): split K over more WGs when the workspace holds the slabs
    // (without the slabs the kernel would have to fall back to S = 1, whose fp32 summation order,
    // hence the fp16 bits, differ: the same shape must give the same bits whatever the caller's
    // buffer, so a short workspace is an error here, as for the split-K decode)
    const int S = prefill_split(M, N, K);
    if (S > 1 && (!workspace || workspace_bytes < kTicketBytes + prefill_slab_bytes(M, N, S))) return FQ_ERR_WORKSPACE;
    float *slabs = S > 1 ? reinterpret_cast<float *>((char *)workspace + kTicketBytes) : nullptr;
    const unsigned grid = (unsigned)(nwg * S);
    if (acc_dbg)
        hipLaunchKernelGGL(fq_gemm_prefill_kernel<true>, dim3(grid), dim3(PF_WAVES * 64), 0, s, xq, xs,
                           (const uint32_t *)w_packed, M, N, K, d, acc_dbg, nullptr, S, slabs);
    else
        hipLaunchKernelGGL(fq_gemm_prefill_kernel<false>, dim3(grid), dim3(PF_WAVES * 64), 0, s, xq, xs,
                           (const uint32_t *)w_packed, M, N, K, d, acc_dbg, nullptr, S, slabs);
    FQ_LAUNCH_CHECK();
    if (S > 1) {
        const long nthr = (long)M * NT * 4;
        hipLaunchKernelGGL(fq_splitk_reduce_kernel, dim3((unsigned)((nthr + 255) / 256)), dim3(256), 0, s,
                           (const float *)slabs, S, M, N, d);
        FQ_LAUNCH_CHECK();
    }
    return FQ_OK;
}

// ---- prefill with resident unpacked weights: the int8 B operands of fq_unpack_w8_kernel kept for
// the model's lifetime (1 byte per weight, 4/3 of the fq6 image) instead of unpacked on every call
extern "C" size_t fq_prefill_weight_bytes(int N, int K) {
    if (N <= 0 || K <= 0 || K % FQ_GROUP) return 0;
    return prefill_u8_bytes(N, K);
}

extern "C" fq_status fq_prefill_unpack_weights(const void *w_packed, int N, int K, void *w_u8, fq_stream_t stream) {
    if (!w_packed || !w_u8) return FQ_ERR_NULL;
    if (N <= 0 || K <= 0 || K % FQ_GROUP) return FQ_ERR_SHAPE;
    const long nblk = (long)((N + 15) / 16) * (K / FQ_GROUP);
    hipLaunchKernelGGL(fq_unpack_w8_kernel, dim3((unsigned)((nblk * 64 + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, (const char *)w_packed, nblk, (char *)w_u8);
    FQ_LAUNCH_CHECK();
    return FQ_OK;
}

extern "C" fq_status fq_gemm_w6ax_u8(const int8_t *xq, const uint16_t *xs, const void *w_packed, const void *w_u8,
                                     int M, int N, int K, int abits, uint16_t *d, int32_t *acc_dbg, void *workspace,
                                     size_t workspace_bytes, fq_stream_t stream) {
    if (!xq || !xs || !w_packed || !w_u8 || !d) return FQ_ERR_NULL;
    if (M <= 0 || N <= 0 || K <= 0 || K % FQ_GROUP) return FQ_ERR_SHAPE;
    if (abits != 6 && abits != 8) return FQ_ERR_BITS;
    if (M < PF_U8_MIN_M)  // (decode and mid-M plans do not read unpacked operands: the same bits)
        return fq_gemm_w6ax(xq, xs, w_packed, M, N, K, abits, d, acc_dbg, workspace, workspace_bytes, stream);
    const int NT = (N + 15) / 16;
    const long nwg = (long)((M + PF_BM - 1) / PF_BM) * ((NT + PF_TILES - 1) / PF_TILES);
    if (nwg > 0x7fffffffL) return FQ_ERR_SHAPE;
    return launch_prefill_u8(xq, xs, w_packed, (const char *)w_u8, M, N, K, d, acc_dbg, (hipStream_t)stream);
}

// The next input's arguments of fq_gemm_w6ax_q / _u8_q: its buffers are written while other workgroups
// still read the operands, so nothing may overlap.
static fq_status q_args_check(const int8_t *xq, const uint16_t *xs, int M, int N, int K, const uint16_t *d,
                              const int8_t *qxq, const uint16_t *qxs, int qM, int qK, int qbits) {
    if (!qxq || !qxs) return FQ_ERR_NULL;
    if (M <= 0 || N <= 0 || K <= 0 || K % FQ_GROUP) return FQ_ERR_SHAPE;
    if (qM <= 0 || qK <= 0 || qK % FQ_GROUP || (size_t)qM * qK > (size_t)M * N) return FQ_ERR_SHAPE;
    if (qbits != 6 && qbits != 8) return FQ_ERR_BITS;
    const size_t qb = (size_t)qM * qK, qsb = (size_t)(qK / FQ_GROUP) * qM * 2, db = (size_t)M * N * 2;
    if (ranges_overlap(qxq, qb, xq, (size_t)M * K) || ranges_overlap(qxq, qb, xs, (size_t)(K / FQ_GROUP) * M * 2) ||
        ranges_overlap(qxq, qb, d, db) || ranges_overlap(qxs, qsb, xq, (size_t)M * K) ||
        ranges_overlap(qxs, qsb, xs, (size_t)(K / FQ_GROUP) * M * 2) || ranges_overlap(qxs, qsb, d, db) ||
        ranges_overlap(qxq, qb, qxs, qsb))
        return FQ_ERR_SHAPE;
    return FQ_OK;
}

// Decode sizes with the quantizer in the GEMM's epilogue (decode_qe_epilogue): the unfused plan at
// M <= 16 with no k-split and one ticket per 128-column group of d.
static bool decode_q_plan(int M, int N, int K, DecodePlan *p) {
    if (M > 16 || N % FQ_GROUP || (size_t)(N / FQ_GROUP) > kTicketBytes / 4 || (size_t)M * N >= ((size_t)1 << 31))
        return false;
    *p = decode_plan(M, N, K, false);
    return p->fits && p->S == 1 && p->NCH == 1 && p->MT <= 16;
}
template <int MT, int XS, int SS>
static fq_status launch_decode_q(const DecodePlan &p, const int8_t *xq, const uint16_t *xs, const void *wpk, int M,
                                 int N, int K, int abits, uint16_t *d, void *ws, const DecodeQ &q, hipStream_t s) {
    if ((size_t)p.NT * (K / FQ_GROUP) * FQ_BLOCK >= ((size_t)1 << 32)) return FQ_ERR_SHAPE;  // (buffer offsets)
    DecodePacked pk;
    if (p.NT / p.grid != p.IPW - (p.NT % p.grid != 0) ||
        !decode_pack(N, K, abits, p.xwin, 1, 1, p.IPW, p.RC, M, p.NT % p.grid, p.grid, &pk))
        return FQ_ERR_SHAPE;
    hipLaunchKernelGGL((fq_gemm_decode_q_kernel<MT, XS, SS>), dim3(p.grid), dim3(decode_waves(MT) * 64),
                       decode_lds_bytes(p, M, N, K), s, xq, xs, (const uint32_t *)wpk, d, (char *)ws, pk.w0, pk.w1,
                       pk.w2, pk.w3, q.qxq, q.qxs, q.qM, q.qK, q.qbits);
    FQ_LAUNCH_CHECK();
    return FQ_OK;
}
template <int MT>
static fq_status dispatch_decode_q(const DecodePlan &p, const int8_t *xq, const uint16_t *xs, const void *wpk, int M,
                                   int N, int K, int abits, uint16_t *d, void *ws, const DecodeQ &q, hipStream_t s) {
    if (p.XS == 0) return launch_decode_q<MT, 0, 0>(p, xq, xs, wpk, M, N, K, abits, d, ws, q, s);
    if (p.SS == 0) return launch_decode_q<MT, 1, 0>(p, xq, xs, wpk, M, N, K, abits, d, ws, q, s);
    return launch_decode_q<MT, 1, 1>(p, xq, xs, wpk, M, N, K, abits, d, ws, q, s);
}

extern "C" size_t fq_gemm_q_workspace_bytes(int M, int N, int K) {
    const size_t g = fq_gemm_workspace_bytes(M, N, K);
    DecodePlan p;
    if (M <= 0 || N <= 0 || K <= 0 || K % FQ_GROUP || !decode_q_plan(M, N, K, &p)) return g;
    return g > kTicketBytes ? g : kTicketBytes;  // (the epilogue's group tickets)
}

extern "C" fq_status fq_gemm_w6ax_q(const int8_t *xq, const uint16_t *xs, const void *w_packed, int M, int N, int K,
                                    int abits, uint16_t *d, int8_t *qxq, uint16_t *qxs, int qM, int qK, int qbits,
                                    void *workspace, size_t workspace_bytes, fq_stream_t stream) {
    if (!xq || !xs || !w_packed || !d) return FQ_ERR_NULL;
    const fq_status qs = q_args_check(xq, xs, M, N, K, d, qxq, qxs, qM, qK, qbits);
    if (qs != FQ_OK) return qs;
    if (abits != 6 && abits != 8) return FQ_ERR_BITS;
    DecodePlan p;
#ifdef FQ_DEV_ABLATION
    const bool noq = getenv("FQ_DEV_NOQE") && atoi(getenv("FQ_DEV_NOQE"));  // (development: the two-launch form)
#else
    const bool noq = false;
#endif
    if (!noq && decode_q_plan(M, N, K, &p) && workspace && workspace_bytes >= kTicketBytes) {
        const DecodeQ q = {qxq, qxs, qM, qK, qbits};
        hipStream_t s = (hipStream_t)stream;
        switch (p.MT) {
            case 4: return dispatch_decode_q<4>(p, xq, xs, w_packed, M, N, K, abits, d, workspace, q, s);
            case 8: return dispatch_decode_q<8>(p, xq, xs, w_packed, M, N, K, abits, d, workspace, q, s);
            default: return dispatch_decode_q<16>(p, xq, xs, w_packed, M, N, K, abits, d, workspace, q, s);
        }
    }
    // (no epilogue form, or no ticket workspace: the GEMM, then the quantizer -- the same bits)
    const fq_status st = fq_gemm_w6ax(xq, xs, w_packed, M, N, K, abits, d, nullptr, workspace, workspace_bytes, stream);
    return st != FQ_OK ? st : fq_quantize_act(d, qM, qK, qbits, qxq, qxs, stream);
}

extern "C" fq_status fq_gemm_w6ax_u8_q(const int8_t *xq, const uint16_t *xs, const void *w_packed, const void *w_u8,
                                       int M, int N, int K, int abits, uint16_t *d, int8_t *qxq, uint16_t *qxs, int qM,
                                       int qK, int qbits, void *workspace, size_t workspace_bytes, fq_stream_t stream) {
    const fq_status qs = q_args_check(xq, xs, M, N, K, d, qxq, qxs, qM, qK, qbits);
    if (qs != FQ_OK) return qs;
    if (M < PF_U8_MIN_M) {  // (decode and mid-M plans do not read the unpacked operands: fq_gemm_w6ax_q's forms)
        if (!w_u8) return FQ_ERR_NULL;
        return fq_gemm_w6ax_q(xq, xs, w_packed, M, N, K, abits, d, qxq, qxs, qM, qK, qbits, workspace, workspace_bytes,
                              stream);
    }
    if (N % FQ_GROUP) {  // (no epilogue form: the GEMM, then the quantizer -- the same bits)
        const fq_status st = fq_gemm_w6ax_u8(xq, xs, w_packed, w_u8, M, N, K, abits, d, nullptr, workspace,
                                             workspace_bytes, stream);
        return st != FQ_OK ? st : fq_quantize_act(d, qM, qK, qbits, qxq, qxs, stream);
    }
    if (!xq || !xs || !w_packed || !w_u8 || !d) return FQ_ERR_NULL;
    if (K <= 0 || K % FQ_GROUP) return FQ_ERR_SHAPE;
    if (abits != 6 && abits != 8) return FQ_ERR_BITS;
    const int NT = (N + 15) / 16;
    const long nwg = (long)((M + PF_BM - 1) / PF_BM) * ((NT + PF_TILES - 1) / PF_TILES);
    if (nwg > 0x7fffffffL || (size_t)M * N >= ((size_t)1 << 40)) return FQ_ERR_SHAPE;
    const PbQ q = {qxq, qxs, qM, qK, qbits};
    return launch_prefill_u8(xq, xs, w_packed, (const char *)w_u8, M, N, K, d, nullptr, (hipStream_t)stream, &q);
}

extern "C" fq_status fq_gather_wait(const fq_gather *gather, uint32_t *err, fq_stream_t stream) {
    if (!gather) return FQ_ERR_NULL;
    hipLaunchKernelGGL(fq_gather_wait_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, gather, err);
    FQ_LAUNCH_CHECK();
    return FQ_OK;
}
