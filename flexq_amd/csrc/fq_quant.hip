// fq_quant.hip -- dynamic activation quantizer, fq6 weight packer and the reference-layout
// converters for gfx950.  HBM-bound byte work: 16-byte-per-lane coalesced loads, 16-lane
// (one DPP row) max-reductions, no LDS round trips.
#include <type_traits>

#include "fq_common.h"

// =============================================================================================
// Activation quantizer.  One 128-wide group = 16 lanes x 8 fp16 (16 B per lane), so one wave
// instruction covers 4 groups = 1 KiB.  Groups are enumerated flat over [M][K/128] (row-major,
// contiguous in memory), so any K % 128 == 0 works without per-row tails.
// Arithmetic restates e2e .../flexqgemm/src/pack/bit_packing.cu:125-164 exactly:
//   absmax in fp16 (exact as float), maxv = absmax / (2^(b-1)-1) in fp32, scale = half(maxv),
//   q = clamp(roundf(float(x) / float(scale)), lo, hi) with CUDA's saturating conversion.
// Output variants:
//   MODE 0: xq int8 [M][K] + xs fp16 [K/128][M]          (this build's GEMM input)
//   MODE 1: reference bit planes [K/128][M/c][b][c][4] + duplicated x_scale (drop-in pack)
// =============================================================================================
// IDX: index type -- 32-bit when M*K fits (64-bit division alone costs ~100 instructions per
// lane, comparable to the quantizer itself), 64-bit otherwise.
// The arguments (at most 56 bytes, the wave count passed explicitly: no hidden-argument read) are
// preloaded into SGPRs (Makefile KPRELOAD): the batch-16 step runs one such launch per linear.
template <int MODE, typename IDX>
__global__ __launch_bounds__(256) void fq_quantize_act_kernel(
    const uint16_t *__restrict__ x, int M, int K, int bits, int nwaves_, int8_t *__restrict__ xq,
    uint16_t *__restrict__ xs, int32_t *__restrict__ planes, uint16_t *__restrict__ xs_dup) {
    using U = typename std::conditional<sizeof(IDX) == 4, unsigned, unsigned long>::type;
    const int G = K / FQ_GROUP;
    const IDX T = (IDX)M * G;  // total groups
    const int lane = threadIdx.x & 63;
    const int sub = lane & 15;  // position inside the group
    const IDX wave = (IDX)((blockIdx.x * 256u + threadIdx.x) >> 6);
    const IDX nwaves = (IDX)nwaves_;

    for (IDX chunk = wave; chunk * 4 < T; chunk += nwaves) {
        const IDX gi = chunk * 4 + (lane >> 4);  // flat group index of this lane
        const bool valid = gi < T;
        uint4 raw = make_uint4(0, 0, 0, 0);
        if (valid) raw = *reinterpret_cast<const uint4 *>(x + gi * FQ_GROUP + sub * 8);
        uint2 codes;
        const uint16_t sh = quant_group16(raw, bits, codes);
        const IDX m = (IDX)((U)gi / (U)G), g = gi - m * G;
        if (MODE == 0) {
            if (valid) {
                *reinterpret_cast<uint2 *>(xq + gi * FQ_GROUP + sub * 8) = codes;
                if (sub == 0) xs[g * M + m] = sh;
            }
        } else {
            // Bit planes: word j of a group covers k = 32j..32j+31 with k0 at bit 31
            // (__brev(__ballot) at bit_packing.cu:109).  Lane sub = 4j+u holds k = 32j+8u+i.
            const int chunkM = M < 8 ? M : 8;
            const int u = sub & 3, j = sub >> 2;
            for (int b = 0; b < bits; b++) {
                uint32_t byte = 0;
#pragma unroll
                for (int i = 0; i < 8; i++) byte |= (((i < 4 ? codes.x : codes.y) >> (8 * (i & 3) + b)) & 1u) << (7 - i);
                uint32_t word = byte << (8 * (3 - u));
                word |= __shfl_xor(word, 1, 64);
                word |= __shfl_xor(word, 2, 64);
                if (valid && u == 0) {
                    long idx = g * ((long)M * bits * 4) + (m / chunkM) * (bits * chunkM * 4) +
                               b * (chunkM * 4) + (m % chunkM) * 4 + j;
                    planes[idx] = (int32_t)word;
                }
            }
            if (valid && sub == 0) {
                const int ld = 2 * ((M + 3) / 4 * 4);  // SCALE_PACKING_A(SCALE_SIZE_X(M))
                xs_dup[g * ld + 2 * m] = sh;
                xs_dup[g * ld + 2 * m + 1] = sh;
            }
        }
    }
}

static int quant_grid(long groups) {
    long waves = (groups + 3) / 4;
    long blocks = (waves + 3) / 4;
    if (blocks > 4096) blocks = 4096;
    return (int)(blocks < 1 ? 1 : blocks);
}

extern "C" fq_status fq_quantize_act(const uint16_t *x, int M, int K, int abits, int8_t *xq,
                                     uint16_t *xs, fq_stream_t stream) {
    if (!x || !xq || !xs) return FQ_ERR_NULL;
    if (M <= 0 || K <= 0 || K % FQ_GROUP) return FQ_ERR_SHAPE;
    if (abits != 6 && abits != 8) return FQ_ERR_BITS;
    const long groups = (long)M * (K / FQ_GROUP);
    const int grid = quant_grid(groups);
    if (groups * FQ_GROUP < (1L << 31))
        hipLaunchKernelGGL((fq_quantize_act_kernel<0, int>), dim3(grid), dim3(256), 0, (hipStream_t)stream, x, M, K,
                           abits, grid * 4, xq, xs, nullptr, nullptr);
    else
        hipLaunchKernelGGL((fq_quantize_act_kernel<0, long>), dim3(grid), dim3(256), 0, (hipStream_t)stream, x, M, K,
                           abits, grid * 4, xq, xs, nullptr, nullptr);
    FQ_LAUNCH_CHECK();
    return FQ_OK;
}

extern "C" fq_status fq_ref_quantize_bit_packing(const uint16_t *x, int32_t *packed,
                                                 uint16_t *x_scale_dup, int M, int K, int bits,
                                                 fq_stream_t stream) {
    if (!x || !packed || !x_scale_dup) return FQ_ERR_NULL;
    if (M <= 0 || K <= 0 || K % FQ_GROUP || (M > 8 && M % 8)) return FQ_ERR_SHAPE;
    if (bits != 6 && bits != 8) return FQ_ERR_BITS;
    const long groups = (long)M * (K / FQ_GROUP);
    const int grid = quant_grid(groups);
    hipLaunchKernelGGL((fq_quantize_act_kernel<1, long>), dim3(grid), dim3(256), 0, (hipStream_t)stream, x, M, K, bits,
                       grid * 4, nullptr, nullptr, packed, x_scale_dup);
    FQ_LAUNCH_CHECK();
    return FQ_OK;
}

// =============================================================================================
// Reference bit-plane packing of raw b-bit integers (engine/src/pack/bit_packing.cu:76-133).
// One thread per output word (row, 32-k word, bit); offline / test path.
// =============================================================================================
__global__ void fq_ref_bit_packing_kernel(const int32_t *__restrict__ in, int32_t *__restrict__ out,
                                          int R, int K, int bits) {
    const long total = (long)R * (K / 32) * bits;
    const int chunk = R < 8 ? R : 8;
    for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (long)gridDim.x * blockDim.x) {
        const int b = (int)(t % bits);
        const long rk = t / bits;
        const int kt = (int)(rk % (K / 32));
        const int r = (int)(rk / (K / 32));
        const int32_t *src = in + (long)r * K + kt * 32;
        uint32_t word = 0;
#pragma unroll 8
        for (int i = 0; i < 32; i++) word |= (((uint32_t)src[i] >> b) & 1u) << (31 - i);
        const long idx = (long)(kt / 4) * ((long)R * bits * 4) + (r / chunk) * (bits * chunk * 4) +
                         b * (chunk * 4) + (r % chunk) * 4 + (kt % 4);
        out[idx] = (int32_t)word;
    }
}

extern "C" fq_status fq_ref_bit_packing(const int32_t *in, int32_t *packed, int M, int K, int bits,
                                        fq_stream_t stream) {
    if (!in || !packed) return FQ_ERR_NULL;
    if (M <= 0 || K <= 0 || K % FQ_GROUP || (M > 8 && M % 8)) return FQ_ERR_SHAPE;
    if (bits < 1 || bits > 8) return FQ_ERR_BITS;
    const long total = (long)M * (K / 32) * bits;
    long blocks = (total + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(fq_ref_bit_packing_kernel, dim3((int)blocks), dim3(256), 0,
                       (hipStream_t)stream, in, packed, M, K, bits);
    FQ_LAUNCH_CHECK();
    return FQ_OK;
}

// =============================================================================================
// fq6 weight layout (oracle fqo_pack_fq6):
//   uint32 [Npad/16][K/128][3 plane r][64 lane][2 kstep s]
//   lane l, kstep s: column n = 16t + (l&15), k = 128g + 64s + 16(l>>4) + j (j = 0..15),
//   i.e. the B operand of v_mfma_i32_16x16x64_i8 for k-step s of the group
//   byte b of word (r, s) = ((v[4r+b] & 63) << 2) | ((v[12+b] >> 2r) & 3)
// One thread builds one lane's 24 bytes of a (tile, group) block and writes its three 8-byte
// plane words, so each wave writes three 512 B contiguous runs.  The image ends with the group
// scales blocked the same way, fp16 [Npad/16][K/128][16] (lanes 0..15 write them): a wave's
// scales for consecutive groups of one tile are contiguous, so the GEMM stages them with a few
// coalesced DMAs and each scale line is fetched by exactly one CU.
// =============================================================================================
__device__ __forceinline__ uint32_t fq6_word(const int v[16], int r) {
    uint32_t w = 0;
#pragma unroll
    for (int b = 0; b < 4; b++) {
        uint32_t byte = (((uint32_t)v[4 * r + b] & 63u) << 2) | (((uint32_t)v[12 + b] >> (2 * r)) & 3u);
        w |= byte << (8 * b);
    }
    return w;
}

// slot = (t*G + g)*64 + l
__device__ __forceinline__ void fq6_lane(long slot, int G, int &t, int &g, int &l) {
    l = (int)(slot & 63);
    const long tg = slot >> 6;
    g = (int)(tg % G);
    t = (int)(tg / G);
}
__device__ __forceinline__ int fq6_col(int t, int l) { return 16 * t + (l & 15); }
__device__ __forceinline__ int fq6_k(int g, int s, int l) { return 128 * g + 64 * s + 16 * (l >> 4); }

__device__ __forceinline__ void fq6_store(uint32_t *__restrict__ out, long slot, int l, const uint32_t p[3][2]) {
    const long base = (slot >> 6) * 384 + l * 2;  // ((t*G+g)*3 + r)*128 + l*2
#pragma unroll
    for (int r = 0; r < 3; r++) *reinterpret_cast<uint2 *>(out + base + r * 128) = make_uint2(p[r][0], p[r][1]);
}

__host__ __device__ static inline long fq6_slots(int N, int K) { return (long)((N + 15) / 16) * (K / FQ_GROUP) * 64; }
// the blocked scale region of an image: fp16 [Npad/16][G][16] after the weight blocks
__device__ __forceinline__ uint16_t *fq6_scales(uint32_t *img, int N, int K) {
    return reinterpret_cast<uint16_t *>(reinterpret_cast<char *>(img) + (size_t)((N + 15) / 16) * (K / FQ_GROUP) * 1536);
}
__device__ __forceinline__ const uint16_t *fq6_scales(const uint32_t *img, int N, int K) {
    return reinterpret_cast<const uint16_t *>(reinterpret_cast<const char *>(img) + (size_t)((N + 15) / 16) * (K / FQ_GROUP) * 1536);
}
// lanes 0..15 of a (t, g) slot store the 16 scales of the block (0 for pad columns)
__device__ __forceinline__ void fq6_store_scale(uint32_t *img, int N, int K, long slot, int l, int n, uint16_t v) {
    if (l < 16) fq6_scales(img, N, K)[(slot >> 6) * 16 + l] = (n < N) ? v : (uint16_t)0;
}

__global__ void fq_pack_w6_kernel(const int8_t *__restrict__ wq, const uint16_t *__restrict__ ws, int N,
                                  int K, uint32_t *__restrict__ out) {
    const int G = K / FQ_GROUP;
    const long total = fq6_slots(N, K);
    for (long slot = (long)blockIdx.x * blockDim.x + threadIdx.x; slot < total;
         slot += (long)gridDim.x * blockDim.x) {
        int t, g, l;
        fq6_lane(slot, G, t, g, l);
        const int n = fq6_col(t, l);
        uint32_t p[3][2];
#pragma unroll
        for (int s = 0; s < 2; s++) {
            int v[16];
            if (n < N) {
                const int4 raw = *reinterpret_cast<const int4 *>(wq + (long)n * K + fq6_k(g, s, l));
                const int w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
                for (int j = 0; j < 16; j++) v[j] = (int)(int8_t)((w[j >> 2] >> (8 * (j & 3))) & 255);
            } else {
#pragma unroll
                for (int j = 0; j < 16; j++) v[j] = 0;
            }
#pragma unroll
            for (int r = 0; r < 3; r++) p[r][s] = fq6_word(v, r);
        }
        fq6_store(out, slot, l, p);
        fq6_store_scale(out, N, K, slot, l, n, n < N ? ws[(long)g * N + n] : 0);
    }
}

__global__ void fq_unpack_w6_kernel(const uint32_t *__restrict__ in, int N, int K,
                                    int8_t *__restrict__ wq, uint16_t *__restrict__ ws) {
    const int G = K / FQ_GROUP;
    const long total = fq6_slots(N, K);
    for (long slot = (long)blockIdx.x * blockDim.x + threadIdx.x; slot < total;
         slot += (long)gridDim.x * blockDim.x) {
        int t, g, l;
        fq6_lane(slot, G, t, g, l);
        const int n = fq6_col(t, l);
        if (n >= N) continue;
        if (ws && l < 16) ws[(long)g * N + n] = fq6_scales(in, N, K)[(slot >> 6) * 16 + l];
        const long base = (slot >> 6) * 384 + l * 2;
        const uint2 P0 = *reinterpret_cast<const uint2 *>(in + base);
        const uint2 P1 = *reinterpret_cast<const uint2 *>(in + base + 128);
        const uint2 P2 = *reinterpret_cast<const uint2 *>(in + base + 256);
        const uint32_t q0[2] = {P0.x, P0.y}, q1[2] = {P1.x, P1.y}, q2[2] = {P2.x, P2.y};
#pragma unroll
        for (int s = 0; s < 2; s++) {
            v4i o = unpack_fq6(q0[s], q1[s], q2[s]);
            int4 res;
            int *rp = reinterpret_cast<int *>(&res);
#pragma unroll
            for (int d = 0; d < 4; d++) {
                uint32_t x = (uint32_t)o[d], y = 0;
#pragma unroll
                for (int b = 0; b < 4; b++) {
                    int8_t w = (int8_t)(x >> (8 * b)) >> 2;  // each byte holds 4*w
                    y |= ((uint32_t)(uint8_t)w) << (8 * b);
                }
                rp[d] = (int)y;
            }
            *reinterpret_cast<int4 *>(wq + (long)n * K + fq6_k(g, s, l)) = res;
        }
    }
}

static int grid_for(long total) {
    long blocks = (total + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    return (int)(blocks < 1 ? 1 : blocks);
}

extern "C" size_t fq_packed_w_bytes(int N, int K) {
    if (N <= 0 || K <= 0 || K % FQ_GROUP) return 0;
    return (size_t)((N + 15) / 16) * (K / FQ_GROUP) * (1536 + 32);
}

extern "C" fq_status fq_pack_w6(const int8_t *wq, const uint16_t *ws, int N, int K, void *w_packed,
                                fq_stream_t stream) {
    if (!wq || !ws || !w_packed) return FQ_ERR_NULL;
    if (N <= 0 || K <= 0 || K % FQ_GROUP) return FQ_ERR_SHAPE;
    const long total = fq6_slots(N, K);
    hipLaunchKernelGGL(fq_pack_w6_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream,
                       wq, ws, N, K, (uint32_t *)w_packed);
    FQ_LAUNCH_CHECK();
    return FQ_OK;
}

extern "C" fq_status fq_unpack_w6(const void *w_packed, int N, int K, int8_t *wq, uint16_t *ws,
                                  fq_stream_t stream) {
    if (!wq || !w_packed) return FQ_ERR_NULL;
    if (N <= 0 || K <= 0 || K % FQ_GROUP) return FQ_ERR_SHAPE;
    const long total = fq6_slots(N, K);
    hipLaunchKernelGGL(fq_unpack_w6_kernel, dim3(grid_for(total)), dim3(256), 0,
                       (hipStream_t)stream, (const uint32_t *)w_packed, N, K, wq, ws);
    FQ_LAUNCH_CHECK();
    return FQ_OK;
}

// ---- fp16 weight -> scales (pass 1) and codes + fq6 (pass 2), engine rounding rule ----------
__global__ void fq_weight_scale_kernel(const uint16_t *__restrict__ w, int N, int K,
                                       uint16_t *__restrict__ ws) {
    // one 16-lane row per (n, g): same reduction as the activation quantizer (bits = 6)
    const int G = K / FQ_GROUP;
    const long T = (long)N * G;
    const int lane = threadIdx.x & 63, sub = lane & 15;
    const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const long nwaves = ((long)gridDim.x * blockDim.x) >> 6;
    for (long chunk = wave; chunk * 4 < T; chunk += nwaves) {
        const long gi = chunk * 4 + (lane >> 4);
        const bool valid = gi < T;
        uint4 raw = make_uint4(0, 0, 0, 0);
        if (valid) raw = *reinterpret_cast<const uint4 *>(w + gi * FQ_GROUP + sub * 8);
        const uint32_t d[4] = {raw.x, raw.y, raw.z, raw.w};
        float mx = -1.0f;
#pragma unroll
        for (int i = 0; i < 8; i++) mx = fmaxf(mx, fabsf(h2f((uint16_t)(d[i >> 1] >> (16 * (i & 1))))));
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
        if (valid && sub == 0) {
            const long n = gi / G, g = gi % G;
            ws[g * N + n] = f2h(mx / 31.0f);
        }
    }
}

__global__ void fq_weight_pack_kernel(const uint16_t *__restrict__ w, const uint16_t *__restrict__ ws,
                                      int N, int K, uint32_t *__restrict__ out,
                                      int8_t *__restrict__ wq_out) {
    const int G = K / FQ_GROUP;
    const long total = fq6_slots(N, K);
    for (long slot = (long)blockIdx.x * blockDim.x + threadIdx.x; slot < total;
         slot += (long)gridDim.x * blockDim.x) {
        int t, g, l;
        fq6_lane(slot, G, t, g, l);
        const int n = fq6_col(t, l);
        uint32_t p[3][2];
        const float r = (n < N) ? h2f(ws[(long)g * N + n]) : 1.0f;
#pragma unroll
        for (int s = 0; s < 2; s++) {
            const int k0 = fq6_k(g, s, l);
            int v[16];
            if (n < N) {
                const uint4 *src = reinterpret_cast<const uint4 *>(w + (long)n * K + k0);
                const uint4 a = src[0], b = src[1];
                const uint32_t d[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
                for (int j = 0; j < 16; j++)
                    v[j] = sat_clamp(round_half_away(h2f((uint16_t)(d[j >> 1] >> (16 * (j & 1)))) / r), -32, 31);
                if (wq_out) {
                    uint32_t pk[4];
#pragma unroll
                    for (int q = 0; q < 4; q++)
                        pk[q] = (v[4 * q] & 255) | ((v[4 * q + 1] & 255) << 8) | ((v[4 * q + 2] & 255) << 16) |
                                ((uint32_t)(v[4 * q + 3] & 255) << 24);
                    *reinterpret_cast<uint4 *>(wq_out + (long)n * K + k0) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
                }
            } else {
#pragma unroll
                for (int j = 0; j < 16; j++) v[j] = 0;
            }
#pragma unroll
            for (int rr = 0; rr < 3; rr++) p[rr][s] = fq6_word(v, rr);
        }
        fq6_store(out, slot, l, p);
        fq6_store_scale(out, N, K, slot, l, n, n < N ? ws[(long)g * N + n] : 0);
    }
}

extern "C" fq_status fq_quantize_pack_w6(const uint16_t *w, int N, int K, void *w_packed,
                                         uint16_t *ws, int8_t *wq_out, fq_stream_t stream) {
    if (!w || !w_packed || !ws) return FQ_ERR_NULL;
    if (N <= 0 || K <= 0 || K % FQ_GROUP) return FQ_ERR_SHAPE;
    hipLaunchKernelGGL(fq_weight_scale_kernel, dim3(quant_grid((long)N * (K / FQ_GROUP))), dim3(256),
                       0, (hipStream_t)stream, w, N, K, ws);
    FQ_LAUNCH_CHECK();
    const long total = fq6_slots(N, K);
    hipLaunchKernelGGL(fq_weight_pack_kernel, dim3(grid_for(total)), dim3(256), 0,
                       (hipStream_t)stream, w, ws, N, K, (uint32_t *)w_packed, wq_out);
    FQ_LAUNCH_CHECK();
    return FQ_OK;
}

// ---- reference bit-plane layout -> this build's layouts ------------------------------------
__device__ __forceinline__ int bitplane_value(const int32_t *__restrict__ planes, int R, int bits,
                                              int r, int k) {
    const int chunk = R < 8 ? R : 8;
    const int kt = k >> 5;
    const long base = (long)(kt / 4) * ((long)R * bits * 4) + (r / chunk) * (bits * chunk * 4) +
                      (r % chunk) * 4 + (kt % 4);
    int v = 0;
    for (int b = 0; b < bits; b++) {
        const int bit = ((uint32_t)planes[base + b * (chunk * 4)] >> (31 - (k & 31))) & 1;
        v += (b == bits - 1) ? -(bit << b) : (bit << b);
    }
    return v;
}

__global__ void fq_import_ref_w_kernel(const int32_t *__restrict__ planes, const uint16_t *__restrict__ ws,
                                       int N, int K, uint32_t *__restrict__ out) {
    const int G = K / FQ_GROUP;
    const long total = fq6_slots(N, K);
    for (long slot = (long)blockIdx.x * blockDim.x + threadIdx.x; slot < total;
         slot += (long)gridDim.x * blockDim.x) {
        int t, g, l;
        fq6_lane(slot, G, t, g, l);
        const int n = fq6_col(t, l);
        uint32_t p[3][2];
#pragma unroll
        for (int s = 0; s < 2; s++) {
            int v[16];
            const int k0 = fq6_k(g, s, l);
#pragma unroll
            for (int j = 0; j < 16; j++) v[j] = (n < N) ? bitplane_value(planes, N, 6, n, k0 + j) : 0;
#pragma unroll
            for (int r = 0; r < 3; r++) p[r][s] = fq6_word(v, r);
        }
        fq6_store(out, slot, l, p);
        fq6_store_scale(out, N, K, slot, l, n, n < N ? ws[(long)g * N + n] : 0);
    }
}

__global__ void fq_import_ref_x_kernel(const int32_t *__restrict__ planes,
                                       const uint16_t *__restrict__ xs_dup, int M, int K, int bits,
                                       int8_t *__restrict__ xq, uint16_t *__restrict__ xs) {
    const long total = (long)M * K;
    const int ld = 2 * ((M + 3) / 4 * 4);
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long)gridDim.x * blockDim.x) {
        const int m = (int)(i / K), k = (int)(i % K);
        xq[i] = (int8_t)bitplane_value(planes, M, bits, m, k);
        if ((k & (FQ_GROUP - 1)) == 0) xs[(long)(k / FQ_GROUP) * M + m] = xs_dup[(long)(k / FQ_GROUP) * ld + 2 * m];
    }
}

extern "C" fq_status fq_import_ref_w(const int32_t *w_bitplanes, const uint16_t *w_scale, int N, int K,
                                     void *w_packed, fq_stream_t stream) {
    if (!w_bitplanes || !w_scale || !w_packed) return FQ_ERR_NULL;
    if (N <= 0 || K <= 0 || K % FQ_GROUP || (N > 8 && N % 8)) return FQ_ERR_SHAPE;
    const long total = fq6_slots(N, K);
    hipLaunchKernelGGL(fq_import_ref_w_kernel, dim3(grid_for(total)), dim3(256), 0,
                       (hipStream_t)stream, w_bitplanes, w_scale, N, K, (uint32_t *)w_packed);
    FQ_LAUNCH_CHECK();
    return FQ_OK;
}

extern "C" fq_status fq_import_ref_x(const int32_t *x_bitplanes, const uint16_t *x_scale_dup, int M,
                                     int K, int bits, int8_t *xq, uint16_t *xs, fq_stream_t stream) {
    if (!x_bitplanes || !x_scale_dup || !xq || !xs) return FQ_ERR_NULL;
    if (M <= 0 || K <= 0 || K % FQ_GROUP || (M > 8 && M % 8)) return FQ_ERR_SHAPE;
    if (bits != 6 && bits != 8) return FQ_ERR_BITS;
    hipLaunchKernelGGL(fq_import_ref_x_kernel, dim3(grid_for((long)M * K)), dim3(256), 0,
                       (hipStream_t)stream, x_bitplanes, x_scale_dup, M, K, bits, xq, xs);
    FQ_LAUNCH_CHECK();
    return FQ_OK;
}
