// fq_api.hip -- remaining C-ABI entry points: info, fused linear, FQBMMA-style state API.
#include "fq_common.h"

fq_status fq_decode_linear_fused(const uint16_t *x, int M, int N, int K, int abits, const void *w_packed,
                                 uint16_t *d, int32_t *acc_dbg, void *workspace, size_t workspace_bytes,
                                 hipStream_t s, bool *launched, const fq_gather *gat,
                                 const fq_gather *wgat = nullptr, uint32_t *werr = nullptr);
fq_status fq_gemm_w6ax_impl(const int8_t *xq, const uint16_t *xs, const void *w_packed, int M, int N, int K,
                            int abits, uint16_t *d, int32_t *acc_dbg, void *workspace, size_t workspace_bytes,
                            fq_stream_t stream, const fq_gather *gat);
fq_status fq_decode_linear_pro(int pro, const uint16_t *xh, const DecodePro &prod, int M, int N, int K, int abits,
                               const void *w_packed, uint16_t *d, void *workspace, size_t workspace_bytes,
                               hipStream_t s, bool *launched);
fq_status fq_rmsnorm_quantize_to(const uint16_t *input, const uint16_t *residual, uint16_t *res_out,
                                 const uint16_t *gamma, float eps, int M, int K, int abits, int8_t *xq, uint16_t *xs,
                                 uint16_t *normed_out, fq_stream_t stream);

extern "C" const char *fq_version(void) { return "flexq_amd 0.4.0 (gfx950, int8-MFMA W6Ax)"; }
extern "C" int fq_abi_version(void) { return FQ_ABI_VERSION; }

extern "C" const char *fq_status_string(fq_status s) {
    switch (s) {
        case FQ_OK: return "ok";
        case FQ_ERR_NULL: return "null pointer argument";
        case FQ_ERR_SHAPE: return "unsupported shape (K must be a positive multiple of 128)";
        case FQ_ERR_BITS: return "unsupported bit width (W6 with A6 or A8)";
        case FQ_ERR_WORKSPACE: return "workspace missing or too small";
        case FQ_ERR_HIP: return "HIP launch failed";
        case FQ_ERR_TIMEOUT: return "a decode chain wait timed out on this chain workspace (fq_chain_reset)";
        default: return "unknown status";
    }
}

extern "C" fq_status fq_linear_w6ax(const uint16_t *x, int M, int N, int K, int abits,
                                    const void *w_packed, uint16_t *d,
                                    int8_t *xq_buf, uint16_t *xs_buf, void *workspace,
                                    size_t workspace_bytes, fq_stream_t stream) {
    if (!x || !w_packed || !d) return FQ_ERR_NULL;
    if (M <= 0 || N <= 0 || K <= 0 || K % FQ_GROUP) return FQ_ERR_SHAPE;
    if (abits != 6 && abits != 8) return FQ_ERR_BITS;
    // decode sizes: one launch, the quantizer runs inside the GEMM's prologue (xq/xs untouched)
    bool launched = false;
    fq_status st = fq_decode_linear_fused(x, M, N, K, abits, w_packed, d, nullptr, workspace,
                                          workspace_bytes, (hipStream_t)stream, &launched, nullptr);
    if (launched || st != FQ_OK) return st;
    if (!xq_buf || !xs_buf) return FQ_ERR_NULL;
    st = fq_quantize_act(x, M, K, abits, xq_buf, xs_buf, stream);
    if (st != FQ_OK) return st;
    return fq_gemm_w6ax(xq_buf, xs_buf, w_packed, M, N, K, abits, d, nullptr, workspace,
                        workspace_bytes, stream);
}

extern "C" fq_status fq_linear_w6ax_gather(const uint16_t *x, int M, int N, int K, int abits,
                                           const void *w_packed, const fq_gather *gather, int8_t *xq_buf,
                                           uint16_t *xs_buf, void *workspace, size_t workspace_bytes,
                                           fq_stream_t stream) {
    if (!x || !w_packed || !gather) return FQ_ERR_NULL;
    if (M <= 0 || M > 32 || N <= 0 || N % 16 || K <= 0 || K % FQ_GROUP) return FQ_ERR_SHAPE;
    if (abits != 6 && abits != 8) return FQ_ERR_BITS;
    bool launched = false;
    fq_status st = fq_decode_linear_fused(x, M, N, K, abits, w_packed, nullptr, nullptr, workspace,
                                          workspace_bytes, (hipStream_t)stream, &launched, gather);
    if (launched || st != FQ_OK) return st;
    if (!xq_buf || !xs_buf) return FQ_ERR_NULL;
    st = fq_quantize_act(x, M, K, abits, xq_buf, xs_buf, stream);
    if (st != FQ_OK) return st;
    return fq_gemm_w6ax_impl(xq_buf, xs_buf, w_packed, M, N, K, abits, nullptr, nullptr, workspace,
                             workspace_bytes, stream, gather);
}

// The gather kernel with the previous gather's wait folded into its prologue (one launch) where the
// linear fuses its quantizer; otherwise fq_gather_wait, then fq_linear_w6ax_gather.
extern "C" fq_status fq_linear_w6ax_gather_after(const uint16_t *x, const fq_gather *in_gather, uint32_t *err, int M,
                                                 int N, int K, int abits, const void *w_packed,
                                                 const fq_gather *gather, int8_t *xq_buf, uint16_t *xs_buf,
                                                 void *workspace, size_t workspace_bytes, fq_stream_t stream) {
    if (!x || !w_packed || !gather || !in_gather) return FQ_ERR_NULL;
    if (M <= 0 || M > 32 || N <= 0 || N % 16 || K <= 0 || K % FQ_GROUP) return FQ_ERR_SHAPE;
    if (abits != 6 && abits != 8) return FQ_ERR_BITS;
    bool launched = false;
    fq_status st = fq_decode_linear_fused(x, M, N, K, abits, w_packed, nullptr, nullptr, workspace, workspace_bytes,
                                          (hipStream_t)stream, &launched, gather, in_gather, err);
    if (launched || st != FQ_OK) return st;
    st = fq_gather_wait(in_gather, err, stream);
    if (st != FQ_OK) return st;
    return fq_linear_w6ax_gather(x, M, N, K, abits, w_packed, gather, xq_buf, xs_buf, workspace, workspace_bytes,
                                 stream);
}

static bool overlaps(const void *a, size_t na, const void *b, size_t nb) {
    if (!a || !b) return false;
    const uintptr_t x = (uintptr_t)a, y = (uintptr_t)b;
    return x < y + nb && y < x + na;
}

// ---- producers fused into the linear (the caller side of the path) --------
// One launch at decode sizes (the producer runs in the decode kernel's prologue); otherwise the
// producer kernel into xq_buf / xs_buf, then the GEMM.  Same bits either way: both run
// fq_common.h's producer arithmetic and the same quantizer and GEMM plan.
extern "C" fq_status fq_rmsnorm_linear_w6ax(const uint16_t *input, const uint16_t *residual, uint16_t *residual_out,
                                            const uint16_t *gamma, float eps, int M, int N, int K, int abits,
                                            const void *w_packed, uint16_t *d, int8_t *xq_buf, uint16_t *xs_buf,
                                            void *workspace, size_t workspace_bytes, fq_stream_t stream) {
    if (!residual || !gamma || !w_packed || !d || (input && !residual_out)) return FQ_ERR_NULL;
    if (M <= 0 || N <= 0 || K <= 0 || K % FQ_GROUP) return FQ_ERR_SHAPE;
    if (abits != 6 && abits != 8) return FQ_ERR_BITS;
    const uintptr_t al = (uintptr_t)residual | (uintptr_t)gamma | (uintptr_t)input | (uintptr_t)residual_out;
    if (al & 15) return FQ_ERR_SHAPE;
    // the one-launch form: workgroup 0 writes residual_out while the others still read the residual,
    // the input and gamma, so residual_out must overlap none of them (the unfused form would be
    // alias-safe, but both forms must give the same bits)
    const size_t rb = (size_t)M * K * 2;
    if (input && (overlaps(residual_out, rb, residual, rb) || overlaps(residual_out, rb, input, rb) ||
                  overlaps(residual_out, rb, gamma, (size_t)K * 2)))
        return FQ_ERR_SHAPE;
    bool launched = false;
    const DecodePro pro = {input, gamma, residual_out, eps, K, nullptr, nullptr};
    fq_status st = fq_decode_linear_pro(1, residual, pro, M, N, K, abits, w_packed, d, workspace, workspace_bytes,
                                        (hipStream_t)stream, &launched);
    if (launched || st != FQ_OK) return st;
    if (!xq_buf || !xs_buf) return FQ_ERR_NULL;
    st = fq_rmsnorm_quantize_to(input, residual, input ? residual_out : nullptr, gamma, eps, M, K, abits, xq_buf,
                                xs_buf, nullptr, stream);
    if (st != FQ_OK) return st;
    return fq_gemm_w6ax(xq_buf, xs_buf, w_packed, M, N, K, abits, d, nullptr, workspace, workspace_bytes, stream);
}

extern "C" fq_status fq_layernorm_linear_w6ax(const uint16_t *input, const uint16_t *residual, const uint16_t *bias,
                                              uint16_t *residual_out, const uint16_t *gamma, const uint16_t *beta,
                                              float eps, int M, int N, int K, int abits, const void *w_packed,
                                              uint16_t *d, int8_t *xq_buf, uint16_t *xs_buf, void *workspace,
                                              size_t workspace_bytes, fq_stream_t stream) {
    if (!residual || !gamma || !w_packed || !d) return FQ_ERR_NULL;
    if (M <= 0 || N <= 0 || K <= 0 || K % FQ_GROUP) return FQ_ERR_SHAPE;
    if (abits != 6 && abits != 8) return FQ_ERR_BITS;
    const uintptr_t al = (uintptr_t)residual | (uintptr_t)gamma | (uintptr_t)input | (uintptr_t)residual_out |
                         (uintptr_t)beta | (uintptr_t)bias;
    if (al & 15) return FQ_ERR_SHAPE;
    const size_t rb = (size_t)M * K * 2, vb = (size_t)K * 2;  // (as fq_rmsnorm_linear_w6ax)
    if (overlaps(residual_out, rb, residual, rb) || overlaps(residual_out, rb, input, rb) ||
        overlaps(residual_out, rb, gamma, vb) || overlaps(residual_out, rb, beta, vb) ||
        overlaps(residual_out, rb, bias, vb))
        return FQ_ERR_SHAPE;
    bool launched = false;
    const DecodePro pro = {input, gamma, residual_out, eps, K, beta, bias};
    fq_status st = fq_decode_linear_pro(4, residual, pro, M, N, K, abits, w_packed, d, workspace, workspace_bytes,
                                        (hipStream_t)stream, &launched);
    if (launched || st != FQ_OK) return st;
    if (!xq_buf || !xs_buf) return FQ_ERR_NULL;
    st = fq_layernorm_quantize(input, residual, bias, residual_out, gamma, beta, eps, M, K, abits, xq_buf, xs_buf,
                               nullptr, stream);
    if (st != FQ_OK) return st;
    return fq_gemm_w6ax(xq_buf, xs_buf, w_packed, M, N, K, abits, d, nullptr, workspace, workspace_bytes, stream);
}

extern "C" fq_status fq_silu_linear_w6ax(const uint16_t *gate, const uint16_t *up, int ld, int M, int N, int K,
                                         int abits, const void *w_packed, uint16_t *d, int8_t *xq_buf,
                                         uint16_t *xs_buf, void *workspace, size_t workspace_bytes,
                                         fq_stream_t stream) {
    if (!gate || !up || !w_packed || !d) return FQ_ERR_NULL;
    if (M <= 0 || N <= 0 || K <= 0 || K % FQ_GROUP || ld < K || ld % 8 || M > 65535) return FQ_ERR_SHAPE;
    if (abits != 6 && abits != 8) return FQ_ERR_BITS;
    if (((uintptr_t)gate | (uintptr_t)up) & 15) return FQ_ERR_SHAPE;
    bool launched = false;
    const DecodePro pro = {up, nullptr, nullptr, 0.0f, ld, nullptr, nullptr};
    fq_status st = fq_decode_linear_pro(2, gate, pro, M, N, K, abits, w_packed, d, workspace, workspace_bytes,
                                        (hipStream_t)stream, &launched);
    if (launched || st != FQ_OK) return st;
    if (!xq_buf || !xs_buf) return FQ_ERR_NULL;
    st = fq_silu_mul_quantize(gate, up, ld, M, K, abits, xq_buf, xs_buf, nullptr, stream);
    if (st != FQ_OK) return st;
    return fq_gemm_w6ax(xq_buf, xs_buf, w_packed, M, N, K, abits, d, nullptr, workspace, workspace_bytes, stream);
}

// ---- FQBMMAOpState-style interface (flexq_bmma_op.h:19-34,163-188) ---------------------------
// scratch layout: [GEMM workspace (split-K tickets first) | weight image (bit-plane W only) |
//                  xq int8 [M][K] | xs fp16 [K/128][M]], each 256-byte aligned.
static size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }
static size_t bmma_ws_bytes(int M, int N, int K) { return align256(fq_gemm_workspace_bytes(M, N, K)); }
static size_t bmma_img_bytes(int N, int K, int w_format) {
    return w_format == FQ_W_BITPLANES ? align256(fq_packed_w_bytes(N, K)) : 0;
}
static size_t bmma_x_bytes(int M, int K) { return align256((size_t)M * K) + align256((size_t)M * (K / FQ_GROUP) * 2); }

static size_t bmma_scratch(int M, int N, int K, int w_format) {
    if (M <= 0 || N <= 0 || K <= 0 || K % FQ_GROUP) return 0;
    return bmma_ws_bytes(M, N, K) + bmma_img_bytes(N, K, w_format) + bmma_x_bytes(M, K);
}
extern "C" size_t fq_bmma_scratch_bytes(int M, int N, int K) { return bmma_scratch(M, N, K, FQ_W_BITPLANES); }
extern "C" size_t fq_bmma_image_scratch_bytes(int M, int N, int K) { return bmma_scratch(M, N, K, FQ_W_IMAGE); }

static fq_bmma_state bmma_init(const int32_t *X, const void *W, int w_format, const uint16_t *X_SCALE,
                               const uint16_t *W_SCALE, int M, int N, int K, uint16_t *D, int group_size,
                               int bias, int x_bits, int w_bits, void *scratch, size_t scratch_bytes) {
    fq_bmma_state st = {};
    st.M = M;
    st.N = N;
    st.K = K;
    st.x_bits = x_bits;
    st.w_bits = w_bits;
    st.group_size = group_size;
    st.w_format = w_format;
    st.X = X;
    st.W = W;
    st.X_SCALE = X_SCALE;
    st.W_SCALE = W_SCALE;
    st.D = D;
    st.scratch = scratch;
    st.scratch_bytes = scratch_bytes;
    st.prepared = 0;
    // FQBMMAOp::initialize's acceptance rules (flexq_bmma_op.h:81-133): group 128, no bias,
    // K % 128 == 0; plus this build's W6 / A{6,8}, the bit-plane row rule (rows <= 8 or a multiple
    // of 8, for X and -- in bit-plane form -- for W) and the scratch it needs.  Bit-plane W needs
    // its W_SCALE (the reference reads it in every GEMM); an image already carries its scales.
    const bool rows_ok = (M <= 8 || M % 8 == 0) && (w_format == FQ_W_IMAGE || N <= 8 || N % 8 == 0);
    st.init_success = X && W && X_SCALE && D && (w_format == FQ_W_IMAGE || W_SCALE) &&
                      group_size == FQ_GROUP && !bias && M > 0 && N > 0 && K > 0 && K % FQ_GROUP == 0 &&
                      rows_ok && w_bits == 6 && (x_bits == 6 || x_bits == 8) && scratch &&
                      scratch_bytes >= bmma_scratch(M, N, K, w_format) &&
                      (size_t)((N + 15) / 16) <= 65536;
    return st;
}

extern "C" fq_bmma_state fq_bmma_init(const int32_t *X, const int32_t *W, const uint16_t *X_SCALE,
                                      const uint16_t *W_SCALE, int M, int N, int K, uint16_t *D,
                                      int group_size, int bias, int x_bits, int w_bits, void *scratch,
                                      size_t scratch_bytes) {
    return bmma_init(X, W, FQ_W_BITPLANES, X_SCALE, W_SCALE, M, N, K, D, group_size, bias, x_bits, w_bits,
                     scratch, scratch_bytes);
}

extern "C" fq_bmma_state fq_bmma_init_image(const int32_t *X, const void *W_image, const uint16_t *X_SCALE,
                                            int M, int N, int K, uint16_t *D, int group_size, int bias,
                                            int x_bits, int w_bits, void *scratch, size_t scratch_bytes) {
    return bmma_init(X, W_image, FQ_W_IMAGE, X_SCALE, nullptr, M, N, K, D, group_size, bias, x_bits, w_bits,
                     scratch, scratch_bytes);
}

extern "C" fq_status fq_bmma_exec(fq_bmma_state *st, fq_stream_t stream) {
    if (!st || !st->init_success) return FQ_ERR_NULL;
    char *base = (char *)st->scratch;
    const size_t wsb = bmma_ws_bytes(st->M, st->N, st->K), imgb = bmma_img_bytes(st->N, st->K, st->w_format);
    void *ws = base;
    void *img = base + wsb;
    int8_t *xq = (int8_t *)(base + wsb + imgb);
    uint16_t *xs = (uint16_t *)(base + wsb + imgb + align256((size_t)st->M * st->K));
    fq_status s;
    if (!st->prepared) {  // first exec on this scratch: zero the ticket region, import W once
        if ((s = fq_workspace_init(ws, wsb, stream)) != FQ_OK) return s;
        if (st->w_format == FQ_W_BITPLANES &&
            (s = fq_import_ref_w((const int32_t *)st->W, st->W_SCALE, st->N, st->K, img, stream)) != FQ_OK)
            return s;
        st->prepared = 1;
    }
    // decode sizes: one launch, the planes unpacked inside the GEMM; otherwise imported into xq / xs
    return fq_gemm_w6ax_planes(st->X, st->X_SCALE, st->w_format == FQ_W_BITPLANES ? img : st->W, st->M, st->N,
                               st->K, st->x_bits, st->D, xq, xs, ws, fq_gemm_workspace_bytes(st->M, st->N, st->K),
                               stream);
}
