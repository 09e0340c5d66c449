// fq_api.hip -- remaining C-ABI entry points: info, fused linear, FQBMMA-style state API.
#include "fq_common.h"

fq_status fq_decode_linear_fused(const uint16_t *x, int M, int N, int K, int abits, const void *w_packed,
                                 uint16_t *d, int32_t *acc_dbg, void *workspace, size_t workspace_bytes,
                                 hipStream_t s, bool *launched);

extern "C" const char *fq_version(void) { return "flexq_amd 0.1.0 (gfx950, int8-MFMA W6Ax)"; }

extern "C" const char *fq_status_string(fq_status s) {
    switch (s) {
        case FQ_OK: return "ok";
        case FQ_ERR_NULL: return "null pointer argument";
        case FQ_ERR_SHAPE: return "unsupported shape (K must be a positive multiple of 128)";
        case FQ_ERR_BITS: return "unsupported bit width (W6 with A6 or A8)";
        case FQ_ERR_WORKSPACE: return "workspace missing or too small";
        case FQ_ERR_HIP: return "HIP launch failed";
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
                                          workspace_bytes, (hipStream_t)stream, &launched);
    if (launched || st != FQ_OK) return st;
    if (!xq_buf || !xs_buf) return FQ_ERR_NULL;
    st = fq_quantize_act(x, M, K, abits, xq_buf, xs_buf, stream);
    if (st != FQ_OK) return st;
    return fq_gemm_w6ax(xq_buf, xs_buf, w_packed, M, N, K, abits, d, nullptr, workspace,
                        workspace_bytes, stream);
}

// ---- FQBMMAOpState-style interface over reference-layout activations -------------------------
static size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

extern "C" size_t fq_bmma_scratch_bytes(int M, int N, int K) {
    if (M <= 0 || N <= 0 || K <= 0 || K % FQ_GROUP) return 0;
    return align256((size_t)M * K) + align256((size_t)M * (K / FQ_GROUP) * 2) +
           align256(fq_gemm_workspace_bytes(M, N, K));
}

extern "C" fq_bmma_state fq_bmma_init(const int32_t *X, const void *W, const uint16_t *X_SCALE,
                                      const uint16_t *W_SCALE, int M, int N, int K, uint16_t *D,
                                      int group_size, int bias, int x_bits, int w_bits,
                                      void *scratch, size_t scratch_bytes) {
    fq_bmma_state st = {};
    st.M = M;
    st.N = N;
    st.K = K;
    st.x_bits = x_bits;
    st.w_bits = w_bits;
    st.group_size = group_size;
    st.X = X;
    st.W = W;
    st.X_SCALE = X_SCALE;
    st.W_SCALE = W_SCALE;
    st.D = D;
    st.scratch = scratch;
    st.scratch_bytes = scratch_bytes;
    // Same acceptance rules as FQBMMAOp::initialize (flexq_bmma_op.h:81-133): group 128, no bias,
    // K % 128 == 0; plus this build's W6 / A{6,8} and the bit-plane row rule (M <= 8 or M % 8 == 0).
    // W is the weight image (fq_import_ref_w(W planes, W_SCALE) once, offline): it carries the
    // group scales, so W_SCALE is kept for the signature and may be NULL.
    st.init_success = X && W && X_SCALE && D && group_size == FQ_GROUP && !bias &&
                      M > 0 && N > 0 && K > 0 && K % FQ_GROUP == 0 && (M <= 8 || M % 8 == 0) &&
                      w_bits == 6 && (x_bits == 6 || x_bits == 8) && scratch &&
                      scratch_bytes >= fq_bmma_scratch_bytes(M, N, K);
    return st;
}

extern "C" fq_status fq_bmma_exec(const fq_bmma_state *st, fq_stream_t stream) {
    if (!st || !st->init_success) return FQ_ERR_NULL;
    char *base = (char *)st->scratch;
    int8_t *xq = (int8_t *)base;
    uint16_t *xs = (uint16_t *)(base + align256((size_t)st->M * st->K));
    void *ws = base + align256((size_t)st->M * st->K) + align256((size_t)st->M * (st->K / FQ_GROUP) * 2);
    fq_status s = fq_import_ref_x(st->X, st->X_SCALE, st->M, st->K, st->x_bits, xq, xs, stream);
    if (s != FQ_OK) return s;
    return fq_gemm_w6ax(xq, xs, st->W, st->M, st->N, st->K, st->x_bits, st->D, nullptr,
                        ws, fq_gemm_workspace_bytes(st->M, st->N, st->K), stream);
}
