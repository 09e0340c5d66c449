/*
 * flexq_hip.h -- C ABI of the MI355X-native (gfx950) W6Ax quantized-linear engine.
 *
 * The library (flexq_amd/libflexq_hip.so) replaces the hot path of FlexQ (hoffmann-muki/FlexQ):
 * INT6 weight packing, dynamic per-group (g = 128) INT6/INT8 activation quantization and the
 * W6A6 / W6A8 GEMM with per-group dequantization to fp16.  Paths below are relative to the
 * reference checkout.
 *
 * Conventions
 *   - Plain pointers and sizes only.  Every pointer argument except where marked "host" is a
 *     device pointer owned by the caller; the library never allocates or frees device memory
 *     inside an entry point, never synchronises, and never prints.  All work is enqueued on the
 *     given stream (NULL = the default stream), so every entry point is safe to capture in a HIP
 *     graph.  fp16 values are passed as uint16_t bit patterns.
 *   - Every entry point returns an fq_status; non-zero means nothing was enqueued (argument
 *     errors) or the launch failed (FQ_ERR_HIP).  The reference's error behaviour was
 *     print-and-return (flexq_gemm_wrapper.cu:44,88,93) or `initSuccess=false`
 *     (flexq_bmma_op.h:103-126); here the same conditions return a status code instead.
 *   - Group size is fixed at 128 along K (flexq_bmma_kernel.h:54,71); K % 128 == 0 is required
 *     (test_bgemm_kernel.cu:173-176, flexq_gemm_wrapper.cu:43-46).  Weight bits are 6; activation
 *     bits are 6 or 8 (the two instantiated families, flexq_bmma_library.cu:23-497).
 *
 * Data layouts owned by this build
 *   xq   int8  [M][K]               activation codes (values in [-32,31] for A6, [-128,127] for A8)
 *   xs   fp16  [K/128][M]           activation group scales
 *   wpk  bytes fq_packed_w_bytes(N,K): the weight image -- 6-bit codes in "fq6" blocks (16
 *                                   columns x one 128-group, 1.5 KiB, MFMA-operand ordered,
 *                                   0.75 B per weight) followed by the group scales blocked the
 *                                   same way (fp16 [N/16][K/128][16]); built once, offline
 *   ws   fp16  [K/128][N]           weight group scales in the reference's W_SCALE layout
 *                                   (test_bgemm_kernel.cu:57-63): an input of the packers only
 *   d    fp16  [M][N]               output, row-major
 * Reference layouts (bit planes, duplicated half2 x-scales) are accepted by the fq_ref_* and
 * fq_import_* entry points.
 */
#ifndef FLEXQ_HIP_H
#define FLEXQ_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t *fq_stream_t; /* == hipStream_t */

/* ABI version.  3: fq_bmma_init takes reference bit-plane W + W_SCALE (the weight-image form is
 * fq_bmma_init_image) and fq_bmma_state carries w_format / prepared; split-K prefill without its
 * workspace returns FQ_ERR_WORKSPACE.  A caller built against another version should compare
 * FQ_ABI_VERSION with fq_abi_version() at start-up. */
#define FQ_ABI_VERSION 6   /* 4: FQ_ERR_TIMEOUT and the host-visible chain status (fq_chain_bind_status);
                              5: fq_chain_bind_status takes the chain workspace's size and zeroes the word,
                                 a timed-out chain writes NaN outputs;
                              6: fq_gemm_w6ax_q / fq_gemm_q_workspace_bytes (the next input's codes from the
                                 decode GEMM's epilogue) */
int fq_abi_version(void);

typedef int fq_status;
#define FQ_OK 0
#define FQ_ERR_NULL 1      /* a required pointer is NULL */
#define FQ_ERR_SHAPE 2     /* M/N/K out of the supported range (K % 128, layout limits) */
#define FQ_ERR_BITS 3      /* unsupported bit width */
#define FQ_ERR_WORKSPACE 4 /* workspace missing or smaller than fq_gemm_workspace_bytes() */
#define FQ_ERR_HIP 5       /* the HIP launch itself failed */
#define FQ_ERR_TIMEOUT 6   /* a decode chain's in-kernel wait timed out earlier on this chain workspace:
                              the results of that launch and of every later one are undefined; nothing
                              was enqueued (fq_chain_reset clears it) */

/* ---- library info ------------------------------------------------------------------------ */
const char *fq_version(void);
const char *fq_status_string(fq_status s);

/* ---- sizes ------------------------------------------------------------------------------- */
/* Bytes of the weight image for an [N][K] matrix (N padded to 16 internally): 1568 B per
 * 16 columns x 128 k (1536 B codes + 32 B scales). */
size_t fq_packed_w_bytes(int N, int K);
/* Bytes of scratch fq_gemm_w6ax / fq_linear_w6ax need for this shape (0 if none).  The buffer
 * must be zero-filled once after allocation (fq_workspace_init).  Layout: a 256 KiB ticket
 * region (split-K decode, M <= 32; the kernels leave it zeroed) followed by the split-K slabs
 * (decode, and prefill at 32 < M < 2048 when its 128 x 128 tiles are too few for the chip) or,
 * for M >= 2048, the unpacked int8 weights of the prefill GEMM (rewritten every call).  One
 * buffer of the largest size may serve every shape on one stream.  A shape that needs split-K
 * slabs returns FQ_ERR_WORKSPACE when the buffer is missing or short (the bits must not depend on
 * the caller's buffer); at M >= 2048 a missing or short one only means the weights are unpacked
 * per workgroup instead of once per call (bit-identical). */
size_t fq_gemm_workspace_bytes(int M, int N, int K);
fq_status fq_workspace_init(void *workspace, size_t bytes, fq_stream_t stream);

/* ---- weight packing (offline) ------------------------------------------------------------- */
/* int8 weight codes [N][K] (values in [-32,31]) + ws [K/128][N] -> weight image.  Replaces
 * flexq_bit_packing(const int*, int*, M, K, BIT, stream) applied to weights
 * (engine/src/pack/bit_packing.h:34, test_bgemm_kernel.cu:222-223); the W_SCALE the reference
 * passes to every GEMM call is folded into the image here, once. */
fq_status fq_pack_w6(const int8_t *wq, const uint16_t *ws, int N, int K, void *w_packed,
                     fq_stream_t stream);
/* Inverse, for checks: image -> int8 [N][K] (+ ws [K/128][N] when ws != NULL). */
fq_status fq_unpack_w6(const void *w_packed, int N, int K, int8_t *wq, uint16_t *ws,
                       fq_stream_t stream);
/* fp16 weight [N][K] -> per-(row,128-group) symmetric 6-bit codes -> image, plus ws [K/128][N].
 * Same rounding rule as fq_quantize_act (the offline converter the reference does not ship,
 * LlamaDecoderLayerWeight.cc:381-410 loads its output). wq_out (int8 [N][K]) is optional. */
fq_status fq_quantize_pack_w6(const uint16_t *w, int N, int K, void *w_packed, uint16_t *ws,
                              int8_t *wq_out, fq_stream_t stream);

/* ---- activation quantization (online) ----------------------------------------------------- */
/* fp16 x [M][K] -> xq int8 [M][K], xs fp16 [K/128][M]: dynamic per-(row,128-group) symmetric
 * quantization with the reference engine's arithmetic (e2e .../flexqgemm/src/pack/
 * bit_packing.cu:125-164): scale = half(absmax / (2^(b-1)-1)), q = clamp(roundf(x/scale)).
 * All-zero groups quantize to 0 (the reference's NaN path).  abits in {6, 8}. */
fq_status fq_quantize_act(const uint16_t *x, int M, int K, int abits, int8_t *xq, uint16_t *xs,
                          fq_stream_t stream);

/* ---- GEMM ------------------------------------------------------------------------------- */
/* d[M][N] = fp16( sum_g float(half(xs[g][m]*ws[g][n])) * acc[m][n][g] ), ws from the image,
 * acc[m][n][g] = sum_{k in g} xq[m][k]*wq[n][k] (exact int32).  Replaces
 * FQBMMAInitFn/FQBMMAExecFn (engine/src/bgemm/flexq_bmma_op.h:163-188) and
 * FLEXQGEMMWrapper::gemm(int* A ...) (e2e .../flexq_gemm_wrapper.cu:21-97).
 * acc_dbg: optional int32 [M][N][K/128] copy of the group accumulators (bit-exact checks).
 * workspace: fq_gemm_workspace_bytes(M,N,K) bytes, initialised once by fq_workspace_init. */
fq_status fq_gemm_w6ax(const int8_t *xq, const uint16_t *xs, const void *w_packed, int M, int N,
                       int K, int abits, uint16_t *d, int32_t *acc_dbg, void *workspace,
                       size_t workspace_bytes, fq_stream_t stream);

/* Quantize + GEMM in one call.  Replaces FLEXQGEMMWrapper::gemm(const half* A ...)
 * (flexq_gemm_wrapper.cu:99-122).  Decode sizes (M <= 32, fq_linear_act_scratch_bytes() == 0)
 * run as ONE launch: the GEMM quantizes its activation groups itself and xq_buf/xs_buf are not
 * touched (may be NULL).  Otherwise xq_buf/xs_buf are caller scratch of M*K bytes and
 * 2*M*(K/128) bytes (the reference's activation workspace, LlamaV2ContextAttentionLayer.cc:793). */
size_t fq_linear_act_scratch_bytes(int M, int N, int K);
fq_status fq_linear_w6ax(const uint16_t *x, int M, int N, int K, int abits, const void *w_packed,
                         uint16_t *d, int8_t *xq_buf, uint16_t *xs_buf, void *workspace,
                         size_t workspace_bytes, fq_stream_t stream);

/* ---- decode chain ------------------------------------------------------------------------------
 * n consecutive linears, each computed as its entry point would in order -- fq_linear_w6ax (pro 0),
 * fq_rmsnorm_linear_w6ax (pro 1), fq_silu_linear_w6ax (pro 2); bit-identical outputs and residual
 * outputs -- where a link's x / in may lie inside the previous link's d and an RMSNorm link's residual
 * may be an earlier RMSNorm link's res_out (a decoder layer's o_proj -> RMSNorm + gate_up -> SiLU * up +
 * down_proj -> RMSNorm + next qkv).  Runs of up to 8 links, the first a plain linear, run as ONE
 * persistent launch when every link's decode plan allows it (M <= 4, N a multiple of 16 and >= 16 x
 * the CU count, x 16-byte aligned; RMSNorm at M = 1, K = 4096) and no output of the run overlaps
 * another output or an input except through those hand-offs: each linear's weight stream starts
 * before it waits, inside the kernel, for its inputs (read from tagged hand-off granules in the chain
 * workspace), not behind a kernel boundary.  Other links run as their entry points
 * (xq_buf / xs_buf as there: only links that do not fuse their quantizer use them; workspace as theirs).
 * chain_ws: the chain workspace, 256-byte aligned, fq_chain_workspace_bytes(links, n, M) bytes (a
 * shorter one runs shorter runs or plain linears), zeroed once by fq_chain_workspace_init and then
 * written by chain launches only (one per stream; it may serve every chain of that stream).
 * A chain launch never hangs: a wait that does not end within ~1 s sets the word at byte offset
 * fq_chain_error_offset() of chain_ws (sticky; results undefined; every later wait on that workspace
 * returns at once) and, when a host status word is bound (fq_chain_bind_status), that word too; every
 * output of a linear whose wait failed (or saw the error word) is written as fp16 NaN, so the undefined
 * results cannot be consumed silently by a caller that does not read the status; from
 * then on fq_linear_chain_w6ax on chain_ws returns FQ_ERR_TIMEOUT without enqueuing anything, until
 * fq_chain_reset (the reference's convention: FQBMMAOp::initialize sets initSuccess = false and the
 * wrapper prints and returns, flexq_bmma_op.h:103-126, flexq_gemm_wrapper.cu:93).
 * Co-residency: every workgroup of a chain launch waits for workgroups of the same launch, so the
 * launch needs all of its workgroups (one per CU) resident at once.  The host checks that the kernel
 * can hold one workgroup per CU (the occupancy query; otherwise the links run as their entry points),
 * but it cannot see CUs held by kernels of other streams or processes: a caller that overlaps other
 * kernels with a chain (concurrent streams, several processes on one GPU) must expect a timeout there,
 * which the status above reports.
 * No FlexQ counterpart: the reference launches one kernel per GEMM call (flexq_gemm_wrapper.cu:99-122). */
typedef struct fq_chain_link {
    const uint16_t *x;     /* fp16 [M][K]; pro 1: the residual; pro 2: the gate (rows of stride ldh) */
    const void *w_packed;  /* weight image [N][K] */
    uint16_t *d;           /* fp16 [M][N] */
    int N, K, abits;
    int pro;               /* 0: fq_linear_w6ax; 1: fq_rmsnorm_linear_w6ax (M = 1, K = 4096 to chain);
                              2: fq_silu_linear_w6ax */
    const uint16_t *in;    /* pro 1: the input added to the residual (or NULL); pro 2: up */
    const uint16_t *gamma; /* pro 1 */
    uint16_t *res_out;     /* pro 1 with in: residual + in */
    float eps;             /* pro 1 */
    int ldh;               /* pro 2: row stride of gate and up */
} fq_chain_link;
fq_status fq_linear_chain_w6ax(const fq_chain_link *links, int n, int M, void *chain_ws, size_t chain_ws_bytes,
                               int8_t *xq_buf, uint16_t *xs_buf, void *workspace, size_t workspace_bytes,
                               fq_stream_t stream);
size_t fq_chain_workspace_bytes(const fq_chain_link *links, int n, int M);
fq_status fq_chain_workspace_init(void *chain_ws, size_t bytes, fq_stream_t stream);
size_t fq_chain_error_offset(void);
/* Host-visible chain status.  host_status (host): a 4-byte word of pinned, device-mapped host memory
 * (hipHostMalloc, or torch's pinned memory), owned by the caller and kept alive with chain_ws (and while
 * any launch on chain_ws may be in flight).  Binding zeroes the word (on the host) and enqueues one small
 * kernel on `stream` that records its device address in chain_ws (call it after fq_chain_workspace_init).
 * FQ_ERR_NULL when host_status is not device-mapped; FQ_ERR_WORKSPACE when chain_ws is not 256-byte
 * aligned or chain_ws_bytes is below the chain's sync area (4096 bytes; the word's address lives there). */
fq_status fq_chain_bind_status(void *chain_ws, size_t chain_ws_bytes, uint32_t *host_status, fq_stream_t stream);
/* FQ_ERR_TIMEOUT once a wait on chain_ws timed out (the bound word, read on the host: no
 * synchronisation, so a timeout shows once the launch that hit it has finished); FQ_OK otherwise,
 * also for a workspace without a bound word.  A captured graph's replays do not pass through
 * fq_linear_chain_w6ax: read this after synchronising with the replays. */
fq_status fq_chain_status(const void *chain_ws);
/* Clear a timed-out chain workspace: re-zero its `bytes` (stream-ordered), re-bind its host word and
 * clear it.  No chain launch on chain_ws may be in flight (synchronise first). */
fq_status fq_chain_reset(void *chain_ws, size_t bytes, fq_stream_t stream);

/* ---- prefill with resident unpacked weights ------------------------------------------------------
 * At M >= 2048 fq_gemm_w6ax unpacks the weight image into int8 MFMA operands in its workspace on
 * every call (fq_unpack_w8_kernel: 0.75 B read + 1 B written per weight).  A caller that keeps the
 * unpacked operands for the model's lifetime (1 byte per weight) skips that pass:
 * fq_prefill_unpack_weights writes them once (w_u8 of fq_prefill_weight_bytes(N, K) bytes, 256-byte
 * aligned) and fq_gemm_w6ax_u8 runs the prefill GEMM over them -- bit-identical to fq_gemm_w6ax; below
 * M = 2048 it IS fq_gemm_w6ax (those plans do not read unpacked operands).  The reference has no
 * prefill kernel (its BLOCK_M <= 8 tiles re-stream W, flexq_bmma_op.h:111-114). */
size_t fq_prefill_weight_bytes(int N, int K);
fq_status fq_prefill_unpack_weights(const void *w_packed, int N, int K, void *w_u8, fq_stream_t stream);
fq_status fq_gemm_w6ax_u8(const int8_t *xq, const uint16_t *xs, const void *w_packed, const void *w_u8, int M,
                          int N, int K, int abits, uint16_t *d, int32_t *acc_dbg, void *workspace,
                          size_t workspace_bytes, fq_stream_t stream);
/* fq_gemm_w6ax_u8 that also emits the NEXT linear's quantized input: d's leading qM * qK values,
 * read row-major as a [qM][qK] activation (qK % 128 == 0, qM * qK <= M * N), quantized to qbits
 * into qxq (int8 [qM][qK]) and qxs (fp16 [qK/128][qM]) -- bit-identical to
 * fq_quantize_act(d, qM, qK, qbits, qxq, qxs) after the GEMM; qxq and qxs may not overlap xq, xs, d
 * or each other (FQ_ERR_SHAPE).  With N % 128 == 0 on the 256 x 256
 * prefill tiles it runs in the GEMM's epilogue (a tile row holds two whole 128-column groups), so no
 * separate quantize pass reads d back; otherwise it is the GEMM, then fq_quantize_act.  The reference
 * quantizes every GEMM input in its own packing kernel (flexq_gemm_wrapper.cu:99-122). */
fq_status fq_gemm_w6ax_u8_q(const int8_t *xq, const uint16_t *xs, const void *w_packed, const void *w_u8, int M,
                            int N, int K, int abits, uint16_t *d, int8_t *qxq, uint16_t *qxs, int qM, int qK,
                            int qbits, void *workspace, size_t workspace_bytes, fq_stream_t stream);
/* The same at any M without prepared operands: fq_gemm_w6ax, then the next input's codes -- bit-identical
 * to fq_quantize_act(d, qM, qK, qbits, qxq, qxs) after the GEMM; the same argument rules (FQ_ERR_SHAPE on
 * an overlap).  At M <= 16 with N % 128 == 0 and no k-split the quantizer runs in the decode GEMM's
 * epilogue: every workgroup stores its 16-column tiles write-through, takes one agent-scope ticket per
 * 128-column group, and the group's last workgroup re-loads its M x 128 outputs and quantizes them (one
 * launch instead of two; the reference quantizes every input in its own packing kernel,
 * flexq_gemm_wrapper.cu:99-122).  That form needs a workspace of fq_gemm_q_workspace_bytes(M, N, K)
 * bytes, initialised once by fq_workspace_init (its tickets return to zero after every launch); with a
 * shorter one the call runs the two-launch form (same bits).  fq_gemm_w6ax_u8_q below M = 2048 is this. */
size_t fq_gemm_q_workspace_bytes(int M, int N, int K);
fq_status fq_gemm_w6ax_q(const int8_t *xq, const uint16_t *xs, const void *w_packed, int M, int N, int K,
                         int abits, uint16_t *d, int8_t *qxq, uint16_t *qxs, int qM, int qK, int qbits,
                         void *workspace, size_t workspace_bytes, fq_stream_t stream);

/* ---- fused producers of the activation codes ---------------------------- */
/* Residual add + RMSNorm (T5 / LLaMA style: no mean, no bias) + dynamic group quantization, one
 * launch.  Replaces generalAddResidualT5LayerNormFlexQFusion / invokeGeneralAddResidualT5PreLayerNorm
 * (e2e .../kernels/layernorm_kernels.cu:1851-2106) with this engine's activation format:
 *   residual[m][k] = half_clamp(float(input[m][k]) + float(residual[m][k]))   (in place; input
 *                    may be NULL: no add, the residual is only read)
 *   normed[m][k]   = half_clamp((float(residual[m][k]) * rs[m]) * float(gamma[k])),
 *                    rs[m] = 1 / sqrt(sum_k float(residual[m][k])^2 / K + eps)
 *   xq, xs         = fq_quantize_act(normed, abits)     (bit-identical codes and scales)
 * half_clamp = the reference's clamp_inf_for_half (+-64504, then fp16).  normed_out (fp16
 * [M][K]) is optional.  K % 128 == 0, K <= 32768, 16-byte aligned rows. */
fq_status fq_rmsnorm_quantize(const uint16_t *input, uint16_t *residual, const uint16_t *gamma,
                              float eps, int M, int K, int abits, int8_t *xq, uint16_t *xs,
                              uint16_t *normed_out, fq_stream_t stream);
/* SiLU(gate) * up + dynamic group quantization, one launch.  Replaces flexq_generic_activation
 * (e2e .../kernels/activation_kernels.cu:245-450, launch :556-590; A8 for down_proj,
 * FfnLayer.cc:67-77):  act[m][n] = half(silu(float(gate[m][n])) * float(up[m][n])),
 * silu(v) = v / (1 + exp(-v)); gate and up rows have stride ld (elements), e.g. the two halves of
 * a merged [gate | up] output with ld = 2N.  xq int8 [M][N], xs fp16 [N/128][M], act_out
 * (fp16 [M][N]) optional.  N % 128 == 0, 16-byte aligned rows. */
fq_status fq_silu_mul_quantize(const uint16_t *gate, const uint16_t *up, int ld, int M, int N,
                               int abits, int8_t *xq, uint16_t *xs, uint16_t *act_out,
                               fq_stream_t stream);
/* OPT-family residual + bias + LayerNorm (mean and variance, gamma, beta) + dynamic group
 * quantization, one launch.  Replaces generalAddBiasResidualLayerNormOpt2FlexQFusion
 * (e2e .../kernels/layernorm_kernels.cu:316-575) and its pre-attention form
 * invokeGeneralLayerNorm (:2325-2420: residual only):
 *   v[m][k]        = ((0 + float(bias[k])) + float(residual[m][k])) + float(input[m][k])   (fp32;
 *                    bias and input may be NULL: skipped)
 *   res_out[m][k]  = half(v)            (optional; may be the residual itself, nothing else it reads)
 *   mean, rs       = (s / (K/2)) / 2,  1 / sqrt(((q / (K/2)) / 2 - mean^2) + eps), s and q the
 *                    row's fp32 sums of v and v^2 over half2 pairs (the build's fixed order)
 *   normed[m][k]   = ((half(v) - half(mean)) * half(rs)) * gamma[k] [+ beta[k]], fp16 operations
 *   xq, xs         = fq_quantize_act(normed, abits)
 * normed_out optional.  K % 128 == 0, K <= 32768, 16-byte aligned rows. */
fq_status fq_layernorm_quantize(const uint16_t *input, const uint16_t *residual, const uint16_t *bias,
                                uint16_t *res_out, const uint16_t *gamma, const uint16_t *beta,
                                float eps, int M, int K, int abits, int8_t *xq, uint16_t *xs,
                                uint16_t *normed_out, fq_stream_t stream);

/* ---- producer + linear in one call: the decoder layer's three W6Ax linears that follow a producer
 * (qkv and gate_up after the add-residual RMSNorm, down_proj after SiLU * up).  At decode sizes the
 * producer runs inside the decode GEMM's prologue -- one launch instead of two: RMSNorm when
 * M == 1 and K == 4096 (each of the 8 waves normalises and quantizes 4 of the 32 groups, the
 * 512-thread producer's chunking), SiLU * up whenever fq_linear_w6ax would fuse its quantizer.
 * Otherwise the producer kernel writes xq_buf / xs_buf (the *_scratch_bytes below) and the GEMM
 * follows.  Outputs are bit-identical to fq_rmsnorm_quantize / fq_silu_mul_quantize followed by
 * fq_gemm_w6ax, both ways.
 * fq_rmsnorm_linear_w6ax: d = linear(RMSNorm(residual + input) codes); with input != NULL,
 *   residual_out (NOT the residual itself: other workgroups are still reading it) receives
 *   residual + input; with input == NULL the residual is only read.  Replaces the reference's
 *   generalAddResidualT5LayerNormFlexQFusion + FLEXQGEMMWrapper::gemm pair
 *   (LlamaContextDecoder.cc:576-592 then FfnLayer.cc:440-452).
 * fq_silu_linear_w6ax: d = linear(codes of silu(gate) * up), gate / up rows of stride ld, K the
 *   activation width (down_proj's input).  Replaces flexq_generic_activation + the down_proj GEMM
 *   (FfnLayer.cc:521-558). */
size_t fq_rmsnorm_linear_scratch_bytes(int M, int N, int K); /* M*K + 2*M*(K/128), or 0: fused */
size_t fq_silu_linear_scratch_bytes(int M, int N, int K);
fq_status fq_rmsnorm_linear_w6ax(const uint16_t *input, const uint16_t *residual, uint16_t *residual_out,
                                 const uint16_t *gamma, float eps, int M, int N, int K, int abits,
                                 const void *w_packed, uint16_t *d, int8_t *xq_buf, uint16_t *xs_buf,
                                 void *workspace, size_t workspace_bytes, fq_stream_t stream);
fq_status fq_silu_linear_w6ax(const uint16_t *gate, const uint16_t *up, int ld, int M, int N, int K,
                              int abits, const void *w_packed, uint16_t *d, int8_t *xq_buf,
                              uint16_t *xs_buf, void *workspace, size_t workspace_bytes,
                              fq_stream_t stream);
/* fq_layernorm_linear_w6ax: d = linear(codes of LayerNorm(residual [+ input] [+ bias])), the OPT
 *   decoder's LayerNorm -> qkv / fc1 pair (generalAddBiasResidualLayerNormOpt2FlexQFusion, then
 *   FLEXQGEMMWrapper::gemm).  One launch when M == 1 and K == 4096 (the RMSNorm form's chunking);
 *   otherwise fq_layernorm_quantize into xq_buf / xs_buf, then the GEMM.  residual_out (may be NULL)
 *   receives half(v); in the one-launch form it must not be the residual (other workgroups still
 *   read it) and must not overlap any input.  Bit-identical to fq_layernorm_quantize + fq_gemm_w6ax. */
size_t fq_layernorm_linear_scratch_bytes(int M, int N, int K);
fq_status fq_layernorm_linear_w6ax(const uint16_t *input, const uint16_t *residual, const uint16_t *bias,
                                   uint16_t *residual_out, const uint16_t *gamma, const uint16_t *beta,
                                   float eps, int M, int N, int K, int abits, const void *w_packed,
                                   uint16_t *d, int8_t *xq_buf, uint16_t *xs_buf, void *workspace,
                                   size_t workspace_bytes, fq_stream_t stream);

/* ---- column-parallel decode with the all-gather in the GEMM epilogue -------
 * The north-star N-shard: rank p of P holds columns [col0, col0 + N) of a linear whose full width is
 * ld.  fq_linear_w6ax_gather computes this rank's columns exactly as fq_linear_w6ax does and stores
 * them straight into EVERY rank's gather buffer out[q] (fp16 [M][ld], IPC-mapped device pointers:
 * xGMI peer stores on a node), with system-scope write-through stores; after the launch's last
 * workgroup has seen every store drained it raises flags[q][rank] = *gen + 1 in every rank.
 * The last workgroup also advances *gen to that value; fq_gather_wait (one small launch) then waits
 * for all P flags of this rank and acquires: after it, out[rank] holds the whole [M][ld] output.  This replaces the per-linear RCCL
 * all_gather (nccl_utils.cc:70-82's ftNcclAllGather in the reference) at decode sizes.
 * Use two gather buffers alternately (linear j writes buffer j % 2): a rank can then run at most
 * one linear ahead of any other without overwriting an input still being read.  The struct lives
 * in device memory; done and gen are this rank's own words, zeroed once.  The wait is bounded
 * (~1 s): on timeout *err is set to 1 and the results are undefined (never a hang); while *err is
 * set, fq_gather_wait returns at once.
 * M <= 32, N % 16 == 0, P <= FQ_GATHER_MAX_RANKS. */
#define FQ_GATHER_MAX_RANKS 8
typedef struct fq_gather {
    uint16_t *out[FQ_GATHER_MAX_RANKS];   /* rank q's gather buffer, fp16 [M][ld] */
    uint32_t *flags[FQ_GATHER_MAX_RANKS]; /* rank q's flag words, uint32 [P] */
    uint32_t *done;                       /* this rank's launch ticket */
    uint32_t *gen;                        /* this rank's generation */
    int P, rank, col0, ld;
} fq_gather;
fq_status fq_linear_w6ax_gather(const uint16_t *x, int M, int N, int K, int abits, const void *w_packed,
                                const fq_gather *gather, int8_t *xq_buf, uint16_t *xs_buf, void *workspace,
                                size_t workspace_bytes, fq_stream_t stream);
fq_status fq_gather_wait(const fq_gather *gather, uint32_t *err, fq_stream_t stream);
/* fq_linear_w6ax_gather whose input x is the output of in_gather (this rank's gather buffer of the
 * previous linear), with that gather's wait folded into the launch: the kernel issues its weight
 * DMAs, then one wave polls in_gather's flags (system-scope loads; bounded like fq_gather_wait, err
 * = in_gather's error word) and the activation is read after the poll.  Requires the gather buffers
 * and flags in uncached device memory (hipExtMallocWithFlags(hipDeviceMallocUncached): no acquire
 * fence, so no stale cache line may serve the reads).  One launch where fq_linear_w6ax would fuse its
 * quantizer; otherwise fq_gather_wait(in_gather) then fq_linear_w6ax_gather.  Bit-identical to the
 * two-call form.  The generation advances at each publish, so either wait form may follow any call. */
fq_status fq_linear_w6ax_gather_after(const uint16_t *x, const fq_gather *in_gather, uint32_t *err, int M, int N,
                                      int K, int abits, const void *w_packed, const fq_gather *gather,
                                      int8_t *xq_buf, uint16_t *xs_buf, void *workspace, size_t workspace_bytes,
                                      fq_stream_t stream);

/* ---- reference-layout entry points (drop-in for FlexQ's own formats) ------------------------ */
/* flexq_bit_packing(const int* in, int* out, M, K, BIT, stream) (engine/src/pack/bit_packing.h:34,
 * bit_packing.cu:147-156): raw b-bit patterns [M][K] -> bit planes int32
 * [K/128][M/c][BIT][c][4], c = min(M,8), k0 at bit 31.  M must be <= 8 or a multiple of 8. */
fq_status fq_ref_bit_packing(const int32_t *in, int32_t *packed, int M, int K, int bits,
                             fq_stream_t stream);
/* flexq_bit_packing(const half* in, int* out, half* x_scale, M, K, BIT, stream)
 * (e2e .../flexqgemm/src/pack/bit_packing.h:32-34, FLEXQGEMMWrapper::pack): quantize + bit-plane
 * pack; x_scale_dup is the reference layout half[K/128][2*ceil4(M)] of duplicated pairs. */
fq_status fq_ref_quantize_bit_packing(const uint16_t *x, int32_t *packed, uint16_t *x_scale_dup,
                                      int M, int K, int bits, fq_stream_t stream);
/* Reference bit-plane weights (W_BITS = 6, [K/128][N/c][6][c][4]) + W_SCALE [K/128][N] ->
 * weight image. */
fq_status fq_import_ref_w(const int32_t *w_bitplanes, const uint16_t *w_scale, int N, int K,
                          void *w_packed, fq_stream_t stream);
/* Reference bit-plane activations + duplicated scales -> xq int8 [M][K] + xs [K/128][M]. */
fq_status fq_import_ref_x(const int32_t *x_bitplanes, const uint16_t *x_scale_dup, int M, int K,
                          int bits, int8_t *xq, uint16_t *xs, fq_stream_t stream);
/* GEMM straight from the reference's bit-plane activations: the X / X_SCALE operands of
 * FQBMMAExecFn_t (flexq_bmma_op.h:187-188) and of FLEXQGEMMWrapper::gemm(const int* A ...)
 * (flexq_gemm_wrapper.cu:21-97; FT's decoder attention calls it with the packed output of its
 * fused RMSNorm, LlamaV2DecoderSelfAttentionLayer.cc:653).  At decode sizes (on the LLaMA shapes M = 1, 2
 * and M = 4 at K = 4096) the planes are unpacked inside the GEMM's prologue: ONE launch, no
 * scratch.  Otherwise fq_import_ref_x writes xq_buf / xs_buf (fq_planes_act_scratch_bytes: M*K
 * bytes of codes + 2*M*(K/128) of scales, 0 when fused) and fq_gemm_w6ax follows.  Output
 * bit-identical to fq_import_ref_x + fq_gemm_w6ax.  M <= 8 or M % 8 == 0 (the plane layout);
 * workspace as for fq_gemm_w6ax. */
size_t fq_planes_act_scratch_bytes(int M, int N, int K);
fq_status fq_gemm_w6ax_planes(const int32_t *x_bitplanes, const uint16_t *x_scale_dup, const void *w_packed,
                              int M, int N, int K, int bits, uint16_t *d, int8_t *xq_buf, uint16_t *xs_buf,
                              void *workspace, size_t workspace_bytes, fq_stream_t stream);

/* FQBMMAOpState-style two-call interface (flexq_bmma_op.h:19-34, FQBMMAInitFn_t / FQBMMAExecFn_t
 * at :187-188): init validates and records the arguments -- no launch, and no device-attribute
 * call per init (unlike flexq_bmma_op.h:103) -- and exec runs the GEMM.
 *
 * fq_bmma_init takes the REFERENCE operands: X and W as bit planes (fq_ref_bit_packing layout,
 * W_BITS = 6) with X_SCALE in the reference's duplicated layout and W_SCALE half[K/128][N]
 * (required).  The first fq_bmma_exec on a state zeroes the scratch's ticket region and imports
 * W + W_SCALE into a weight image inside `scratch` (once: FT loads its weights once, and
 * `prepared` records it; set it back to 0 after rewriting W); every exec runs
 * fq_gemm_w6ax_planes on X's bit planes (decode sizes: one launch, the planes unpacked inside the
 * GEMM; otherwise imported into the scratch first).  Run the first exec eagerly before capturing
 * a graph.
 * fq_bmma_init_image is the fast path for callers that keep the weight image (fq_import_ref_w /
 * fq_pack_w6 output) themselves: no W_SCALE, no image in scratch.  A caller cannot pass one form
 * for the other by accident: the two entry points name the form.
 * Rejections (init_success = 0, like FQBMMAOp::initialize): NULL operands, group_size != 128,
 * bias, K % 128, W_BITS != 6, X_BITS not 6/8, bit-plane rows (M, and N for bit-plane W) neither
 * <= 8 nor a multiple of 8, scratch smaller than fq_bmma_scratch_bytes / _image_scratch_bytes.
 * The caller's scratch needs no initialisation. */
#define FQ_W_BITPLANES 0 /* reference bit planes + W_SCALE */
#define FQ_W_IMAGE 1     /* this build's weight image */
typedef struct fq_bmma_state {
    int init_success;
    int M, N, K, x_bits, w_bits, group_size;
    int w_format;            /* FQ_W_BITPLANES or FQ_W_IMAGE */
    int prepared;            /* set by the first exec: tickets zeroed, W imported */
    const int32_t *X;        /* reference bit-plane activations */
    const void *W;           /* bit planes (FQ_W_BITPLANES) or a weight image (FQ_W_IMAGE) */
    const uint16_t *X_SCALE; /* reference duplicated layout half[K/128][2*ceil4(M)] */
    const uint16_t *W_SCALE; /* half[K/128][N] (FQ_W_BITPLANES) */
    uint16_t *D;             /* half[M][N] */
    void *scratch;
    size_t scratch_bytes;
} fq_bmma_state;
size_t fq_bmma_scratch_bytes(int M, int N, int K);
size_t fq_bmma_image_scratch_bytes(int M, int N, int K);
fq_bmma_state fq_bmma_init(const int32_t *X, const int32_t *W, const uint16_t *X_SCALE,
                           const uint16_t *W_SCALE, int M, int N, int K, uint16_t *D,
                           int group_size, int bias, int x_bits, int w_bits, void *scratch,
                           size_t scratch_bytes);
fq_bmma_state fq_bmma_init_image(const int32_t *X, const void *W_image, const uint16_t *X_SCALE,
                                 int M, int N, int K, uint16_t *D, int group_size, int bias,
                                 int x_bits, int w_bits, void *scratch, size_t scratch_bytes);
/* FQBMMAExecFn_t(FQBMMAOpState&, stream): the state is updated (prepared) on the first call. */
fq_status fq_bmma_exec(fq_bmma_state *state, fq_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* FLEXQ_HIP_H */
