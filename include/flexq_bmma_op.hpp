/*
 * flexq_bmma_op.hpp -- C++ drop-in for FlexQ's FQBMMA function-pointer interface
 * (e2e/src/fastertransformer/kernels/flexqgemm/src/bgemm/flexq_bmma_op.h:19-34,159-184 and the
 * instance declarations of flexq_bmma_library.h) over this build's engine (libflexq_hip.so).
 *
 * A caller written against the reference -- FasterTransformer's FLEXQGEMMWrapper::gemm
 * (flexq_gemm_wrapper.cu:21-97) picks an instance by name, calls `state = (*init_fn)(...)` and then
 * `(*exec_fn)(state, stream)` -- compiles unchanged against this header (hipStream_t for
 * cudaStream_t) and links against libflexq_hip.so:
 *
 *   FQBMMAOpState                 the reference's struct, member for member
 *   FQBMMAInitFn_t / ExecFn_t     the reference's typedefs (the e2e, const-qualified form)
 *   FQBMMA_<X>x6xtrue_..._InitFn  the eight instances the reference wrapper names (W6A6 and W6A8,
 *   FQBMMA_<X>x6xtrue_..._ExecFn  M = 1, 2, 4 and the general one); every instance runs this
 *                                 build's own M-bucket dispatch, so the tile names are only names
 *
 * Operands are the reference's: X = bit-plane activations (fq_ref_bit_packing / pack() layout),
 * X_SCALE = duplicated half2 scales half[K/128][2*ceil4(M)], W = bit-plane weights (W_BITS = 6),
 * W_SCALE = half[K/128][N], D = half[M][N].
 *
 * init validates like FQBMMAOp::initialize (flexq_bmma_op.h:81-133; plus group_size == 128,
 * bias == false, K % 128 == 0 and the bit-plane row rule: M, N <= 8 or multiples of 8) and records
 * the arguments -- no allocation, no launch, no device-attribute call.  gridDim / blockDim /
 * shared_mem_size describe this build's decode grid (informational; exec does the launching).
 *
 * exec is stream-ordered and never synchronises.  Its first call for a given (W, W_SCALE, N, K)
 * imports the weights into a weight image in library-owned device memory (fq_import_ref_w, once:
 * FT loads its weights once), and its first call on a stream allocates that stream's scratch (the
 * int8 activation codes, x-scales and the GEMM workspace; grown geometrically). Neither is ever
 * freed while the process runs, so a HIP graph captured around exec stays valid; run one exec of
 * each shape eagerly before capturing.  After rewriting the weights behind a W pointer, call
 * fq_bmma_op_forget_weight(W) (the old image is retired, not freed).  Errors are printed as
 * "[FlexQ][Error] ..." and exec returns, as the reference's wrapper does (.cu:44,88,93).
 */
#pragma once

#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include "flexq_hip.h"

struct FQBMMAOpState {
    size_t shared_mem_size;
    dim3 gridDim;
    dim3 blockDim;
    bool initSuccess = false;
    struct Argument_t {
        int M, N, K;
        const int *X;
        const int *W;
        half *X_SCALE;
        const half *W_SCALE;
        half *D;
        int group_size;
        bool bias = false;
    } args;
};

typedef FQBMMAOpState (*FQBMMAInitFn_t)(const int *, const int *, half *, const half *, int, int, int, half *, int, bool);
typedef void (*FQBMMAExecFn_t)(FQBMMAOpState &, hipStream_t);

/* the reference's instance names (FQ_NAME_FUN, common/base.h:286-289) */
#define FQ_AMD_DECL_INSTANCE(name)          \
    extern FQBMMAInitFn_t name##_InitFn;    \
    extern FQBMMAExecFn_t name##_ExecFn;
FQ_AMD_DECL_INSTANCE(FQBMMA_6x6xtrue_1x32x256_8x48x128_8x8x128_2_1)
FQ_AMD_DECL_INSTANCE(FQBMMA_6x6xtrue_2x32x512_16x48x128_8x8x128_2_1)
FQ_AMD_DECL_INSTANCE(FQBMMA_6x6xtrue_4x32x512_24x48x128_8x8x128_2_1)
FQ_AMD_DECL_INSTANCE(FQBMMA_6x6xtrue_8x16x256_48x48x128_8x8x128_4_1)
FQ_AMD_DECL_INSTANCE(FQBMMA_8x6xtrue_1x32x256_8x48x128_8x8x128_4_1)
FQ_AMD_DECL_INSTANCE(FQBMMA_8x6xtrue_2x32x256_16x48x128_8x8x128_4_1)
FQ_AMD_DECL_INSTANCE(FQBMMA_8x6xtrue_4x64x256_32x48x128_8x8x128_4_1)
FQ_AMD_DECL_INSTANCE(FQBMMA_8x6xtrue_8x64x384_64x48x128_8x8x128_2_1)
#undef FQ_AMD_DECL_INSTANCE

extern "C" {
/* Drop the library's weight image bound to the bit-plane pointer W (all shapes); the image is
 * retired, not freed, since a captured graph may still read it.  Returns the entries dropped. */
int fq_bmma_op_forget_weight(const void *W);
/* Device bytes the FQBMMA instances hold (weight images + per-stream scratch, retired included). */
size_t fq_bmma_op_device_bytes(void);
}
