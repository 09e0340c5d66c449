/*
 * flexq_gemm_wrapper.hpp -- header-only C++ drop-in for FlexQ's FLEXQGEMMWrapper
 * (e2e/src/fastertransformer/kernels/flexqgemm/flexq_gemm_wrapper.h:6-48, .cu:9-122) over the C ABI
 * of include/flexq_hip.h.  A FasterTransformer layer that holds a FLEXQGEMMWrapper
 * (FfnLayer.cc:371-401, LlamaV2ContextAttentionLayer.cc:145-161) switches by changing the include
 * and the namespace; the member signatures are the reference's, with hipStream_t for cudaStream_t.
 *
 *   FLEXQGEMMWrapper(X_BITS, W_BITS, SIGNED)  W6 with A6 or A8, SIGNED = true (the instantiated
 *                                             families, flexq_bmma_library.cu:23-497)
 *   pack(in, packed, x_scale, M, K, BIT, s)   = flexq_bit_packing(const half*...): quantize + bit
 *                                             planes + duplicated x-scales (fq_ref_quantize_bit_packing)
 *   gemm(M, N, K, const int* A, B, ...)       A = bit-plane activations from pack(), x_scale their
 *                                             duplicated scales; B = bit-plane weights (W_BITS = 6),
 *                                             w_scale = half[K/128][N] passed as float* (the
 *                                             reference reinterprets it the same way, .cu:37-38)
 *   gemm(M, N, K, const half* A, B, ...)      quantize + GEMM; at decode sizes ONE launch
 *                                             (fq_linear_w6ax), x_scale is not written
 *
 * Differences, all host-side:
 *   - B is imported into this build's weight image once per distinct B pointer (the image carries
 *     W_SCALE), into device memory the wrapper owns and frees in its destructor; FT's weights are
 *     loaded once and never rewritten.  set_weight_image(B, image) binds a caller-owned image
 *     instead (no allocation), forget_weight(B) drops a binding after B is rewritten.
 *   - flexq_gemm_workspace is never required and never touched: FT's callers pass 6*M*maxK/8 bytes
 *     (LlamaV2ContextAttentionLayer.cc:793, DecoderSelfAttentionLayer.cc:228) or nullptr and 0 (the
 *     int path, FfnLayer.cc:371-401,521-561); both are accepted unchanged.  The activation codes
 *     (int8, M*K bytes: more than the 6*M*K/8 bit planes the reference's pack() writes there), their
 *     scales, the split-K tickets / slabs and the prefill unpack buffer live in ONE wrapper-owned
 *     device scratch, zeroed on allocation and grown geometrically (x1.5, 1 MiB granules) so that a
 *     rising sequence of shapes allocates O(log) times; superseded buffers are kept until
 *     release_retired() or destruction, so a captured graph never addresses freed memory.
 *   - gemm(const half* A ...) does not write x_scale.  The reference's half path writes the
 *     duplicated x-scales there as a side effect of its internal pack() (.cu:118); this build keeps
 *     them in its scratch (or, at decode sizes, never leaves the GEMM's LDS).  No FT caller reads
 *     x_scale after the call; call pack() when the bit planes and x_scale are wanted.
 *   - C (bias), scale_inter and scale_out are unused, as in the reference (bias = true is rejected
 *     by FQBMMAOp::initialize, flexq_bmma_op.h:103-126).
 * Errors are printed as "[FlexQ][Error] ..." and the call returns, like the reference
 * (.cu:44,88,93); status() holds the last fq_status for callers that want to check.
 */
#pragma once

#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <unordered_map>
#include <vector>

#include "flexq_hip.h"

namespace flexq_amd {

class FLEXQGEMMWrapper {
  public:
    FLEXQGEMMWrapper(int X_BITS, int W_BITS, bool SIGNED) : x_bits_(X_BITS), w_bits_(W_BITS), signed_(SIGNED) {}
    ~FLEXQGEMMWrapper() {
        for (auto &kv : images_)
            if (kv.second.owned) (void)hipFree(kv.second.ptr);
        if (scratch_) (void)hipFree(scratch_);
        release_retired();
    }
    FLEXQGEMMWrapper(const FLEXQGEMMWrapper &) = delete;
    FLEXQGEMMWrapper &operator=(const FLEXQGEMMWrapper &) = delete;

    /* caller workspace (flexq_gemm_workspace) gemm() needs: none.  Whatever the caller passes
     * (FT: 6*M*maxK/8 bytes, or nullptr and 0) is accepted and left untouched. */
    static size_t workspace_bytes(int M, int N, int K) {
        (void)M, (void)N, (void)K;
        return 0;
    }

    void pack(const half *in_data, int *packed_data, half *x_scale, int M, int K, int BIT, hipStream_t stream) {
        report(fq_ref_quantize_bit_packing(reinterpret_cast<const uint16_t *>(in_data), packed_data,
                                           reinterpret_cast<uint16_t *>(x_scale), M, K, BIT, (fq_stream_t)stream),
               "pack");
    }

    void gemm(const int M, const int N, const int K, const int *A, const int *B, const half *C, half *D,
              float *x_scale, const float *w_scale, const float *scale_inter, const float *scale_out, bool bias,
              char *flexq_gemm_workspace, size_t flexq_gemm_ws_bytes, hipStream_t stream = nullptr) {
        (void)C, (void)scale_inter, (void)scale_out, (void)flexq_gemm_workspace, (void)flexq_gemm_ws_bytes;
        if (!check(M, N, K, bias)) return;
        const void *img = image_for(B, reinterpret_cast<const uint16_t *>(w_scale), N, K, stream);
        if (!img) return;
        Scratch sc;
        if (!scratch(M, N, K, stream, &sc)) return;
        // decode sizes: the planes are unpacked inside the GEMM (one launch); otherwise imported
        // into the wrapper's scratch first
        report(fq_gemm_w6ax_planes(A, reinterpret_cast<const uint16_t *>(x_scale), img, M, N, K, x_bits_,
                                   reinterpret_cast<uint16_t *>(D), sc.xq, sc.xs, sc.ws, sc.ws_bytes,
                                   (fq_stream_t)stream),
               "gemm");
    }

    void gemm(const int M, const int N, const int K, const half *A, const int *B, const half *C, half *D,
              float *x_scale, const float *w_scale, const float *scale_inter, const float *scale_out, bool bias,
              char *flexq_gemm_workspace, size_t flexq_gemm_ws_bytes, hipStream_t stream = nullptr) {
        (void)C, (void)x_scale, (void)scale_inter, (void)scale_out, (void)flexq_gemm_workspace, (void)flexq_gemm_ws_bytes;
        if (!check(M, N, K, bias)) return;
        const void *img = image_for(B, reinterpret_cast<const uint16_t *>(w_scale), N, K, stream);
        if (!img) return;
        Scratch sc;
        if (!scratch(M, N, K, stream, &sc)) return;
        report(fq_linear_w6ax(reinterpret_cast<const uint16_t *>(A), M, N, K, x_bits_, img,
                              reinterpret_cast<uint16_t *>(D), sc.xq, sc.xs, sc.ws, sc.ws_bytes, (fq_stream_t)stream),
               "gemm");
    }

    /* bind a caller-owned weight image (fq_import_ref_w / fq_pack_w6 output) to the pointer B */
    void set_weight_image(const int *B, const void *image) { images_[B] = Image{const_cast<void *>(image), false}; }
    void forget_weight(const int *B) {
        auto it = images_.find(B);
        if (it == images_.end()) return;
        if (it->second.owned) retired_.push_back(it->second.ptr);  // a graph may still read it
        images_.erase(it);
    }
    fq_status status() const { return last_; }

  private:
    struct Image {
        void *ptr;
        bool owned;
    };
    static size_t align(size_t v) { return (v + 255) & ~(size_t)255; }

    bool report(fq_status s, const char *what) {
        last_ = s;
        if (s != FQ_OK) fprintf(stderr, "[FlexQ][Error] %s: %s\n", what, fq_status_string(s));
        return s == FQ_OK;
    }

    bool check(int M, int N, int K, bool bias) {
        if (K < 128 || K % 128 != 0) return report(FQ_ERR_SHAPE, "unsupported K");  // .cu:43-46
        if (w_bits_ != 6 || (x_bits_ != 6 && x_bits_ != 8) || !signed_) return report(FQ_ERR_BITS, "unsupported w/a bits");
        if (M <= 0 || N <= 0) return report(FQ_ERR_SHAPE, "unsupported M/N");
        if (bias) return report(FQ_ERR_SHAPE, "bias is not supported (FQBMMAOp::initialize)");
        return true;
    }

    static bool capturing(hipStream_t stream) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        return !(hipStreamIsCapturing(stream, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone);
    }

    /* an import (or a scratch zeroing) enqueued inside a graph capture would run only when the graph
     * replays, so an eager call before that would read an unfilled image: the first use of a weight
     * and scratch growth are refused while the stream captures (make the first call eagerly) */
    const void *image_for(const int *B, const uint16_t *w_scale, int N, int K, hipStream_t stream) {
        auto it = images_.find(B);
        if (it != images_.end()) return it->second.ptr;
        if (capturing(stream)) {
            report(FQ_ERR_HIP, "first use of a weight inside a graph capture (make the first call eagerly)");
            return nullptr;
        }
        void *img = nullptr;
        if (hipMalloc(&img, fq_packed_w_bytes(N, K)) != hipSuccess) {
            report(FQ_ERR_HIP, "weight image allocation");
            return nullptr;
        }
        if (!report(fq_import_ref_w(B, w_scale, N, K, img, (fq_stream_t)stream), "weight import")) {
            (void)hipFree(img);
            return nullptr;
        }
        images_[B] = Image{img, true};
        return img;
    }

    struct Scratch {
        void *ws;
        size_t ws_bytes;
        int8_t *xq;
        uint16_t *xs;
    };
    /* [GEMM workspace: at least the ticket region | xq int8 [M][K] | xs fp16 [K/128][M]]; the ticket
     * region is always reserved at the head, so the codes of a shape without split-K never land on
     * tickets a later split-K shape expects zeroed */
    static size_t ws_region(int M, int N, int K) {
        const size_t need = fq_gemm_workspace_bytes(M, N, K), tickets = 256 * 1024;
        return align(need > tickets ? need : tickets);
    }
    bool scratch(int M, int N, int K, hipStream_t stream, Scratch *out) {
        const size_t wsr = ws_region(M, N, K);
        const size_t need = wsr + align((size_t)M * K) + align((size_t)M * (K / 128) * 2);
        if (need > scratch_bytes_ && capturing(stream))
            return report(FQ_ERR_HIP, "scratch growth inside a graph capture (make the first call of this shape eagerly)");
        if (need > scratch_bytes_) {
            size_t nb = scratch_bytes_ + scratch_bytes_ / 2;  // geometric growth
            if (nb < need) nb = need;
            nb = (nb + (1 << 20) - 1) & ~(size_t)((1 << 20) - 1);
            void *p = nullptr;
            if (hipMalloc(&p, nb) != hipSuccess) return report(FQ_ERR_HIP, "scratch allocation");
            if (!report(fq_workspace_init(p, nb, (fq_stream_t)stream), "scratch init")) {
                (void)hipFree(p);
                return false;
            }
            if (scratch_) retired_.push_back(scratch_);  // a captured graph may still address it
            scratch_ = p;
            scratch_bytes_ = nb;
        }
        char *base = static_cast<char *>(scratch_);
        out->ws = base;
        out->ws_bytes = wsr;
        out->xq = reinterpret_cast<int8_t *>(base + wsr);
        out->xs = reinterpret_cast<uint16_t *>(base + wsr + align((size_t)M * K));
        return true;
    }

    int x_bits_, w_bits_;
    bool signed_;
    fq_status last_ = FQ_OK;
    std::unordered_map<const int *, Image> images_;
    std::vector<void *> retired_;  // superseded scratch and forgotten images
    void *scratch_ = nullptr;
    size_t scratch_bytes_ = 0;

  public:
    /* free superseded scratch buffers and images dropped by forget_weight() (once no captured
     * graph reads them; the destructor frees them too) */
    void release_retired() {
        for (void *p : retired_) (void)hipFree(p);
        retired_.clear();
    }
    size_t scratch_bytes() const { return scratch_bytes_; }
    size_t retired_count() const { return retired_.size(); }
};

}  // namespace flexq_amd
