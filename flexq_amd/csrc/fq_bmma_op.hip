// fq_bmma_op.hip -- the reference's FQBMMA function-pointer instances (include/flexq_bmma_op.hpp)
// over this build's C ABI.  Host code only: the GEMM is fq_gemm_w6ax, the operand imports are
// fq_import_ref_w / fq_import_ref_x (fq_quant.hip).
//
// Reference: e2e/src/fastertransformer/kernels/flexqgemm/src/bgemm/flexq_bmma_op.h:19-34 (state),
// :64-133 (initialize), :159-184 (InitFn / ExecFn and their typedefs), flexq_bmma_library.h (the
// instance names), flexq_gemm_wrapper.cu:53-97 (the caller: one named instance per (bits, M)).
#include <cstdio>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

#include "../../include/flexq_bmma_op.hpp"
#include "fq_common.h"

namespace {

struct WeightKey {
    const void *W;
    const void *W_SCALE;
    int N, K;
    bool operator<(const WeightKey &o) const { return std::tie(W, W_SCALE, N, K) < std::tie(o.W, o.W_SCALE, o.N, o.K); }
};
struct Scratch {
    void *ptr = nullptr;
    size_t bytes = 0;
};

// Library-owned device memory of the instances: never freed while the process runs (a captured
// graph bakes these addresses in), superseded buffers retired instead.
std::mutex g_mu;
// an imported weight image, the stream its import was enqueued on, and an event recorded behind the
// import (null once it has completed).  Imports are always eager: an import captured into a graph would
// fill the image only when that graph replays, so an eager exec (or another graph) before the replay
// would read it unfilled -- the first exec of a weight inside a capture is refused.
struct Image {
    void *img;
    hipStream_t owner;
    hipEvent_t ready;
};

bool stream_capturing(hipStream_t s) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return !(hipStreamIsCapturing(s, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone);
}
std::map<WeightKey, Image> g_images;
std::map<hipStream_t, Scratch> g_scratch;
std::vector<void *> g_retired;
size_t g_device_bytes = 0;

size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

bool report(fq_status s, const char *what) {
    if (s != FQ_OK) fprintf(stderr, "[FlexQ][Error] %s: %s\n", what, fq_status_string(s));
    return s == FQ_OK;
}

int device_cus_cached() {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
    }
    return cus;
}

// scratch layout for one call: [GEMM workspace, at least the split-K ticket region | xq int8 [M][K] |
// xs fp16 [K/128][M]].  The ticket region is always reserved at the head, so codes of a shape
// without split-K never land on the tickets a later split-K shape expects zeroed.
size_t ws_region(int M, int N, int K) {
    const size_t need = fq_gemm_workspace_bytes(M, N, K);
    return align256(need > FQ_TICKET_BYTES ? need : FQ_TICKET_BYTES);
}
size_t scratch_need(int M, int N, int K) {
    return ws_region(M, N, K) + align256((size_t)M * K) + align256((size_t)M * (K / FQ_GROUP) * 2);
}

const void *weight_image(const FQBMMAOpState::Argument_t &a, hipStream_t s) {
    std::lock_guard<std::mutex> lk(g_mu);
    const WeightKey key{a.W, a.W_SCALE, a.N, a.K};
    auto it = g_images.find(key);
    if (it != g_images.end()) {
        // another stream's first use must not overtake the import enqueued on the owner's stream
        Image &im = it->second;
        if (im.ready && s != im.owner) {
            const bool capturing = stream_capturing(s);
            if (hipEventQuery(im.ready) == hipSuccess) {
                (void)hipEventDestroy(im.ready);
                im.ready = nullptr;  // the import has completed: no stream needs to wait any more
            } else if (capturing) {
                // an event recorded outside this capture cannot order a captured node: refuse rather than
                // record a graph without the dependency
                report(FQ_ERR_HIP, "FQBMMA exec: captured use of a weight image whose eager import is still in "
                                   "flight on another stream (synchronise before capturing)");
                return nullptr;
            } else if (hipStreamWaitEvent(s, im.ready, 0) != hipSuccess) {
                report(FQ_ERR_HIP, "FQBMMA exec: ordering against the weight import");
                return nullptr;
            }
        }
        return im.img;
    }
    if (stream_capturing(s)) {
        report(FQ_ERR_HIP, "FQBMMA exec: first use of a weight inside a graph capture (run the first exec eagerly: "
                           "its import would only run when the graph replays)");
        return nullptr;
    }
    void *img = nullptr;
    const size_t bytes = fq_packed_w_bytes(a.N, a.K);
    if (hipMalloc(&img, bytes) != hipSuccess) {
        report(FQ_ERR_HIP, "FQBMMA exec: weight image allocation");
        return nullptr;
    }
    if (!report(fq_import_ref_w(reinterpret_cast<const int32_t *>(a.W), reinterpret_cast<const uint16_t *>(a.W_SCALE),
                                a.N, a.K, img, (fq_stream_t)s),
                "FQBMMA exec: weight import")) {
        (void)hipFree(img);
        return nullptr;
    }
    hipEvent_t ready = nullptr;
    if (hipEventCreateWithFlags(&ready, hipEventDisableTiming) == hipSuccess && hipEventRecord(ready, s) != hipSuccess) {
        (void)hipEventDestroy(ready);
        ready = nullptr;
    }
    g_images[key] = Image{img, s, ready};
    g_device_bytes += bytes;
    return img;
}

void *stream_scratch(size_t need, hipStream_t s, size_t *bytes) {
    std::lock_guard<std::mutex> lk(g_mu);
    Scratch &sc = g_scratch[s];
    if (sc.bytes < need && stream_capturing(s)) {  // (its zeroing would run only when the graph replays)
        report(FQ_ERR_HIP, "FQBMMA exec: scratch growth inside a graph capture (run the shape eagerly first)");
        return nullptr;
    }
    if (sc.bytes < need) {
        // geometric growth (x1.5, 1 MiB granules): a rising sequence of shapes allocates O(log) times
        size_t nb = sc.bytes + sc.bytes / 2;
        if (nb < need) nb = need;
        nb = (nb + (1 << 20) - 1) & ~(size_t)((1 << 20) - 1);
        void *p = nullptr;
        if (hipMalloc(&p, nb) != hipSuccess) {
            report(FQ_ERR_HIP, "FQBMMA exec: scratch allocation");
            return nullptr;
        }
        if (!report(fq_workspace_init(p, nb, (fq_stream_t)s), "FQBMMA exec: scratch init")) {
            (void)hipFree(p);
            return nullptr;
        }
        if (sc.ptr) g_retired.push_back(sc.ptr);
        sc.ptr = p;
        sc.bytes = nb;
        g_device_bytes += nb;
    }
    *bytes = sc.bytes;
    return sc.ptr;
}

template <int XB>
FQBMMAOpState init_impl(const int *X, const int *W, half *X_SCALE, const half *W_SCALE, int M, int N, int K, half *D,
                        int group_size, bool bias) {
    FQBMMAOpState st;
    st.args.M = M;
    st.args.N = N;
    st.args.K = K;
    st.args.X = X;
    st.args.W = W;
    st.args.X_SCALE = X_SCALE;
    st.args.W_SCALE = W_SCALE;
    st.args.D = D;
    st.args.group_size = group_size;
    st.args.bias = bias;
    st.shared_mem_size = 0;
    st.gridDim = dim3((unsigned)device_cus_cached(), 1, 1);
    st.blockDim = dim3(512, 1, 1);
    const char *why = nullptr;
    if (!X || !W || !X_SCALE || !W_SCALE || !D) why = "null operand";
    else if (group_size != FQ_GROUP) why = "group_size must be 128";
    else if (bias) why = "bias is not supported";
    else if (M <= 0 || N <= 0 || K <= 0 || K % FQ_GROUP) why = "unsupported M/N/K (K % 128 == 0 required)";
    else if (!(M <= 8 || M % 8 == 0) || !(N <= 8 || N % 8 == 0)) why = "bit-plane rows (M, N) must be <= 8 or multiples of 8";
    else if ((size_t)((N + 15) / 16) > FQ_TICKET_BYTES / 4) why = "N too large";
    if (why) fprintf(stderr, "[FlexQ][Error] FQBMMA init (W6A%d): %s\n", XB, why);
    st.initSuccess = why == nullptr;
    return st;
}

template <int XB>
void exec_impl(FQBMMAOpState &st, hipStream_t s) {
    if (!st.initSuccess) {
        fprintf(stderr, "[FlexQ][Error] return due to unsuccessful initialization.\n");
        return;
    }
    const FQBMMAOpState::Argument_t &a = st.args;
    const void *img = weight_image(a, s);
    if (!img) return;
    size_t sbytes = 0;
    char *base = static_cast<char *>(stream_scratch(scratch_need(a.M, a.N, a.K), s, &sbytes));
    if (!base) return;
    const size_t wsr = ws_region(a.M, a.N, a.K);
    int8_t *xq = reinterpret_cast<int8_t *>(base + wsr);
    uint16_t *xs = reinterpret_cast<uint16_t *>(base + wsr + align256((size_t)a.M * a.K));
    report(fq_gemm_w6ax_planes(a.X, reinterpret_cast<const uint16_t *>(a.X_SCALE), img, a.M, a.N, a.K, XB,
                               reinterpret_cast<uint16_t *>(a.D), xq, xs, base, wsr, (fq_stream_t)s),
           "FQBMMA exec");
}

}  // namespace

// The instances the reference's wrapper names (flexq_gemm_wrapper.cu:53-84).  One implementation
// per activation width: this build dispatches on M itself (fq_gemm_w6ax), so the tile shapes in the
// names select nothing.
#define FQ_AMD_INSTANCE(name, xb)                      \
    FQBMMAInitFn_t name##_InitFn = init_impl<xb>;      \
    FQBMMAExecFn_t name##_ExecFn = exec_impl<xb>;
FQ_AMD_INSTANCE(FQBMMA_6x6xtrue_1x32x256_8x48x128_8x8x128_2_1, 6)
FQ_AMD_INSTANCE(FQBMMA_6x6xtrue_2x32x512_16x48x128_8x8x128_2_1, 6)
FQ_AMD_INSTANCE(FQBMMA_6x6xtrue_4x32x512_24x48x128_8x8x128_2_1, 6)
FQ_AMD_INSTANCE(FQBMMA_6x6xtrue_8x16x256_48x48x128_8x8x128_4_1, 6)
FQ_AMD_INSTANCE(FQBMMA_8x6xtrue_1x32x256_8x48x128_8x8x128_4_1, 8)
FQ_AMD_INSTANCE(FQBMMA_8x6xtrue_2x32x256_16x48x128_8x8x128_4_1, 8)
FQ_AMD_INSTANCE(FQBMMA_8x6xtrue_4x64x256_32x48x128_8x8x128_4_1, 8)
FQ_AMD_INSTANCE(FQBMMA_8x6xtrue_8x64x384_64x48x128_8x8x128_2_1, 8)
#undef FQ_AMD_INSTANCE

extern "C" int fq_bmma_op_forget_weight(const void *W) {
    std::lock_guard<std::mutex> lk(g_mu);
    int dropped = 0;
    for (auto it = g_images.begin(); it != g_images.end();) {
        if (it->first.W == W) {
            g_retired.push_back(it->second.img);  // a captured graph may still read it: never freed
            if (it->second.ready) (void)hipEventDestroy(it->second.ready);
            it = g_images.erase(it);
            dropped++;
        } else {
            ++it;
        }
    }
    return dropped;
}

extern "C" size_t fq_bmma_op_device_bytes(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    return g_device_bytes;
}
