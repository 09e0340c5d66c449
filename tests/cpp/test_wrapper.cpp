// test_wrapper.cpp -- drives the two C++ drop-ins the way FasterTransformer's unchanged call sites
// do: include/flexq_gemm_wrapper.hpp (FLEXQGEMMWrapper; FfnLayer.cc:371-401,521-561 call the int
// path with a nullptr workspace, LlamaV2ContextAttentionLayer.cc:793 sizes its workspace
// 6*M*maxK/8 bytes) and include/flexq_bmma_op.hpp (the named FQBMMA init/exec function pointers,
// selected and called exactly as flexq_gemm_wrapper.cu:53-97 does).  It writes its inputs and the
// outputs to <outdir> as raw little-endian files; tests/test_gpu_wrapper.py checks them against the
// CPU oracle.  Test infrastructure only.
//
// usage: test_wrapper <outdir> <M> <N> <K> <abits> <seed>
//        test_wrapper growth          (scratch growth over ascending M stays logarithmic)
//        test_wrapper capture         (a weight's first use inside a graph capture is refused)
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "flexq_bmma_op.hpp"
#include "flexq_gemm_wrapper.hpp"

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                  \
        }                                                                             \
    } while (0)

static uint64_t g_state;
static uint32_t next_u32() {  // splitmix64
    uint64_t z = (g_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return (uint32_t)((z ^ (z >> 31)) >> 32);
}
static float uniform() { return (next_u32() >> 8) * (1.0f / 16777216.0f); }

template <class T>
static void dump(const std::string &path, const std::vector<T> &v) {
    FILE *f = fopen(path.c_str(), "wb");
    if (!f || fwrite(v.data(), sizeof(T), v.size(), f) != v.size()) {
        fprintf(stderr, "cannot write %s\n", path.c_str());
        exit(2);
    }
    fclose(f);
}

// flexq_gemm_wrapper.cu:53-84: the reference's instance choice per (bits, M)
static void pick(int abits, int M, FQBMMAInitFn_t *init_fn, FQBMMAExecFn_t *exec_fn) {
    if (abits == 6) {
        if (M == 1) *init_fn = FQBMMA_6x6xtrue_1x32x256_8x48x128_8x8x128_2_1_InitFn, *exec_fn = FQBMMA_6x6xtrue_1x32x256_8x48x128_8x8x128_2_1_ExecFn;
        else if (M == 2) *init_fn = FQBMMA_6x6xtrue_2x32x512_16x48x128_8x8x128_2_1_InitFn, *exec_fn = FQBMMA_6x6xtrue_2x32x512_16x48x128_8x8x128_2_1_ExecFn;
        else if (M == 4) *init_fn = FQBMMA_6x6xtrue_4x32x512_24x48x128_8x8x128_2_1_InitFn, *exec_fn = FQBMMA_6x6xtrue_4x32x512_24x48x128_8x8x128_2_1_ExecFn;
        else *init_fn = FQBMMA_6x6xtrue_8x16x256_48x48x128_8x8x128_4_1_InitFn, *exec_fn = FQBMMA_6x6xtrue_8x16x256_48x48x128_8x8x128_4_1_ExecFn;
    } else {
        if (M == 1) *init_fn = FQBMMA_8x6xtrue_1x32x256_8x48x128_8x8x128_4_1_InitFn, *exec_fn = FQBMMA_8x6xtrue_1x32x256_8x48x128_8x8x128_4_1_ExecFn;
        else if (M == 2) *init_fn = FQBMMA_8x6xtrue_2x32x256_16x48x128_8x8x128_4_1_InitFn, *exec_fn = FQBMMA_8x6xtrue_2x32x256_16x48x128_8x8x128_4_1_ExecFn;
        else if (M == 4) *init_fn = FQBMMA_8x6xtrue_4x64x256_32x48x128_8x8x128_4_1_InitFn, *exec_fn = FQBMMA_8x6xtrue_4x64x256_32x48x128_8x8x128_4_1_ExecFn;
        else *init_fn = FQBMMA_8x6xtrue_8x64x384_64x48x128_8x8x128_2_1_InitFn, *exec_fn = FQBMMA_8x6xtrue_8x64x384_64x48x128_8x8x128_2_1_ExecFn;
    }
}

// a rising sequence of shapes must not leave one superseded scratch per new maximum
static int growth() {
    const int N = 4096, K = 4096;
    __half *dx, *dd, *dws;
    int32_t *dwp;
    CK(hipMalloc(&dx, (size_t)2048 * K * 2));
    CK(hipMalloc(&dd, (size_t)2048 * N * 2));
    CK(hipMalloc(&dws, (size_t)(K / 128) * N * 2));
    CK(hipMalloc(&dwp, (size_t)6 * N * (K / 32) * 4));
    CK(hipMemset(dx, 0, (size_t)2048 * K * 2));
    CK(hipMemset(dws, 0, (size_t)(K / 128) * N * 2));
    CK(hipMemset(dwp, 0, (size_t)6 * N * (K / 32) * 4));
    flexq_amd::FLEXQGEMMWrapper w(6, 6, true);
    int calls = 0;
    for (int M = 1; M <= 2048; M += 1 + M / 8, calls++) {
        w.gemm(M, N, K, dx, dwp, nullptr, dd, nullptr, reinterpret_cast<const float *>(dws), nullptr, nullptr, false,
               nullptr, 0, nullptr);
        if (w.status() != FQ_OK) return 10;
    }
    CK(hipDeviceSynchronize());
    printf("growth calls=%d scratch_bytes=%zu retired=%zu\n", calls, w.scratch_bytes(), w.retired_count());
    for (void *p : {(void *)dx, (void *)dd, (void *)dws, (void *)dwp}) CK(hipFree(p));
    return w.retired_count() <= 16 ? 0 : 11;
}

// a weight's FIRST use inside a graph capture is refused (its import would fill the image
// only when the graph replays, so an eager call before that would read it unfilled), by the wrapper and
// by the FQBMMA instances; after an eager first use, capturing works and the replay matches the eager D.
static int capture() {
    const int M = 1, N = 1024, K = 1024;
    __half *dx, *dd, *dws, *dxs;
    int32_t *dwp, *dxp;
    CK(hipMalloc(&dx, (size_t)M * K * 2));
    CK(hipMalloc(&dd, (size_t)M * N * 2));
    CK(hipMalloc(&dws, (size_t)(K / 128) * N * 2));
    CK(hipMalloc(&dxs, (size_t)(K / 128) * 8 * 2));
    CK(hipMalloc(&dwp, (size_t)6 * N * (K / 32) * 4));
    CK(hipMalloc(&dxp, (size_t)6 * 8 * (K / 32) * 4));
    std::vector<__half> hx((size_t)M * K), hws((size_t)(K / 128) * N);
    std::vector<int32_t> hwp((size_t)6 * N * (K / 32));
    for (auto &v : hx) v = __float2half(uniform() - 0.5f);
    for (auto &v : hws) v = __float2half(uniform() * 0.01f);
    for (auto &v : hwp) v = (int32_t)next_u32();
    CK(hipMemcpy(dx, hx.data(), hx.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dws, hws.data(), hws.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dwp, hwp.data(), hwp.size() * 4, hipMemcpyHostToDevice));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    const float *wsf = reinterpret_cast<const float *>(dws);
    flexq_amd::FLEXQGEMMWrapper w(6, 6, true);
    hipGraph_t g;
    // 1. the wrapper: a first use inside the capture is refused, nothing is enqueued
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
    w.gemm(M, N, K, dx, dwp, nullptr, dd, nullptr, wsf, nullptr, nullptr, false, nullptr, 0, s);
    const fq_status refused = w.status();
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphDestroy(g));
    if (refused == FQ_OK) return 20;
    // 2. eager first use, then a captured call replays to the same bits
    std::vector<uint16_t> d_eager((size_t)M * N), d_graph((size_t)M * N);
    w.gemm(M, N, K, dx, dwp, nullptr, dd, nullptr, wsf, nullptr, nullptr, false, nullptr, 0, s);
    if (w.status() != FQ_OK) return 21;
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(d_eager.data(), dd, d_eager.size() * 2, hipMemcpyDeviceToHost));
    CK(hipMemset(dd, 0, (size_t)M * N * 2));
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
    w.gemm(M, N, K, dx, dwp, nullptr, dd, nullptr, wsf, nullptr, nullptr, false, nullptr, 0, s);
    const fq_status captured = w.status();
    CK(hipStreamEndCapture(s, &g));
    if (captured != FQ_OK) return 22;
    hipGraphExec_t ge;
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(d_graph.data(), dd, d_graph.size() * 2, hipMemcpyDeviceToHost));
    if (d_eager != d_graph) return 23;
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    // 3. the FQBMMA instance: its first exec of a weight inside a capture is refused too (D untouched)
    CK(hipMemset(dd, 0, (size_t)M * N * 2));
    FQBMMAInitFn_t init_fn;
    FQBMMAExecFn_t exec_fn;
    pick(6, M, &init_fn, &exec_fn);
    FQBMMAOpState st = (*init_fn)(dxp, dwp, dxs, dws, M, N, K, dd, 128, false);
    if (!st.initSuccess) return 24;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
    (*exec_fn)(st, s);
    CK(hipStreamEndCapture(s, &g));
    size_t nodes = 0;
    CK(hipGraphGetNodes(g, nullptr, &nodes));
    CK(hipGraphDestroy(g));
    if (nodes != 0) return 25;  // (refused before enqueuing anything)
    CK(hipStreamDestroy(s));
    for (void *p : {(void *)dx, (void *)dd, (void *)dws, (void *)dxs, (void *)dwp, (void *)dxp}) CK(hipFree(p));
    printf("capture refusals ok\n");
    return 0;
}

int main(int argc, char **argv) {
    if (argc == 2 && std::string(argv[1]) == "growth") return growth();
    if (argc == 2 && std::string(argv[1]) == "capture") return capture();
    if (argc != 7) {
        fprintf(stderr, "usage: %s outdir M N K abits seed\n", argv[0]);
        return 2;
    }
    const std::string out = argv[1];
    const int M = atoi(argv[2]), N = atoi(argv[3]), K = atoi(argv[4]), abits = atoi(argv[5]);
    g_state = strtoull(argv[6], nullptr, 10);
    if (M <= 0 || N <= 0 || K <= 0 || K % 128 || (N > 8 && N % 8) || (M > 8 && M % 8) || (abits != 6 && abits != 8)) {
        fprintf(stderr, "unsupported case\n");
        return 2;
    }
    // host inputs: activations ~ U(-2, 2) with a few outliers, raw 6-bit weight patterns,
    // weight scales U(0, 0.05)
    std::vector<__half> x((size_t)M * K);
    for (size_t i = 0; i < x.size(); i++) x[i] = __float2half((uniform() * 4.f - 2.f) * (i % 97 == 0 ? 16.f : 1.f));
    std::vector<int32_t> wraw((size_t)N * K);
    for (auto &v : wraw) v = (int32_t)(next_u32() & 63);
    std::vector<__half> ws((size_t)(K / 128) * N);
    for (auto &v : ws) v = __float2half(uniform() * 0.05f);

    hipStream_t s;
    CK(hipStreamCreate(&s));
    __half *dx, *dws, *dd1, *dd2, *dd3, *dxs;
    int32_t *dwraw, *dwp, *dxp;
    char *dwork;
    const size_t wpb = (size_t)6 * N * (K / 32) * 4, xpb = (size_t)abits * M * (K / 32) * 4;
    const size_t xsdup = (size_t)(K / 128) * 2 * ((M + 3) / 4 * 4) * 2;
    // the caller workspace exactly as FT sizes it (LlamaV2ContextAttentionLayer.cc:793)
    const size_t work = (size_t)6 * M * K / 8;
    CK(hipMalloc(&dx, x.size() * 2));
    CK(hipMalloc(&dws, ws.size() * 2));
    CK(hipMalloc(&dd1, (size_t)M * N * 2));
    CK(hipMalloc(&dd2, (size_t)M * N * 2));
    CK(hipMalloc(&dd3, (size_t)M * N * 2));
    CK(hipMalloc(&dxs, xsdup));
    CK(hipMalloc(&dwraw, wraw.size() * 4));
    CK(hipMalloc(&dwp, wpb));
    CK(hipMalloc(&dxp, xpb));
    CK(hipMalloc(&dwork, work));
    CK(hipMemcpy(dx, x.data(), x.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dws, ws.data(), ws.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dwraw, wraw.data(), wraw.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemset(dwork, 0xA5, work));  // the caller's workspace needs no initialisation
    // the weights as FT holds them: bit planes (flexq_bit_packing on the raw patterns)
    if (fq_ref_bit_packing(dwraw, dwp, N, K, 6, (fq_stream_t)s) != FQ_OK) return 3;

    flexq_amd::FLEXQGEMMWrapper w(abits, 6, true);
    // 1. gemm(const half* A ...) with FT's 6*M*maxK/8 workspace: quantize + GEMM (one launch at
    //    decode sizes); the workspace is accepted and left untouched
    w.gemm(M, N, K, dx, dwp, nullptr, dd1, reinterpret_cast<float *>(dxs), reinterpret_cast<const float *>(dws),
           nullptr, nullptr, false, dwork, work, s);
    if (w.status() != FQ_OK) return 4;
    // 2. pack() into a bit-plane buffer, then gemm(const int* A ...) with a nullptr workspace, as
    //    FfnLayer.cc:371-401 calls it
    w.pack(dx, dxp, dxs, M, K, abits, s);
    if (w.status() != FQ_OK) return 5;
    for (int rep = 0; rep < 2; rep++) {  // the second call reuses the imported weight image
        w.gemm(M, N, K, dxp, dwp, nullptr, dd2, reinterpret_cast<float *>(dxs), reinterpret_cast<const float *>(dws),
               nullptr, nullptr, false, nullptr, 0, s);
        if (w.status() != FQ_OK) return 6;
    }
    // 3. the FQBMMA function-pointer instances, called as flexq_gemm_wrapper.cu:53-97 does
    FQBMMAInitFn_t init_fn;
    FQBMMAExecFn_t exec_fn;
    pick(abits, M, &init_fn, &exec_fn);
    for (int rep = 0; rep < 2; rep++) {
        FQBMMAOpState state = (*init_fn)(reinterpret_cast<const int *>(dxp), dwp, reinterpret_cast<half *>(dxs),
                                         reinterpret_cast<const half *>(dws), M, N, K, dd3, 128, false);
        if (!state.initSuccess) return 9;
        (*exec_fn)(state, s);
    }
    // 4. the reference's rejections print and return (exactly two "[FlexQ][Error]" lines)
    w.gemm(M, N, 100, dx, dwp, nullptr, dd1, nullptr, nullptr, nullptr, nullptr, false, dwork, work, s);
    if (w.status() != FQ_ERR_SHAPE) return 7;
    FQBMMAOpState bad = (*init_fn)(reinterpret_cast<const int *>(dxp), dwp, reinterpret_cast<half *>(dxs),
                                   reinterpret_cast<const half *>(dws), M, N, K, dd3, 64, false);
    if (bad.initSuccess) return 8;
    CK(hipStreamSynchronize(s));
    {  // the caller's workspace was never written
        std::vector<unsigned char> hw(work);
        CK(hipMemcpy(hw.data(), dwork, work, hipMemcpyDeviceToHost));
        for (unsigned char c : hw)
            if (c != 0xA5) return 12;
    }

    std::vector<__half> d1((size_t)M * N), d2((size_t)M * N), d3((size_t)M * N);
    CK(hipMemcpy(d1.data(), dd1, d1.size() * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(d2.data(), dd2, d2.size() * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(d3.data(), dd3, d3.size() * 2, hipMemcpyDeviceToHost));
    dump(out + "/x.f16", x);
    dump(out + "/wraw.i32", wraw);
    dump(out + "/ws.f16", ws);
    dump(out + "/d_half.f16", d1);
    dump(out + "/d_int.f16", d2);
    dump(out + "/d_bmma.f16", d3);
    for (void *p : {(void *)dx, (void *)dws, (void *)dd1, (void *)dd2, (void *)dd3, (void *)dxs, (void *)dwraw, (void *)dwp,
                    (void *)dxp, (void *)dwork})
        CK(hipFree(p));
    CK(hipStreamDestroy(s));
    printf("test_wrapper ok M=%d N=%d K=%d a%d\n", M, N, K, abits);
    return 0;
}
