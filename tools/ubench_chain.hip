// ubench_chain.hip -- floor of a dependent chain of decode-sized launches (development tool).
//
// What a graph of R back-to-back launches costs per launch when each launch
//   mode 0: does nothing (256 WGs x 512 threads),
//   mode 1: loads one 16-byte chunk per lane of a small "activation" and stores 16 B per WG,
//   mode 2: streams B bytes of a weight buffer (16 B per lane, nt, 8 waves per CU, 4 loads in
//           flight per lane) and stores one dword per WG,
// compared with fq_gemm_decode_kernel's per-launch times on the same byte counts
// (tools/shape_sweep.py).  Build: hipcc -O3 --offload-arch=gfx950 -o tools/ubench_chain tools/ubench_chain.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                           \
        }                                                                                      \
    } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(512) void k_empty(int *out) {
    if (threadIdx.x == 0 && out == nullptr) out[blockIdx.x] = 0;
}

__global__ __launch_bounds__(512) void k_empty_lds(int *out) {
    extern __shared__ int sm[];
    if (threadIdx.x == 0 && out == nullptr) out[blockIdx.x] = sm[0];
}

__global__ __launch_bounds__(512) void k_touch(const v4i *__restrict__ x, v4i *__restrict__ out) {
    const v4i v = x[threadIdx.x & 511];
    if (threadIdx.x == 0) out[blockIdx.x] = v;
}

// each WG streams its contiguous share of `w` (bytes per WG = per_wg, multiple of 8 KiB)
template <int U>
__global__ __launch_bounds__(512) void k_stream(const v4i *__restrict__ w, long per_wg, int *__restrict__ out) {
    const v4i *p = w + (long)blockIdx.x * (per_wg / 16) + threadIdx.x;
    const long n = per_wg / (16 * 512);  // 16 B per lane per step
    v4i acc = {0, 0, 0, 0};
    long i = 0;
    for (; i + U <= n; i += U) {
        v4i r[U];
#pragma unroll
        for (int u = 0; u < U; u++) r[u] = __builtin_nontemporal_load(p + (i + u) * 512);
#pragma unroll
        for (int u = 0; u < U; u++) acc ^= r[u];
    }
    for (; i < n; i++) acc ^= __builtin_nontemporal_load(p + i * 512);
    const int s = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
    if (s == 0x7fffffff) out[blockIdx.x] = s;  // keep the loads alive
}

int main(int argc, char **argv) {
    const int R = 64;
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const long sizes_mb[] = {0, 4, 13, 39, 69, 135};
    const long maxb = 8L << 30;  // rotating over 8 GiB so nothing is cache-resident
    char *w;
    CK(hipMalloc(&w, maxb));
    CK(hipMemset(w, 1, maxb));
    int *out;
    v4i *x, *o4;
    CK(hipMalloc(&out, 4096 * sizeof(int)));
    CK(hipMalloc(&x, 8192 * 16));
    CK(hipMalloc(&o4, 4096 * 16));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto time_graph = [&](auto launch) {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        for (int i = 0; i < R; i++) launch(i);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        float best = 1e30f;
        for (int rep = 0; rep < 5; rep++) {
            CK(hipEventRecord(e0, s));
            CK(hipGraphLaunch(ge, s));
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
        return best * 1000.f / R;  // us per launch
    };
    printf("empty   us/launch=%.2f\n", time_graph([&](int) { hipLaunchKernelGGL(k_empty, dim3(cus), dim3(512), 0, s, out); }));
    for (int g : {1, 64, 256, 1024})
        for (int t : {64, 256, 512})
            printf("empty   grid=%4d threads=%3d us/launch=%.2f\n", g, t,
                   time_graph([&](int) { hipLaunchKernelGGL(k_empty, dim3(g), dim3(t), 0, s, out); }));
    for (int lds : {0, 32768, 98304})
        printf("empty   grid=%4d threads=512 lds=%6d us/launch=%.2f\n", cus, lds,
               time_graph([&](int) { hipLaunchKernelGGL(k_empty_lds, dim3(cus), dim3(512), lds, s, out); }));
    printf("touch   us/launch=%.2f\n", time_graph([&](int) { hipLaunchKernelGGL(k_touch, dim3(cus), dim3(512), 0, s, x, o4); }));
    for (long mb : sizes_mb) {
        if (!mb) continue;
        const long per_wg = ((mb << 20) / cus + 8191) / 8192 * 8192;
        const long bytes = per_wg * cus;
        const long copies = maxb / bytes;
        for (int u : {2, 4, 8}) {
            float us = time_graph([&](int i) {
                const v4i *base = (const v4i *)(w + (long)(i % copies) * bytes);
                if (u == 2) hipLaunchKernelGGL(k_stream<2>, dim3(cus), dim3(512), 0, s, base, per_wg, out);
                if (u == 4) hipLaunchKernelGGL(k_stream<4>, dim3(cus), dim3(512), 0, s, base, per_wg, out);
                if (u == 8) hipLaunchKernelGGL(k_stream<8>, dim3(cus), dim3(512), 0, s, base, per_wg, out);
            });
            printf("stream  MB=%6.1f U=%d us/launch=%7.2f TB/s=%5.2f\n", bytes / 1048576.0, u, us, bytes / us / 1e6);
        }
    }
    CK(hipFree(w));
    return 0;
}
