"""Bit-plane activation path timings (development tool): FT's int-overload call
(FLEXQGEMMWrapper::gemm(const int* A ...), FQBMMAExecFn_t) at the LLaMA-2-7B decode shapes,
graph-timed per launch group on rotating weight images (cold, as in the bench step):
  planes   fq_gemm_w6ax_planes -- the planes unpacked inside the GEMM prologue (one launch)
  import   fq_import_ref_x + fq_gemm_w6ax (the previous two-launch path)
  linear   fq_linear_w6ax on the fp16 activation (this build's own fused path, for reference)"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from flexq_amd import ops  # noqa: E402


def timed(fn, reps=40):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn(0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for i in range(reps):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = None
    for _ in range(3):
        with torch.cuda.stream(s):
            a.record(s)
            g.replay()
            b.record(s)
        b.synchronize()
        t = a.elapsed_time(b) * 1e3 / reps
        best = t if best is None or t < best else best
    return best  # us per call


def main():
    dev = torch.device("cuda:0")
    for M in [int(v) for v in os.environ.get("PB_M", "1,4").split(",")]:
        for (N, K) in [(12288, 4096), (4096, 4096), (22016, 4096), (4096, 11008)]:
            bits = 6
            nimg = 8
            imgs = [ops.quantize_pack_w6(torch.randn((N, K), device=dev).half() * 0.02)[0] for _ in range(nimg)]
            x = torch.randn((M, K), device=dev).half()
            planes, dup = ops.ref_quantize_bit_packing(x, bits)
            xq = torch.empty((M, K), dtype=torch.int8, device=dev)
            xs = torch.empty((K // 128, M), dtype=torch.float16, device=dev)
            out = torch.empty((M, N), dtype=torch.float16, device=dev)
            t_pl = timed(lambda i: ops.gemm_w6ax_planes(planes, dup, imgs[i % nimg], M, N, K, bits, out=out))
            from flexq_amd import _lib
            L = _lib.load()

            def imp(i):
                _lib.call("fq_import_ref_x", planes.data_ptr(), dup.data_ptr(), M, K, bits, xq.data_ptr(),
                          xs.data_ptr(), torch.cuda.current_stream().cuda_stream)
                ops.gemm_w6ax(xq, xs, imgs[i % nimg], N, bits, out=out)
            t_im = timed(imp)
            t_li = timed(lambda i: ops.linear_w6ax(x, imgs[i % nimg], N, bits, out=out))
            d1 = ops.gemm_w6ax_planes(planes, dup, imgs[0], M, N, K, bits)
            imp(0)
            torch.cuda.synchronize()
            d2 = ops.gemm_w6ax(xq, xs, imgs[0], N, bits)
            same = bool(np.array_equal(d1.cpu().numpy().view(np.uint16), d2.cpu().numpy().view(np.uint16)))
            fused = int(L.fq_planes_act_scratch_bytes(M, N, K)) == 0
            print(f"M={M} N={N:5d} K={K:5d}: planes {t_pl:6.2f} us ({'fused' if fused else 'import'})  "
                  f"import+gemm {t_im:6.2f} us  linear(fp16) {t_li:6.2f} us  bit-identical={same}", flush=True)
            del imgs


if __name__ == "__main__":
    main()
