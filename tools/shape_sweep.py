"""Decode launch time per shape (development tool): graph of R fused M = 1 linears over rotating
weight copies (cold images), per-launch microseconds.  usage: python tools/shape_sweep.py [M]
Shapes: N = 4096 * k / 4 for the tile-round sweep (tiles per CU 1 .. 6 over 256 CUs) plus the
LLaMA-2-7B / 70B launches."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from flexq_amd import _lib  # noqa: E402

if os.environ.get("FQ_LIB"):  # A/B against another build of the library
    _lib.LIB_PATH = os.path.abspath(os.environ["FQ_LIB"])
from flexq_amd import ops  # noqa: E402

SHAPES = [(4096, 4096), (8192, 4096), (12288, 4096), (16384, 4096), (20480, 4096), (22016, 4096),
          (24576, 4096), (4096, 11008), (10240, 8192), (8192, 8192), (57344, 8192), (8192, 28672)]


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    shapes = SHAPES
    if len(sys.argv) > 3:  # explicit N K pairs
        a = [int(v) for v in sys.argv[2:]]
        shapes = list(zip(a[0::2], a[1::2]))
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    R = 24
    stream = torch.cuda.Stream()
    for (N, K) in shapes:
        copies = max(2, min(8, int(2.5e9 // (N * K))))  # keep the working set well above the MALL
        imgs = []
        for _ in range(copies):
            wq = torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g)
            imgs.append(ops.pack_w6(wq, (torch.rand((K // 128, N), device=dev, generator=g) * 0.01).half()))
        x = torch.randn((M, K), device=dev, dtype=torch.float16, generator=g)
        out = torch.empty((M, N), device=dev, dtype=torch.float16)
        mode = os.environ.get("FQ_SWEEP", "linear")  # linear | gemm (pre-quantized) | quant (quantizer only)
        xq, xs = ops.quantize_act(x, 6)

        def call(img):
            if mode == "gemm":
                ops.gemm_w6ax(xq, xs, img, N, 6, out=out)
            elif mode == "quant":
                ops.quantize_act(x, 6)
            else:
                ops.linear_w6ax(x, img, N, 6, out=out)
        ops.reserve_workspace(dev, [(M, N, K)], stream=stream)
        with torch.cuda.stream(stream):
            for c in imgs:
                call(c)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=stream):
            for i in range(R):
                call(imgs[i % copies])
        graph.replay()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = 1e9
        for _ in range(5):
            s.record()
            graph.replay()
            e.record()
            e.synchronize()
            best = min(best, s.elapsed_time(e) * 1e3 / R)
        nb = N * K * 0.75 + N * K / 64 + 2 * M * K + 2 * M * N
        print(f"{os.environ.get('FQ_LIB', 'lib')} {mode} M={M} N={N:6d} K={K:6d} tiles/CU={N / 16 / 256:5.2f} us/launch={best:7.2f} TB/s={nb / best / 1e6:5.2f}",
              flush=True)
        del imgs, graph
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
