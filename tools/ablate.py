"""Decode-GEMM ablation timing (development tool; needs abtmp/libflexq_hip_abl.so built with
-DFQ_DEV_ABLATION).  For each ablation mask, captures a HIP graph of R GEMM launches per shape
(weights rotated over several copies so the MALL cannot hold them) and prints us/launch.
  mask 2: no MFMA/dequant   4: no cross-wave reduction/fix-up   6: both (pure streaming)
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from flexq_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.environ.get("FQ_ABL_LIB", os.path.join(ROOT, "abtmp", "libflexq_hip_abl.so"))
from flexq_amd import ops  # noqa: E402

SHAPES = [(12288, 4096), (4096, 4096), (11008, 4096), (4096, 11008), (28672, 8192), (8192, 28672)]


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    R, COPIES = 20, 6
    masks = [int(m) for m in (sys.argv[1] if len(sys.argv) > 1 else "0,2,4,6").split(",")]
    linear = len(sys.argv) > 2 and sys.argv[2] == "linear"  # fused quantize+GEMM from fp16 x
    stream = torch.cuda.Stream()
    for (N, K) in SHAPES:
        copies = []
        for _ in range(COPIES):
            wq = torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g)
            copies.append(ops.pack_w6(wq, (torch.rand((K // 128, N), device=dev, generator=g) * 0.01).half()))
        x = torch.randn((1, K), device=dev, dtype=torch.float16, generator=g)
        xq, xs = ops.quantize_act(x, 6)
        out = torch.empty((1, N), device=dev, dtype=torch.float16)

        def run(c):
            if linear:
                ops.linear_w6ax(x, c, N, 6, out=out)
            else:
                ops.gemm_w6ax(xq, xs, c, N, 6, out=out)
        line = f"N={N:6d} K={K:6d} MB={N * K * 0.75 / 2**20:6.1f}:"
        for m in masks:
            os.environ["FQ_DEV_ABLATION"] = str(m)
            with torch.cuda.stream(stream):
                for i in range(COPIES):
                    run(copies[i])
            torch.cuda.synchronize()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=stream):
                for i in range(R):
                    run(copies[i % COPIES])
            for _ in range(3):
                graph.replay()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                graph.replay()
            e.record()
            e.synchronize()
            us = s.elapsed_time(e) * 1e3 / (5 * R)
            line += f"  abl{m}: {us:7.2f} us ({N * K * 0.75 / us / 1e3:5.0f} GB/s)"
        print(line, flush=True)
        del copies


if __name__ == "__main__":
    main()
