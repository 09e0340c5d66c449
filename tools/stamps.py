"""Decode-kernel timeline (development tool; abtmp/libflexq_hip_abl.so, ablation mask 16).
Per workgroup s_memrealtime stamps (100 MHz): 0 entry, 1 ring prologue issued, 2 first block
landed, 3 item loop done, 4 split-K fix-up done.  Prints, per shape, the kernel span against the
graph-replay time per launch, the dispatch skew and the phase medians (us).  FQ_STAMP_M: rows (default
1; 16 stamps the batch-16 GEMM); FQ_STAMP_SHAPES: "N K N K ..." instead of the default shapes."""
import ctypes
import os
import sys

import numpy as np
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
    M = int(os.environ.get("FQ_STAMP_M", "1"))
    shapes = SHAPES
    if os.environ.get("FQ_STAMP_SHAPES"):
        a = [int(v) for v in os.environ["FQ_STAMP_SHAPES"].split()]
        shapes = list(zip(a[0::2], a[1::2]))
    os.environ["FQ_DEV_ABLATION"] = os.environ.get("FQ_STAMP_MASK", "16")
    L = _lib.load()
    L.fq_dev_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    stream = torch.cuda.Stream()
    for linear in (False, True):
        for (N, K) in shapes:
            copies = []
            for _ in range(COPIES):
                wq = torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g)
                copies.append(ops.pack_w6(wq, (torch.rand((K // 128, N), device=dev, generator=g) * 0.01).half()))
            x = torch.randn((M, K), device=dev, dtype=torch.float16, generator=g)
            xq, xs = ops.quantize_act(x, 6)
            out = torch.empty((M, N), device=dev, dtype=torch.float16)

            def run(c):
                if linear:
                    ops.linear_w6ax(x, c, N, 6, out=out)
                else:
                    ops.gemm_w6ax(xq, xs, c, N, 6, out=out)
            with torch.cuda.stream(stream):
                for c in copies:
                    run(c)
            torch.cuda.synchronize()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=stream):
                for i in range(R):
                    run(copies[i % COPIES])
            graph.replay()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                graph.replay()
            e.record()
            e.synchronize()
            per = s.elapsed_time(e) * 1e3 / (5 * R)
            buf = np.zeros(1024 * 8, np.uint64)
            L.fq_dev_stamps_clear() if hasattr(L, 'fq_dev_stamps_clear') else None
            L.fq_dev_stamps(buf.ctypes.data, buf.size)
            st = buf.reshape(1024, 8).astype(np.int64)
            st = st[st[:, 0] > 0]
            # keep the last launch only: entries within 200 us of the latest entry
            st = st[st[:, 0] > st[:, 0].max() - 20000]
            t0 = st[:, 0].min()
            us = lambda v: v / 100.0  # 100 MHz ticks -> us
            end = np.maximum(st[:, 3], st[:, 4])
            print(f"{'linear' if linear else 'gemm  '} M={M} N={N:6d} K={K:6d} wgs={len(st):4d} per_launch={per:6.2f} "
                  f"span={us(end.max() - t0):6.2f} skew={us(st[:, 0].max() - t0):5.2f} "
                  f"stage={us(np.median(st[:, 7] - st[:, 0])):5.2f} issue={us(np.median(st[:, 1] - st[:, 0])):5.2f} first={us(np.median(st[:, 2] - st[:, 1])):5.2f} "
                  f"loop={us(np.median(st[:, 3] - st[:, 2])):6.2f} (max {us((st[:, 3] - st[:, 2]).max()):6.2f}) "
                  f"end_spread={us(end.max() - end.min()):5.2f} fixup={us(np.median(np.maximum(st[:, 4] - st[:, 3], 0))):5.2f}"
                  + (f" xwait={us(np.median(st[:, 5] - st[:, 1])):5.2f} quant={us(np.median(st[:, 6] - st[:, 5])):5.2f}"
                     + (f" quant2={us(np.median(st[:, 4] - st[:, 6])):5.2f}" if os.environ.get("FQ_STAMP_MASK") in ("48", "112") else "")
                     if linear else ""),
                  flush=True)
            del copies, graph


if __name__ == "__main__":
    main()
