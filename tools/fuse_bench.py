"""Decode linear: fused one-launch quantize+GEMM vs quantize launch + GEMM launch (development tool).
For each M and LLaMA-2-7B shape, a HIP graph of linears over weight copies totalling > 768 MB
(no Infinity Cache reuse), per-launch time for
  linear : ops.linear_w6ax (what the plan picks: fused or split)
  split  : ops.quantize_act + ops.gemm_w6ax (two launches)
  gemm   : ops.gemm_w6ax alone (pre-quantized activations)
usage: python tools/fuse_bench.py [M,M,...] [7b|70b]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from flexq_amd import ops  # noqa: E402

SHAPES = {"7b": [(12288, 4096, 6), (4096, 4096, 6), (22016, 4096, 6), (4096, 11008, 8)],
          "70b": [(10240, 8192, 6), (8192, 8192, 6), (57344, 8192, 6), (8192, 28672, 8)]}


def graph_us(fn, n, reps=5):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        gph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gph, stream=s):
            fn()
    gph.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        gph.replay()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps / n * 1e3


def main():
    Ms = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1, 2, 4, 8, 16, 32]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    for (N, K, ab) in SHAPES[sys.argv[2] if len(sys.argv) > 2 else "7b"]:
        nbytes = ops.packed_w_bytes(N, K)
        copies = max(2, (768 << 20) // nbytes + 1)
        wq = torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g)
        ws = (torch.rand((K // 128, N), device=dev, generator=g) * 0.01).half()
        img0 = ops.pack_w6(wq, ws)
        imgs = [img0.clone() for _ in range(copies)]
        del wq, ws, img0
        for M in Ms:
            x = torch.randn((M, K), device=dev, dtype=torch.float16, generator=g)
            out = torch.empty((M, N), device=dev, dtype=torch.float16)
            xq = torch.empty((M, K), dtype=torch.int8, device=dev)
            t_lin = graph_us(lambda: [ops.linear_w6ax(x, w, N, ab, out=out) for w in imgs], copies)

            def split():
                for w in imgs:
                    q, s = ops.quantize_act(x, ab)
                    ops.gemm_w6ax(q, s, w, N, ab, out=out)
            t_split = graph_us(split, copies)
            q, s = ops.quantize_act(x, ab)
            t_gemm = graph_us(lambda: [ops.gemm_w6ax(q, s, w, N, ab, out=out) for w in imgs], copies)
            fused = ops.act_scratch_bytes(M, N, K) == 0
            gbs = (nbytes + 2 * M * K + 2 * M * N) / t_lin / 1e3
            print(f"N={N:6d} K={K:6d} M={M:3d}: linear {t_lin:7.2f} us ({'fused' if fused else 'split'}, "
                  f"{gbs:6.0f} GB/s) | split {t_split:7.2f} us | gemm only {t_gemm:7.2f} us", flush=True)
            del x, out, xq
        del imgs


if __name__ == "__main__":
    main()
