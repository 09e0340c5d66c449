"""Per-shape kernel timing sweep (development tool): W6Ax GEMM vs torch fp16 (rocBLAS/hipBLASLt).

python tools/kbench.py [--shapes llama7b|llama70b|all] [--m 1,16] [--iters 50]
Prints one line per (M, N, K, abits): us per call, algorithmic GB/s, TFLOPS-equiv, fp16 us, ratio.
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from flexq_amd import ops  # noqa: E402

SHAPES = {
    "llama7b": [(12288, 4096, 6), (4096, 4096, 6), (11008, 4096, 6), (4096, 11008, 6)],
    "llama70b": [(24576, 8192, 6), (8192, 8192, 6), (28672, 8192, 6), (8192, 28672, 6)],
    "llama3_8b": [(6144, 4096, 8), (4096, 4096, 8), (14336, 4096, 8), (4096, 14336, 8)],
}


def alg_bytes(M, N, K, abits):
    return N * K * 6 / 8 + 2 * N * K / 128 + M * K + 2 * M * K / 128 + 2 * M * N


def time_fn(fn, iters, reps=3):
    best = None
    for _ in range(reps):
        fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        t = s.elapsed_time(e) / iters * 1e3
        best = t if best is None else min(best, t)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="llama7b,llama70b")
    ap.add_argument("--m", default="1,16")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--copies", type=int, default=4, help="rotate weight copies to defeat the 256 MiB MALL")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    for group in a.shapes.split(","):
        for (N, K, abits) in SHAPES[group]:
            copies = []
            for c in range(a.copies):
                wq = torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g)
                pk = ops.pack_w6(wq)
                ws = (torch.rand((K // 128, N), device=dev, generator=g) * 0.01).half()
                wf = torch.randn((N, K), device=dev, dtype=torch.float16, generator=g)
                copies.append((pk, ws, wf))
                del wq
            for M in [int(m) for m in a.m.split(",")]:
                x = torch.randn((M, K), device=dev, dtype=torch.float16, generator=g)
                xq, xs = ops.quantize_act(x, abits)
                out = torch.empty((M, N), device=dev, dtype=torch.float16)
                it = [0]

                def run():
                    pk, ws, _ = copies[it[0] % len(copies)]
                    it[0] += 1
                    ops.gemm_w6ax(xq, xs, pk, ws, N, abits, out=out)

                def run_fp16():
                    _, _, wf = copies[it[0] % len(copies)]
                    it[0] += 1
                    torch.matmul(x, wf.t())

                def run_q():
                    ops.quantize_act(x, abits)

                t = time_fn(run, a.iters)
                tf = time_fn(run_fp16, a.iters)
                tq = time_fn(run_q, a.iters)
                gbs = alg_bytes(M, N, K, abits) / t / 1e3
                tflops = 2 * M * N * K / t / 1e6
                print(f"M={M:5d} N={N:6d} K={K:6d} a{abits}: gemm {t:8.2f} us {gbs:7.0f} GB/s {tflops:8.2f} TFLOPS | "
                      f"quant {tq:6.2f} us | fp16 {tf:8.2f} us ({2*N*K/tf/1e3:6.0f} GB/s) | speedup {tf/t:5.2f}x",
                      flush=True)
            del copies


if __name__ == "__main__":
    main()
