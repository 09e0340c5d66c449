"""Fused producer timings (development tool): fq_rmsnorm_quantize and fq_silu_mul_quantize at the
LLaMA-2-7B / 70B decode and prefill sizes, graph-timed, with algorithmic HBM bytes and GB/s.
  rmsnorm: reads input + residual + gamma (4 B/elem), writes residual + codes + scales (3 B/elem + K/64)
  silu:    reads gate + up (4 B/elem), writes codes + scales (1 B/elem + N/64)"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from flexq_amd import ops  # noqa: E402


def timed(fn, reps=50):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s):  # replay() launches on the current stream
        a.record(s)
        g.replay()
        b.record(s)
    b.synchronize()
    return a.elapsed_time(b) * 1e3 / reps  # us


def main():
    dev = torch.device("cuda:0")
    for (M, K, F) in [(1, 4096, 11008), (16, 4096, 11008), (1, 8192, 28672), (2048, 4096, 14336), (16384, 4096, 14336)]:
        res = torch.randn((M, K), device=dev).half()
        inp = torch.randn((M, K), device=dev).half()
        gamma = torch.ones(K, device=dev).half()
        t = timed(lambda: ops.rmsnorm_quantize(res, gamma, 6, input=inp))
        by = M * K * (2 + 2 + 2 + 1) + 2 * K + 2 * M * K // 128
        gu = torch.randn((M, 2 * F), device=dev).half()
        t2 = timed(lambda: ops.silu_mul_quantize(gu[:, :F], gu[:, F:], 8))
        by2 = M * F * (2 + 2 + 1) + 2 * M * F // 128
        print(f"M={M:6d} K={K:5d}: rmsnorm+quant {t:8.2f} us {by / t / 1e3:7.0f} GB/s | "
              f"F={F:5d}: silu*up+quant {t2:8.2f} us {by2 / t2 / 1e3:7.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
