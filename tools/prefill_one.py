"""Run one prefill GEMM shape a few times (profiling target for rocprofv3 --pmc).
usage: python tools/prefill_one.py M N K [reps]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from flexq_amd import ops  # noqa: E402


def main():
    M, N, K = (int(v) for v in sys.argv[1:4])
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    wq = torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g)
    ws = (torch.rand((K // 128, N), device=dev, generator=g) * 0.01).half()
    img = ops.pack_w6(wq, ws)
    xq = torch.randint(-128, 128, (M, K), dtype=torch.int8, device=dev, generator=g)
    xs = (torch.rand((K // 128, M), device=dev, generator=g) * 0.01).half()
    out = torch.empty((M, N), device=dev, dtype=torch.float16)
    for _ in range(reps):
        ops.gemm_w6ax(xq, xs, img, N, 8, out=out)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        ops.gemm_w6ax(xq, xs, img, N, 8, out=out)
    e.record()
    e.synchronize()
    t = s.elapsed_time(e) / reps * 1e3
    print(f"M={M} N={N} K={K}: {t:.1f} us {2.0 * M * N * K / t / 1e6:.1f} TOPS")


if __name__ == "__main__":
    main()
