"""Producer-in-GEMM timings (development tool): per-launch microseconds of a graph of R dependent
decode calls, M = 1, for the LLaMA-2-7B shapes that follow a producer --
  qkv / gate_up (K = 4096): linear_w6ax | rmsnorm_linear_w6ax (fused) | rmsnorm_quantize + gemm
  down (K = 11008):         linear_w6ax | silu_linear_w6ax (fused)    | silu_mul_quantize + gemm
over rotating weight copies (cold images).  usage: python tools/fusedpro_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flexq_amd import ops  # noqa: E402


def timed(fn, R, stream):
    with torch.cuda.stream(stream):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            fn()
        g.replay()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(5):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record(stream)
            g.replay()
            e.record(stream)
            e.synchronize()
            best = min(best, s.elapsed_time(e) * 1e3 / R)
    return best


def main():
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev).manual_seed(0)
    stream = torch.cuda.Stream()
    R = 24
    for (N, K, kind) in [(12288, 4096, "norm"), (22016, 4096, "norm"), (4096, 4096, "norm"), (4096, 11008, "silu")]:
        copies = max(2, min(8, int(2.5e9 // (N * K))))
        imgs = [ops.pack_w6(torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=gen),
                            (torch.rand((K // 128, N), device=dev, generator=gen) * 0.01).half()) for _ in range(copies)]
        x = torch.randn((1, K), device=dev, dtype=torch.float16, generator=gen)
        gamma = torch.ones(K, device=dev, dtype=torch.float16)
        res = [torch.randn((1, K), device=dev, dtype=torch.float16, generator=gen) for _ in range(2)]
        gu = torch.randn((1, 2 * K), device=dev, dtype=torch.float16, generator=gen)
        out = torch.empty((1, N), device=dev, dtype=torch.float16)
        ab = 6 if kind == "norm" else 8
        rows = {"linear": lambda: [ops.linear_w6ax(x, imgs[i % copies], N, ab, out=out) for i in range(R)]}
        if kind == "norm":
            def fused():
                for i in range(R):
                    ops.rmsnorm_linear_w6ax(res[i & 1], gamma, imgs[i % copies], N, 6, input=x,
                                            residual_out=res[(i + 1) & 1], out=out)

            def split():
                for i in range(R):
                    xq, xs = ops.rmsnorm_quantize(res[0], gamma, 6, input=x)
                    ops.gemm_w6ax(xq, xs, imgs[i % copies], N, 6, out=out)
        else:
            def fused():
                for i in range(R):
                    ops.silu_linear_w6ax(gu[:, :K], gu[:, K:], imgs[i % copies], N, 8, out=out)

            def split():
                for i in range(R):
                    xq, xs = ops.silu_mul_quantize(gu[:, :K], gu[:, K:], 8)
                    ops.gemm_w6ax(xq, xs, imgs[i % copies], N, 8, out=out)
        rows["fused_" + kind] = fused
        rows["producer+gemm"] = split
        print(f"N={N:6d} K={K:6d} " + "  ".join(f"{k}={timed(f, R, stream):6.2f}us" for k, f in rows.items()), flush=True)


if __name__ == "__main__":
    main()
