"""Prefill (M > 32) W6A8 GEMM throughput vs hipBLASLt (development tool).
For each LLaMA-3-8B shape at M tokens: fq_gemm_w6ax (pre-quantized int8 X), fq_linear_w6ax
(quantize + GEMM), torch fp16 F.linear and torch._int_mm (int8 x int8 -> int32)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from flexq_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.environ.get("FQ_LIB", _lib.LIB_PATH)  # development variants (tools/libflexq_*.so)
from flexq_amd import ops  # noqa: E402

SHAPES = [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]


def timed(fn, reps=int(os.environ.get("FQ_REPS", "10"))):
    """us per call: the calls captured into one HIP graph (no host launch gaps), replayed after a
    warm-up replay; FQ_EAGER=1 times eager calls instead (the round-5 form, which put the first shape
    behind the GPU's clock ramp and the per-call host path)."""
    fn()
    torch.cuda.synchronize()
    if os.environ.get("FQ_EAGER") == "1":
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        e.synchronize()
        return s.elapsed_time(e) / reps * 1e3  # us
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):  # (workspaces are per stream: grow this one before the capture)
        fn()
    st.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) / reps * 1e3)
    return best


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    a = torch.randn((8192, 8192), device=dev, dtype=torch.float16)
    for _ in range(200):  # ~1 s of GEMMs first: the clocks are up before the first shape is timed
        a = torch.nn.functional.linear(a, a) * 1e-3
    torch.cuda.synchronize()
    del a
    for (N, K) in SHAPES:
        wq = torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g)
        ws = (torch.rand((K // 128, N), device=dev, generator=g) * 0.01).half()
        img = ops.pack_w6(wq, ws)
        x = torch.randn((M, K), device=dev, dtype=torch.float16, generator=g)
        xq, xs = ops.quantize_act(x, 8)
        out = torch.empty((M, N), device=dev, dtype=torch.float16)
        t_gemm = timed(lambda: ops.gemm_w6ax(xq, xs, img, N, 8, out=out))
        t_lin = timed(lambda: ops.linear_w6ax(x, img, N, 8, out=out))
        wf = torch.randn((N, K), device=dev, dtype=torch.float16, generator=g)
        t_f16 = timed(lambda: torch.nn.functional.linear(x, wf))
        t_i8 = timed(lambda: torch._int_mm(xq, wq.t()))
        ops_ = 2.0 * M * N * K
        print(f"M={M} N={N:6d} K={K:6d}: w6a8 gemm {t_gemm:9.1f} us {ops_ / t_gemm / 1e6:7.1f} TOPS | "
              f"linear {t_lin:9.1f} us | fp16 {t_f16:9.1f} us {ops_ / t_f16 / 1e6:7.1f} TFLOPS | "
              f"int8 _int_mm {t_i8:9.1f} us {ops_ / t_i8 / 1e6:7.1f} TOPS", flush=True)
        del wq, img, x, xq, wf


if __name__ == "__main__":
    main()
