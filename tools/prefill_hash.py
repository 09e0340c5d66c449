"""Hash of the prefill GEMM outputs (development tool: bit-identity of variant libraries, FQ_LIB).
Prints one sha256 per shape of fq_gemm_w6ax's fp16 output on seeded inputs (the 256 x 256 path and
a ragged one).
usage: FQ_LIB=abtmp/libflexq_hip_x.so python tools/prefill_hash.py"""
import hashlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from flexq_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.environ.get("FQ_LIB", _lib.LIB_PATH)
from flexq_amd import ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    for (M, N, K) in [(4096, 4096, 4096), (4000, 4104, 1024), (2048, 28672, 512)]:
        g = torch.Generator(device=dev).manual_seed(M + N + K)
        wq = torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g)
        ws = (torch.rand((K // 128, N), device=dev, generator=g) * 0.01).half()
        img = ops.pack_w6(wq, ws)
        x = torch.randn((M, K), device=dev, dtype=torch.float16, generator=g)
        xq, xs = ops.quantize_act(x, 8)
        out = ops.gemm_w6ax(xq, xs, img, N, 8)
        torch.cuda.synchronize()
        h = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]
        print(f"M={M} N={N} K={K} sha={h} lib={os.path.basename(_lib.LIB_PATH)}")


if __name__ == "__main__":
    main()
