"""Prefill GEMM ablations (development tool; needs abtmp/libflexq_hip_abl.so, `make -C
flexq_amd/csrc abl`).  FQ_DEV_ABLATION bits: 1 no dequant, 2 no MFMA, 4 no LDS reads,
8 no global loads / DMA, 16 no stores, 32 no A DMA, 64 no weight loads.  M >= 2048: the U8 path
(weights unpacked once per call) like the product.
usage: python tools/prefill_ablate.py M N K"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from flexq_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.environ.get("FQ_ABL_LIB", os.path.join(ROOT, "abtmp", "libflexq_hip_abl.so"))
from flexq_amd import ops  # noqa: E402


def main():
    M, N, K = (int(v) for v in sys.argv[1:4])
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    wq = torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g)
    ws = (torch.rand((K // 128, N), device=dev, generator=g) * 0.01).half()
    img = ops.pack_w6(wq, ws)
    xq = torch.randint(-128, 128, (M, K), dtype=torch.int8, device=dev, generator=g)
    xs = (torch.rand((K // 128, M), device=dev, generator=g) * 0.01).half()
    out = torch.empty((M, N), device=dev, dtype=torch.float16)
    for m in [int(v) for v in os.environ.get("FQ_ABL_LIST", "0,1,2,3,4,5,6,7,8,12,16,17,19").split(",")]:
        os.environ["FQ_DEV_ABLATION"] = str(m)
        for _ in range(3):
            ops.gemm_w6ax(xq, xs, img, N, 8, out=out)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(5):
            ops.gemm_w6ax(xq, xs, img, N, 8, out=out)
        e.record()
        e.synchronize()
        t = s.elapsed_time(e) / 5 * 1e3
        print(f"M={M} N={N} K={K} abl{m}: {t:8.1f} us {2.0 * M * N * K / t / 1e6:7.1f} TOPS", flush=True)


if __name__ == "__main__":
    main()
