"""Where a group step of the 256 x 256 prefill kernel spends its cycles (development tool;
abtmp/libflexq_hip_abl.so, FQ_DEV_ABLATION = 128 + 32).  Per wave of the first 256 workgroups,
s_memtime sums of four segments of every group step: the barrier wait, the stage DMA issue (waves
4-7 issue it all), the compute (LDS reads, MFMAs, dequant) and the trailing wait for the next
stage.  Prints cycles per group step by wave, averaged over the workgroups.  The stamps fence the
segments (no overlap across them), so read the shares, not the total.
usage: python tools/pb_stamps.py [M N K]   (FQ_PB_ABL=1|2|4|8: stamps of an ablated build -- no dequant,
no MFMA, no LDS fragment reads, no DMA)"""
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


def main():
    M, N, K = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (16384, 28672, 4096)
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    abl = int(os.environ.get("FQ_PB_ABL", "0"))
    os.environ["FQ_DEV_ABLATION"] = str(160 + abl)
    L = _lib.load()
    L.fq_dev_pb_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    wq = torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g)
    img = ops.pack_w6(wq, (torch.rand((K // 128, N), device=dev, generator=g) * 0.01).half())
    x = torch.randn((M, K), device=dev, dtype=torch.float16, generator=g)
    xq, xs = ops.quantize_act(x, 8)
    out = torch.empty((M, N), device=dev, dtype=torch.float16)
    for _ in range(3):
        ops.gemm_w6ax(xq, xs, img, N, 8, out=out)
    torch.cuda.synchronize()
    buf = np.zeros(256 * 8 * 4, np.uint64)
    L.fq_dev_pb_stamps(buf.ctypes.data, buf.size)
    st = buf.reshape(256, 8, 4).astype(np.float64) / (K // 128)
    names = ["barrier", "stage-issue", "compute", "dma-wait"]
    print(f"M={M} N={N} K={K} ablation={abl}: s_memtime cycles per group step (mean over 256 WGs)")
    for w in range(8):
        row = " ".join(f"{names[k]}={st[:, w, k].mean():7.0f}" for k in range(4))
        print(f"  wave {w}: {row}  total={st[:, w, :].sum(axis=1).mean():7.0f}")


if __name__ == "__main__":
    main()
