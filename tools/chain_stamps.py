"""Decode-chain timeline (development tool; abtmp/libflexq_hip_abl.so).  Runs the bench's layer
chain (o -> gate_up -> down -> qkv, LLaMA-2-7B, M = 1, each input the leading K values of the previous
output) in a graph, then reads the per-(WG, linear) wave-0 stamps (s_memrealtime, 100 MHz): 0 linear
start, 1 ring issued (a linear after the first: its prologue; the ring itself went out from the
previous linear's tail, stamp 7 there), 2 input quantized (after the in-kernel wait), 3 first block
landed, 4 stream done (its output granules stored), 5 linear end, 6 the poll's first pass matched.  Prints, per linear, medians and spreads over the WGs (us, from the launch's
first stamp) and the hand-off: from the last WG's stream end of linear l to each WG's input-ready
time of linear l + 1.  FQ_STAMPS_PRO=1: the decoder layer's producer chain instead (o -> RMSNorm +
gate_up -> SiLU * up + down -> RMSNorm + qkv, layers.run_layers_chained's links)."""
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

SHAPES = [("o", 4096, 4096, 6), ("gate_up", 22016, 4096, 6), ("down", 4096, 11008, 6), ("qkv", 12288, 4096, 6)]


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    L = _lib.load()
    L.fq_dev_chain_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    NL, NS = 8, 8
    x0 = torch.randn((1, 4096), dtype=torch.float16, device=dev, generator=g)
    chains = []
    for c in range(6):  # rotating weight sets (cold images, as in the step)
        links, prev = [], x0
        imgs, outs = [], []
        for (_, N, K, ab) in SHAPES:
            wq = torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g)
            ws = ((torch.rand((K // 128, N), device=dev, generator=g) + 0.5) / (18.5 * 1.04 * K ** 0.5)).half()
            out = torch.empty((1, N), dtype=torch.float16, device=dev)
            x = prev if prev is x0 else prev.view(-1)[:K].view(1, K)
            links.append((x, ops.pack_w6(wq, ws), N, ab, out))
            imgs.append(links[-1][1])
            outs.append(out)
            prev = out
        if os.environ.get("FQ_STAMPS_PRO"):
            F = 11008
            gam = [torch.rand((4096,), dtype=torch.float16, device=dev, generator=g) + 0.5 for _ in range(2)]
            res = [torch.randn((1, 4096), dtype=torch.float16, device=dev, generator=g) for _ in range(3)]
            gu = outs[1]
            links = [links[0],
                     ops.chain_rmsnorm(res[0], gam[0], imgs[1], 22016, 6, gu, input=outs[0], residual_out=res[1]),
                     ops.chain_silu(gu[:, :F], gu[:, F:], imgs[2], 4096, 6, outs[2]),
                     ops.chain_rmsnorm(res[1], gam[1], imgs[3], 12288, 6, outs[3], input=outs[2], residual_out=res[2])]
        chains.append(links)
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        for ch in chains:
            ops.linear_chain_w6ax(ch)
    s.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        for i in range(12):
            ops.linear_chain_w6ax(chains[i % len(chains)])
    for _ in range(3):
        graph.replay()
    torch.cuda.synchronize()
    st = (ctypes.c_ulonglong * (1024 * NL * NS))()
    assert L.fq_dev_chain_stamps(st, 1024 * NL * NS) == 0
    a = np.frombuffer(st, dtype=np.uint64).reshape(1024, NL, NS)[:256, :len(SHAPES), :8].astype(np.int64)
    t0 = a[:, 0, 0].min()
    us = (a - t0) / 100.0  # 100 MHz -> us
    print("per linear (us from the launch's first stamp): median over WGs [min .. max]")
    names = ["start", "ring issued", "quantized", "first block", "stream done", "end"]
    for li, (name, N, K, _) in enumerate(SHAPES):
        row = "  ".join(f"{nm} {np.median(us[:, li, k]):7.2f} [{us[:, li, k].min():6.2f}..{us[:, li, k].max():6.2f}]"
                        for k, nm in enumerate(names))
        print(f"{name:8s} {N:6d}x{K:<6d} {row}")
    for li in range(1, len(SHAPES)):
        last = us[:, li - 1, 4].max()
        ready = us[:, li, 2]
        print(f"hand-off {SHAPES[li - 1][0]} -> {SHAPES[li][0]}: last producer stream done {last:7.2f}; "
              f"input quantized median {np.median(ready) - last:+.2f} [{ready.min() - last:+.2f} .. {ready.max() - last:+.2f}] us; "
              f"consumer first block {np.median(us[:, li, 3]) - last:+.2f}; ring issued (median) {np.median(us[:, li, 1]) - last:+.2f}")
    print("launch span", f"{us[:, len(SHAPES) - 1, 5].max():.2f} us")
    # the workgroups holding an extra tile of the widest link (bid < N_tiles % grid) against the rest
    wide = max(range(len(SHAPES)), key=lambda li: SHAPES[li][1])
    ir = ((SHAPES[wide][1] + 15) // 16) % 256
    if ir:
        print(f"by workgroup: bid < {ir} (an extra {SHAPES[wide][0]} tile) vs the rest, medians (us)")
        for li, (name, N, K, _) in enumerate(SHAPES):
            row = "  ".join(f"{nm} {np.median(us[:ir, li, k]):7.2f} / {np.median(us[ir:, li, k]):7.2f}"
                            for k, nm in enumerate(names) if k in (0, 3, 4))
            print(f"{name:8s} {row}")
    if os.environ.get("FQ_STAMPS_RAW"):
        np.save(os.environ["FQ_STAMPS_RAW"], us)
    if not os.environ.get("FQ_STAMPS_PRO"):  # plain chain: 6 = the first poll pass matched, 7 = next ring issued (tail)
        for li in range(1, len(SHAPES)):
            last = us[:, li - 1, 4].max()
            tail = us[:, li - 1, 7]
            print(f"edge {SHAPES[li - 1][0]} -> {SHAPES[li][0]}: last producer stream done {last:7.2f}; next ring issued "
                  f"(tail) median {np.median(tail) - last:+.2f}; consumer poll done median {np.median(us[:, li, 6]) - last:+.2f} "
                  f"[{us[:, li, 6].min() - last:+.2f} .. {us[:, li, 6].max() - last:+.2f}]; input quantized "
                  f"{np.median(us[:, li, 2]) - last:+.2f}; first block {np.median(us[:, li, 3]) - last:+.2f} us")
    if os.environ.get("FQ_STAMPS_PRO"):  # 6: both sources arrived (poll done), 7: RMSNorm's barrier passed
        for li in range(1, len(SHAPES)):
            p6, p7 = us[:, li, 6], us[:, li, 7]
            print(f"{SHAPES[li][0]:8s} ring issued -> poll done {np.median(p6 - us[:, li, 1]):+.2f}  "
                  f"poll done -> barrier {np.median(p7 - p6) if p7.max() > 0 else float('nan'):+.2f}  "
                  f"-> quantized {np.median(us[:, li, 2] - (p7 if p7.max() > 0 else p6)):+.2f}")


if __name__ == "__main__":
    main()
