"""32 < M <= 256 (development tool, abtmp/libflexq_hip_abl.so): the decode kernel in row chunks of
32 (FQ_DEV_MIDM=1) against the 128 x 128 prefill kernel with split-K (FQ_DEV_MIDM=0).  Per shape:
int32 group accumulators identical and outputs within 1e-3 relative between the two paths, then
graph-timed GEMM launches (24 per graph over rotating weight copies, as tools/shape_sweep.py).
usage: python tools/midm_sweep.py [M ...]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from flexq_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.environ.get("FQ_LIB", os.path.join(ROOT, "abtmp", "libflexq_hip_abl.so"))
from flexq_amd import ops  # noqa: E402

SHAPES = [(4096, 4096), (12288, 4096), (22016, 4096), (4096, 11008)]


def timed(M, N, K, imgs, xq, xs, out, R=24):
    stream = torch.cuda.Stream()
    ops.reserve_workspace(xq.device, [(M, N, K)], stream)
    with torch.cuda.stream(stream):
        for i in range(len(imgs)):
            ops.gemm_w6ax(xq, xs, imgs[i], N, 8, out=out)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=stream):
        for i in range(R):
            ops.gemm_w6ax(xq, xs, imgs[i % len(imgs)], N, 8, out=out)
    g.replay()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()  # replay() launches on the current stream
        g.replay()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) * 1e3 / R)
    return best


def main():
    Ms = [int(v) for v in sys.argv[1:]] or [33, 48, 64, 96, 128, 192, 256]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    for (N, K) in SHAPES:
        copies = max(2, min(8, int(2.5e9 // (N * K))))
        imgs = []
        for _ in range(copies):
            wq = torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g)
            imgs.append(ops.pack_w6(wq, (torch.rand((K // 128, N), device=dev, generator=g) * 0.01).half()))
        for M in Ms:
            xq = torch.randint(-128, 128, (M, K), dtype=torch.int8, device=dev, generator=g)
            xs = (torch.rand((K // 128, M), device=dev, generator=g) * 0.01).half()
            res = {}
            for mode in ("0", "1"):
                os.environ["FQ_DEV_MIDM"] = mode
                d, acc = ops.gemm_w6ax(xq, xs, imgs[0], N, 8, return_acc=True)
                out = torch.empty((M, N), dtype=torch.float16, device=dev)
                res[mode] = (d.float(), acc, timed(M, N, K, imgs, xq, xs, out))
            same_acc = torch.equal(res["0"][1], res["1"][1])
            a, b = res["0"][0], res["1"][0]
            ok = bool(((a - b).abs() <= 1e-3 * a.abs() + 1e-2).all())
            print(f"M={M:4d} N={N:6d} K={K:6d}: prefill {res['0'][2]:7.2f} us | chunked decode {res['1'][2]:7.2f} us"
                  f" | acc {'identical' if same_acc else 'DIFFER'} | out {'close' if ok else 'FAR'}", flush=True)
            if not (same_acc and ok):
                sys.exit(1)
        del imgs


if __name__ == "__main__":
    main()
