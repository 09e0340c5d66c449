"""Development probe: the decode linear's launch time when its weight image is resident in the
Infinity Cache (graph of launches on ONE image) against a cold stream (rotating over copies far
beyond 256 MiB).  Measured: hot within 1-10 % of cold for every cache policy of the
weight DMA, so the launch is not bound by where its bytes come from; a side-stream prefetch of
the next linear's image (a removed experiment) only added HBM traffic."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from flexq_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.environ.get("FQ_LIB", _lib.LIB_PATH)  # development variants (tools/libflexq_*.so)
from flexq_amd import ops  # noqa: E402


def graph_us(fn, reps=5, launches=20):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s):
        a.record(s)
        for _ in range(reps):
            g.replay()
        b.record(s)
    b.synchronize()
    return a.elapsed_time(b) * 1e3 / (reps * launches)


def main():
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev).manual_seed(0)
    L = 20
    for (N, K) in [(12288, 4096), (4096, 4096), (22016, 4096), (4096, 11008)]:
        copies = max(2, (1536 << 20) // (N * K * 3 // 4))
        pks = [ops.pack_w6(torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=gen),
                           (torch.rand((K // 128, N), device=dev, generator=gen) * 0.01).half()) for _ in range(copies)]
        x = torch.randn((1, K), dtype=torch.float16, device=dev, generator=gen)
        out = torch.empty((1, N), dtype=torch.float16, device=dev)
        hot = graph_us(lambda: [ops.linear_w6ax(x, pks[0], N, 6, out=out) for _ in range(L)])
        cold = graph_us(lambda: [ops.linear_w6ax(x, pks[i % copies], N, 6, out=out) for i in range(L)])
        mb = pks[0].numel() / 1e6
        print(f"N={N:5d} K={K:5d} {mb:5.1f} MB  hot {hot:6.2f} us ({mb / hot:5.2f} TB/s)  cold {cold:6.2f} us "
              f"({mb / cold:5.2f} TB/s)", flush=True)
        del pks


if __name__ == "__main__":
    main()
