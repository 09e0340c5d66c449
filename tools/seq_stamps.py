"""Chain-kernel timeline (development tool; tools/libflexq_hip_abl.so built with -DFQ_DEV_ABLATION).

Runs the bench's LLaMA-2-7B M=1 step as one fq_linear_seq launch and prints, per linear kind,
medians over layers (us, s_memrealtime at 100 MHz) of:
  handoff  last arrival of linear j-1  -> this WG released past B2 (median / max over WGs)
  quant    B2 -> x quantized (wave 0)
  first    x quantized -> first ring block landed (wave 0)
  stream   first block -> wave 0 stream done; spread = max - min over WGs of stream done
  epi      last stream done in the WG -> its arrival returned (reduce + sc1 stores + drain + add)
  span     last arrival of j-1 -> last arrival of j  (the linear's share of the step)
FQ_SEQ_KNOB: 1 = no dependency waits, 2 = no deep prefetch (3 slots)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from flexq_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(ROOT, "tools", "libflexq_hip_abl.so")
import bench  # noqa: E402

SL = 160


def main():
    dev = torch.device("cuda:0")
    cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "llama2-7b-m1"]
    layers = min(cfg[0], SL // 4)
    cfg = (layers,) + cfg[1:]
    L = _lib.load()
    L.fq_dev_seq_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    stack = bench.build_stack(cfg, 0, 1, dev)
    seq = bench.make_seq(stack)
    names = [n for n, _ in bench.linears(stack)]
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream):
        for _ in range(3):
            seq.run()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=stream):
        seq.run()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(stream):
        s.record(stream)
        for _ in range(10):
            g.replay()
        e.record(stream)
    e.synchronize()
    step_us = s.elapsed_time(e) / 10 * 1e3
    g.replay()
    torch.cuda.synchronize()
    grid = seq.plan.grid
    n = len(names)
    buf = np.zeros(256 * SL * 8, dtype=np.uint64)
    assert L.fq_dev_seq_stamps(buf.ctypes.data, buf.size) == 0
    st = buf.reshape(256, SL, 8)[:grid, :n].astype(np.float64) / 100.0  # us
    t0 = st[:, 0, 0].min()
    st -= t0
    arr_last = st[:, :, 2].max(axis=0)
    drain = np.median(st[:, :, 7] - np.maximum(st[:, :, 1], 0), axis=0)
    print(f"step {step_us:.1f} us (graph), kernel span {arr_last[-1]:.1f} us, {n} linears, grid {grid}, "
          f"slots {seq.plan.slots}, knob {os.environ.get('FQ_SEQ_KNOB', '0')}")
    rows = {}
    for j in range(n):
        prev = arr_last[j - 1] if j else 0.0
        rel = st[:, j, 0] - prev
        stream_done = np.maximum(st[:, j, 5], st[:, j, 6])
        d = dict(handoff=np.median(rel), handoff_max=rel.max(),
                 quant=np.median(st[:, j, 3] - st[:, j, 0]),
                 first=np.median(st[:, j, 4] - st[:, j, 3]),
                 stream=np.median(st[:, j, 5] - st[:, j, 4]),
                 spread=stream_done.max() - stream_done.min(),
                 epi=np.median(st[:, j, 2] - stream_done),
                 red_drain=np.median(st[:, j, 7] - st[:, j, 1]),
                 span=arr_last[j] - prev)
        rows.setdefault(names[j], []).append(d)
    keys = ["handoff", "handoff_max", "quant", "first", "stream", "spread", "epi", "red_drain", "span"]
    print(f"{'linear':10s}" + "".join(f"{k:>12s}" for k in keys))
    for name, lst in rows.items():
        print(f"{name:10s}" + "".join(f"{np.median([r[k] for r in lst]):12.2f}" for k in keys))


if __name__ == "__main__":
    main()
