"""Decode chain timing (development tool): the bench's LLaMA-2-7B M = 1 step (bench.build_stack, the
same weights and dependency chain) as one HIP graph of
  launches  one fq_linear_w6ax launch per linear (the headline's form),
  layer     fq_linear_chain_w6ax over each run between attention cores: [qkv_0], [o_i, gate_up_i,
            down_i, qkv_i+1] (the model's boundaries: attention sits between qkv and o),
  chain8    runs of 8 consecutive linears regardless of where attention would sit (information only),
checking that the three give bit-identical step outputs.  Usage: python tools/chain_bench.py [reps] [config]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from flexq_amd import ops  # noqa: E402


def main():
    if os.environ.get("FQ_CHAIN_OLDABI"):  # (A/B against a build from before the producer links: plain links only)
        import ctypes

        class OldLink(ctypes.Structure):
            _fields_ = [("x", ctypes.c_void_p), ("w_packed", ctypes.c_void_p), ("d", ctypes.c_void_p),
                        ("N", ctypes.c_int), ("K", ctypes.c_int), ("abits", ctypes.c_int)]

            def __init__(self, x=None, w_packed=None, d=None, N=0, K=0, abits=0, **_kw):
                super().__init__(x, w_packed, d, N, K, abits)
        ops._ChainLink = OldLink
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    cfg_name = sys.argv[2] if len(sys.argv) > 2 else "llama2-7b-m1"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = bench.CONFIGS[cfg_name]
    M = cfg[1]
    stack = bench.build_stack(cfg, 0, 1, dev, merge=True)
    lins = bench.linears(stack)
    links = [(p["x"], p["pk"], p["Nl"], p["abits"], p["out"]) for _, p in lins]
    layer_runs, cur = [], []
    for (name, _), l in zip(lins, links):
        if name in ("o", "o_proj") and cur:
            layer_runs.append(cur)
            cur = []
        cur.append(l)
    layer_runs.append(cur)
    runs8 = [links[i:i + 8] for i in range(0, len(links), 8)]
    forms = {
        "launches": lambda: bench.run_step(stack, M, 1),
        "layer": lambda: [ops.linear_chain_w6ax(r) for r in layer_runs],
        "chain8": lambda: [ops.linear_chain_w6ax(r) for r in runs8],
    }
    s = torch.cuda.Stream(dev)
    ops.reserve_workspace(dev, [(M, p["Nl"], p["K"]) for _, p in lins] + [(M, 1, 128 * 2048)], stream=s)
    outs, times = {}, {}
    for rep in range(3):  # alternate the forms, three rounds
        for name, fn in forms.items():
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                fn()
            s.synchronize()
            g = bench.capture(fn, s)
            for _ in range(3):
                g.replay()
            torch.cuda.synchronize()
            t = bench.time_graph(g, reps, s) / reps
            times.setdefault(name, []).append(t * 1e3)
            outs[name] = links[-1][4].cpu().numpy().view(np.uint16).copy()
            del g
    for name in forms:
        same = np.array_equal(outs[name], outs["launches"])
        print(f"{name:9s} ms/step {' '.join(f'{v:.4f}' for v in times[name])}  bit-identical: {same}"
              f"  launches/step: {len(links) if name == 'launches' else len(layer_runs) if name == 'layer' else len(runs8)}")
    print("chain error word:", ops.chain_error(dev, stream=s))


if __name__ == "__main__":
    main()
