"""Decode-chain soak test (development tool): the bench's LLaMA-2-7B M = 1 step as layer chains
(tools/chain_bench.py's `layer` form) replayed as a HIP graph for a fixed wall time, the step's
last output compared bit for bit with the per-linear launches' every `check` replays, and the
chain's error word read at the end.  A hand-off race (a stale granule taken for a fresh one) would
show as a mismatch; a lost arrival as a timed-out wait.  Usage: python tools/chain_stress.py
[seconds] [check]"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from flexq_amd import ops  # noqa: E402


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 60.0
    check = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = bench.CONFIGS["llama2-7b-m1"]
    stack = bench.build_stack(cfg, 0, 1, dev, merge=True)
    lins = bench.linears(stack)
    links = [(p["x"], p["pk"], p["Nl"], p["abits"], p["out"]) for _, p in lins]
    runs, cur = [], []
    for (name, _), l in zip(lins, links):
        if name in ("o", "o_proj") and cur:
            runs.append(cur)
            cur = []
        cur.append(l)
    runs.append(cur)
    s = torch.cuda.Stream(dev)
    ops.reserve_workspace(dev, [(1, p["Nl"], p["K"]) for _, p in lins] + [(1, 1, 128 * 2048)], stream=s)
    last = links[-1][4]
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        bench.run_step(stack, 1, 1)
    s.synchronize()
    ref = last.cpu().numpy().view(np.uint16).copy()
    fn = lambda: [ops.linear_chain_w6ax(r) for r in runs]  # noqa: E731
    with torch.cuda.stream(s):
        fn()
    s.synchronize()
    g = bench.capture(fn, s)
    t0, reps, bad, last_print = time.time(), 0, 0, time.time()
    while time.time() - t0 < seconds:
        for _ in range(check):
            g.replay()
        reps += check
        s.synchronize()
        if not np.array_equal(last.cpu().numpy().view(np.uint16), ref):
            bad += 1
        if time.time() - last_print > 20:
            print(f"  {reps} steps, {bad} mismatching checks", flush=True)
            last_print = time.time()
    err = ops.chain_error(dev, stream=s)
    print(f"chain soak: {reps} steps ({reps * len(runs)} chain launches) in {time.time() - t0:.1f} s, "
          f"{reps // check} checks, mismatches {bad}, chain error word {err}")
    sys.exit(1 if bad or err else 0)


if __name__ == "__main__":
    main()
