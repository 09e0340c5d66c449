"""C3 (LLaMA-2-7B, batch 16) step: the separate quantize launch per linear against the next input's
quantizer in the decode GEMM's epilogue (fq_gemm_w6ax_q), both as one HIP graph, alternated in one
process (development tool; bench.py's c3 section takes the faster, bit-identical form).
usage: python tools/c3_qe_ab.py [reps] [M]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from flexq_amd import ops  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    M = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    dev = torch.device("cuda:0")
    layers, _, lins, desc = bench.CONFIGS["llama2-7b-m16"]
    cfg = (layers, M, lins, desc)
    stack = bench.build_stack(cfg, 0, 1, dev, True)
    s = torch.cuda.Stream(dev)
    forms = {"separate": lambda: bench.run_step(stack, M, 1), "epilogue": lambda: bench.run_step_qo(stack, M)}
    graphs, outs = {}, {}
    last = bench.linears(stack)[-1][1]["out"]
    for k, fn in forms.items():
        with torch.cuda.stream(s):
            fn()
        torch.cuda.synchronize()
        graphs[k] = bench.capture(fn, s)
        graphs[k].replay()
        torch.cuda.synchronize()
        outs[k] = last.clone()
    same = torch.equal(outs["separate"].view(torch.int16), outs["epilogue"].view(torch.int16))
    print(f"M={M}: last output bit-identical between the forms: {same}", flush=True)
    for r in range(reps):
        row = []
        for k, g in graphs.items():
            for _ in range(3):
                g.replay()
            t = bench.time_graph(g, 20, s) / 20
            row.append(f"{k} {t * 1e3:.4f} ms")
        print(f"rep {r} (graph): " + " | ".join(row), flush=True)
    for r in range(reps):  # eager launches: the host's per-launch cost is in the step
        row = []
        for k, fn in forms.items():
            with torch.cuda.stream(s):
                for _ in range(3):
                    fn()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                for _ in range(10):
                    fn()
                b.record(s)
            b.synchronize()
            row.append(f"{k} {a.elapsed_time(b) / 10:.4f} ms")
        print(f"rep {r} (eager): " + " | ".join(row), flush=True)
    if not same:
        sys.exit(1)


if __name__ == "__main__":
    main()
