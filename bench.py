"""bench.py -- W6A6 linear-stack throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): LLaMA-2-7B, every linear layer of all 32 decoder layers,
W6A6 group 128, batch 1 (M = 1), random-init weights of that architecture, synthetic fp16
activations resident in HBM.  One "step" = one token through the 32-layer linear stack: per
layer 5 W6A6 linears (qkv 12288x4096, o 4096x4096, gate/up 11008x4096 reading the same input,
down 4096x11008), each = dynamic activation quantization + GEMM + dequant.  The linears form a
dependency chain as in decoding (each reads the previous one's output).  gate and up share their
input, so by default they run as one linear over the concatenated weight image [gate; up]
(22016x4096, output [gate | up], per-column arithmetic unchanged): 4 linears per layer
(--no-merge: 5), one fq_linear_w6ax launch each (at decode sizes a single fused quantize+GEMM
launch), the whole step captured into one HIP graph.

Multi-GPU (one process per GPU; `--gpus N` starts the N ranks itself through a child torchrun
when it is not already under one): by default (`--parallel c4`) `value` is the north-star split,
BASELINE config C4: the LLaMA-2-70B linear stack with every linear column-parallel over the N GPUs
(each rank packs and streams only its N/P rows, ONE all-gather per linear
assembles the dequantized fp16 output over xGMI -- RCCL's all_gather, or the peer-store gather
fused into the GEMM epilogue when every rank's output is bit-identical to the RCCL run's and it is
faster); total work fixed, "scaling": "strong".  C4's one-GPU point is the N = 1 line's
`c4_llama2_70b_1gpu` section (the N = 1 `value` stays BASELINE configs[1], LLaMA-2-7B).  Beside
it: the same split of the 7B stack (`tp_llama2_7b`, `tp_llama2_7b_peer_gather`) and the 7B stack as
independent replicas, one token stream per GPU (`replicas`, weak scaling).  `--parallel tp` /
`--parallel dp` make the 7B split / the replicas the `value` instead.

Output: one JSON line (rank 0) with the metric, the roofline of the dominant kernel (the decode
linear), the north-star comparison against rocBLAS/hipBLASLt fp16 GEMM, and the CPU baseline (the oracle's restatement of the reference's fake-quant QuantLinear
forward, timed on a bounded sample on this host).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
from flexq_amd import ops  # noqa: E402

GROUP = 128
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
I8_MFMA_PEAK_TOPS = 5000.0  # dense int8 MFMA (2x the 2.5 PF dense bf16)

CONFIGS = {
    # name: (layers, M, [(linear, N, K, abits)], description)
    "llama2-7b-m1": (32, 1, [("qkv", 12288, 4096, 6), ("o", 4096, 4096, 6), ("gate", 11008, 4096, 6),
                             ("up", 11008, 4096, 6), ("down", 4096, 11008, 6)],
                     "LLaMA-2-7B all linear shapes, W6A6 g128, batch 1"),
    "llama2-7b-m16": (32, 16, [("qkv", 12288, 4096, 6), ("o", 4096, 4096, 6), ("gate", 11008, 4096, 6),
                               ("up", 11008, 4096, 6), ("down", 4096, 11008, 8)],
                      "LLaMA-2-7B, W6A6 + W6A8 down_proj, batch 16"),
    "llama2-70b-m1": (80, 1, [("qkv", 10240, 8192, 6), ("o", 8192, 8192, 6), ("gate", 28672, 8192, 6),
                              ("up", 28672, 8192, 6), ("down", 8192, 28672, 6)],
                      "LLaMA-2-70B all linear shapes (GQA qkv), W6A6 g128, batch 1"),
    # C5: prefill, seq 2048 x batch 8; every linear W6A8
    "llama3-8b-prefill": (32, 16384, [("qkv", 6144, 4096, 8), ("o", 4096, 4096, 8), ("gate", 14336, 4096, 8),
                                      ("up", 14336, 4096, 8), ("down", 4096, 14336, 8)],
                          "LLaMA-3-8B all linear shapes, W6A8 g128, prefill seq 2048 x batch 8 (M = 16384)"),
}
PREFILL_M = 32  # above this the linear runs quantize + the MFMA-bound prefill GEMM (two launches)


def alg_bytes(M, N, K, abits, fused=True):
    """Algorithmic HBM bytes of one linear launch: packed W (0.75 B/w) + W
    scales (2 B per 128 weights, inside the weight image) + the activations + fp16 D.  Fused (decode) launches read fp16 x (2 B/elem) and quantize
    in-kernel; unfused ones read int8 X + X scales (their quantize launch is bytes_quant)."""
    act = 2 * M * K if fused else M * K + 2 * M * K // GROUP
    return N * K * 6 // 8 + 2 * N * K // GROUP + act + 2 * M * N


def alg_read_bytes(M, N, K, abits, fused=True):
    """The read part of alg_bytes (everything but the 2*M*N fp16 output): what rocprofv3's
    FETCH_SIZE (a read counter) is compared with."""
    return alg_bytes(M, N, K, abits, fused) - 2 * M * N


def fp16_bytes(M, N, K):
    """HBM bytes of one fp16 F.linear: the fp16 weight, the fp16 input and output."""
    return 2 * N * K + 2 * M * K + 2 * M * N


def launch_list(lins, merge):
    """The step's launches: (name, N, K, abits).  merge: gate and up, which read the same input,
    run as one linear over their concatenated weights (one image [2N, K]; output [gate | up])."""
    if not merge:
        return list(lins)
    out, gate = [], None
    for (name, N, K, abits) in lins:
        if name == "gate":
            gate = (N, K, abits)
        elif name == "up":
            assert gate and gate[1] == K and gate[2] == abits
            out.append(("gate_up", gate[0] + N, K, abits))
        else:
            out.append((name, N, K, abits))
    return out


def build_stack(cfg, rank, world, dev, merge=True, seed=1234, peer=False):
    """Random-init weights of the architecture and the step's data flow.  The linears form a real
    dependency chain, as in decoding: the input of each linear is the leading M*K values of the
    previous linear's output buffer (standing in for the out-of-scope attention / norm / SiLU
    between them; gate and up read the same input), so every linear waits for the one before.
    Weight scales give each linear unit gain, so values stay O(1) through all the layers."""
    layers, M, lins, _ = cfg
    g = torch.Generator(device=dev).manual_seed(seed + rank)
    stack = []
    prev = torch.randn((M * lins[0][2],), dtype=torch.float16, device=dev, generator=g)  # the token(s)
    x_first = prev
    shared = {}  # prefill: one output buffer per linear kind, reused by every layer (stream-ordered)
    gathers = {}  # peer-store gather (--gather peer): one PeerGather per full width, buffers alternate
    for _ in range(layers):
        L = {}
        for (name, N, K, abits) in launch_list(lins, merge):
            assert N % (16 * world) == 0, f"{name}: N={N} not divisible into 16-column shards for {world} ranks"
            Nl = N // world
            wq = torch.randint(-32, 32, (Nl, K), dtype=torch.int8, device=dev, generator=g)
            # codes have rms 18.5 and U(0.5, 1.5) has rms 1.04: unit gain per linear
            ws = ((torch.rand((K // GROUP, Nl), device=dev, generator=g) + 0.5) / (18.5 * 1.04 * K ** 0.5)).half()
            pk = ops.pack_w6(wq, ws)  # the weight image: 6-bit codes + blocked group scales
            del wq, ws
            if M > PREFILL_M:
                if name not in shared:
                    shared[name] = (torch.empty((M, Nl), dtype=torch.float16, device=dev),
                                    torch.empty((world * M * Nl,), dtype=torch.float16, device=dev)
                                    if world > 1 else None)
                out, full = shared[name]
            else:
                out = torch.empty((M, Nl), dtype=torch.float16, device=dev)
                full = torch.empty((world * M * Nl,), dtype=torch.float16, device=dev) if world > 1 else None
            src = prev if name != "up" else L["gate"]["x"].view(-1)
            x = src[:M * K].view(M, K)
            L[name] = dict(N=N, Nl=Nl, K=K, abits=abits, pk=pk, out=out, full=full, x=x)
            if M >= ops.PREFILL_U8_MIN_M:  # prefill: the weights' int8 MFMA operands kept resident
                L[name]["w_u8"] = ops.prepare_prefill_weights(pk, Nl, K)
            if peer and world > 1:
                from flexq_amd.dist import PeerGather
                if N not in gathers:
                    gathers[N] = [PeerGather(M, N, device=dev), 0]
                pg, uses = gathers[N]
                full = pg.bufs[uses & 1].view(-1)
                # fold this linear's wait for its input into its launch when the input is the previous
                # linear's gather buffer (merged gate_up: the chain is linear) and the buffers are uncached
                L[name].update(pg=pg, parity=uses & 1, full=full,
                               fold=bool(merge and pg.uncached and (stack or L) and name != "up"))
                gathers[N][1] = uses + 1
            if name != "gate":
                prev = (full if world > 1 else out).view(-1)
        stack.append(L)
    stack[0]["_input"] = x_first
    return stack


def linears(stack):
    return [(n, p) for L in stack for n, p in L.items() if not n.startswith("_")]


def run_step(stack, M, world, group=None, gather=True, staged=False):
    """One token through the linear stack, one launch per linear: fq_linear_w6ax (decode sizes:
    one fused quantize+GEMM launch each), then one RCCL all-gather of the fp16 shard outputs per
    linear when world > 1 (staged: through host memory, for the gloo rehearsal of --share-gpu)."""
    lins_ = linears(stack)
    for i, (name, p) in enumerate(lins_):
        if world > 1 and gather and "pg" in p:  # the all-gather fused into the GEMM epilogue
            # each linear reads the previous one's gather buffer: that gather's wait is folded into
            # this launch (after=...), only the step's last output gets a wait launch
            prev = lins_[i - 1][1] if i > 0 else None
            after = (prev["pg"], prev["parity"]) if prev is not None and "pg" in prev and p.get("fold") else None
            p["pg"].linear(p["x"], p["pk"], p["abits"], parity=p["parity"], after=after,
                           wait=not (i + 1 < len(lins_) and lins_[i + 1][1].get("fold")))
            continue
        ops.linear_w6ax(p["x"], p["pk"], p["Nl"], p["abits"], out=p["out"], w_u8=p.get("w_u8"))
        if world > 1 and gather:
            if staged:
                full = torch.empty(p["full"].shape, dtype=p["full"].dtype)
                dist.all_gather_into_tensor(full, p["out"].view(-1).cpu(), group=group)
                p["full"].copy_(full)
            else:
                dist.all_gather_into_tensor(p["full"], p["out"].view(-1), group=group)


def run_step_qo(stack, M):
    """The step with each linear's activation quantize moved into the previous GEMM's epilogue
    (ops.gemm_w6ax_q: fq_gemm_w6ax_u8_q at prefill sizes, fq_gemm_w6ax_q's decode form at M <= 16): the
    first input is quantized by its own launch, every later one by the GEMM that produces it -- the same
    codes as run_step's separate quantize launches (each linear's input is the leading M x K values of
    the previous output)."""
    lins_ = linears(stack)
    p0 = lins_[0][1]
    xq, xs = ops.quantize_act(p0["x"], p0["abits"])
    for i, (_, p) in enumerate(lins_):
        if i + 1 < len(lins_):
            nx = lins_[i + 1][1]
            assert nx["x"].data_ptr() == p["out"].data_ptr() and tuple(nx["x"].shape) == (M, nx["K"])
            _, xq, xs = ops.gemm_w6ax_q(xq, xs, p["pk"], p["Nl"], p["abits"], p.get("w_u8"), (M, nx["K"]),
                                        nx["abits"], out=p["out"])
        else:
            ops.gemm_w6ax(xq, xs, p["pk"], p["Nl"], p["abits"], out=p["out"], w_u8=p.get("w_u8"))


def chain_runs(stack):
    """The step's linears as decode chains (fq_linear_chain_w6ax), cut where the model's attention core
    sits: qkv_0 | o_0, gate_up_0, down_0, qkv_1 | o_1, ... -- the attention (out of scope) is a kernel of
    its own between qkv and o, so a chain never spans it; each chain is one persistent launch."""
    runs, cur = [], []
    for name, p in linears(stack):
        if name == "o" and cur:
            runs.append(cur)
            cur = []
        cur.append((p["x"], p["pk"], p["Nl"], p["abits"], p["out"]))
    runs.append(cur)
    return runs


def run_chains(runs):
    for r in runs:
        ops.linear_chain_w6ax(r)


def capture(fn, stream):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=stream):
        fn()
    return g


def time_graph(g, reps, stream):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(stream):
        s.record(stream)
        for _ in range(reps):
            g.replay()
        e.record(stream)
    e.synchronize()
    return s.elapsed_time(e) / 1e3  # seconds


NORTH_STAR_SHAPES = [(24576, 8192), (8192, 8192), (28672, 8192), (8192, 28672)]  # test_flexq_kernel.sh:25-28
# the reference's own kernel sweep (engine/test_flexq_kernel.sh:7-39): (model, N, K, abits) at M = 1, 2, 4, 8
REFERENCE_SWEEP = [("llama_7b", 12288, 4096, 6), ("llama_7b", 4096, 4096, 6), ("llama_7b", 11008, 4096, 6),
                   ("llama_7b", 4096, 11008, 8), ("llama_30b", 19968, 6656, 6), ("llama_30b", 6656, 6656, 6),
                   ("llama_30b", 17920, 6656, 6), ("llama_30b", 6656, 17920, 8), ("llama_2_13b", 15360, 5120, 6),
                   ("llama_2_13b", 5120, 5120, 6), ("llama_2_13b", 13824, 5120, 6), ("llama_2_13b", 5120, 13824, 8),
                   ("llama_2_70b", 24576, 8192, 6), ("llama_2_70b", 8192, 8192, 6), ("llama_2_70b", 28672, 8192, 6),
                   ("llama_2_70b", 8192, 28672, 8), ("opt_30b", 21504, 7168, 6), ("opt_30b", 7168, 7168, 6),
                   ("opt_30b", 28672, 7168, 6), ("opt_30b", 7168, 28672, 8)]


def int8_vendor_us(N, K, M, dev, g, s, reps):
    """Context: the vendor int8 GEMM (torch._int_mm, int8 x int8 -> int32 on hipBLASLt; the
    reference's W8A8 cuBLAS baseline, engine/test_cublas_kernel.cu:122-133) at the same N, K; M is
    raised to the smallest size the op accepts when it rejects M.  Returns (us, M run)."""
    copies = max(2, -(-768 * 2**20 // (N * K)))
    w8 = [torch.randint(-128, 128, (N, K), dtype=torch.int8, device=dev, generator=g) for _ in range(copies)]
    for Mi in (M, 17, 32):
        if Mi < M:
            continue
        try:
            x8 = torch.randint(-128, 128, (Mi, K), dtype=torch.int8, device=dev, generator=g)
            with torch.cuda.stream(s):
                torch._int_mm(x8, w8[0].t())
            torch.cuda.synchronize()
            break
        except RuntimeError:
            continue
    else:
        return None, None
    gi = capture(lambda: [torch._int_mm(x8, w8[i % copies].t()) for i in range(reps)], s)
    gi.replay()
    torch.cuda.synchronize()
    t = time_graph(gi, 5, s) / (5 * reps)
    del gi, w8
    return t, Mi


def fp16_compare(shapes, M, abits, dev, reps=20, int8=False):
    """North-star denominator: rocBLAS/hipBLASLt fp16 GEMM (torch F.linear, fp16 weights) vs the
    W6Ax linear at the same (M, N, K).  Each side replays a graph of `reps` launches rotating over
    enough weight copies (>= 768 MB) that the 256 MB MALL cannot serve them.  int8: also the vendor
    int8 GEMM (context only, int8_vendor_us)."""
    out = []
    g = torch.Generator(device=dev).manual_seed(7)
    s = torch.cuda.Stream(dev)
    for (N, K) in shapes:
        x = torch.randn((M, K), dtype=torch.float16, device=dev, generator=g)
        copies = max(2, -(-768 * 2**20 // (2 * N * K)))
        w16 = [torch.randn((N, K), dtype=torch.float16, device=dev, generator=g) * 0.02 for _ in range(copies)]
        y16 = torch.empty((M, N), dtype=torch.float16, device=dev)
        wq = [ops.pack_w6(torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g),
                          (torch.rand((K // GROUP, N), device=dev, generator=g) * 0.02).half()) for _ in range(copies)]
        y6 = torch.empty((M, N), dtype=torch.float16, device=dev)
        with torch.cuda.stream(s):  # eager warm-up (hipBLASLt heuristics, workspaces)
            torch.nn.functional.linear(x, w16[0], out=y16)
            ops.linear_w6ax(x, wq[0], N, abits, out=y6)
        torch.cuda.synchronize()
        g16 = capture(lambda: [torch.nn.functional.linear(x, w16[i % copies], out=y16) for i in range(reps)], s)
        g6 = capture(lambda: [ops.linear_w6ax(x, wq[i % copies], N, abits, out=y6) for i in range(reps)], s)
        for gr in (g16, g6):
            gr.replay()
        torch.cuda.synchronize()
        t16 = time_graph(g16, 5, s) / (5 * reps)
        t6 = time_graph(g6, 5, s) / (5 * reps)
        row = {"N": N, "K": K, "M": M, "fp16_us": round(t16 * 1e6, 2), "w6_us": round(t6 * 1e6, 2),
               "speedup": round(t16 / t6, 3),
               # what the vendor GEMV achieves (a weak one inflates the speedup) and the W6 kernel's own
               # roofline fraction -- the figure the north-star verdict rests on
               "fp16_TBps": round(fp16_bytes(M, N, K) / t16 / 1e12, 3),
               "w6_hbm_frac": round(alg_bytes(M, N, K, abits, ops.act_scratch_bytes(M, N, K) == 0) / t6 / 1e9
                                    / HBM_PEAK_GBS, 4)}
        del g16, g6, w16, wq
        torch.cuda.synchronize()
        if int8:
            ti, mi = int8_vendor_us(N, K, M, dev, g, s, reps)
            if ti is not None:
                row.update(int8_vendor_us=round(ti * 1e6, 2), int8_vendor_M=mi, speedup_vs_int8=round(ti / t6, 3))
            torch.cuda.synchronize()
        out.append(row)
    return out


def reference_sweep(dev, Ms=(1, 2, 4, 8), reps=10, budget=512 * 2**20):
    """README.md:189's comparison on the reference's own sweep (engine/test_flexq_kernel.sh:7-39): every
    (N, K, abits) shape of LLaMA-7B, LLaMA-30B, LLaMA-2-13B, LLaMA-2-70B and OPT-30B at M = 1, 2, 4, 8.
    Per shape and M, graph-timed over rotating weight copies (>= `budget` bytes, beyond the MALL):
      * w6_gemm_us: the W6Ax GEMM on pre-quantized activations (what test_bgemm_kernel times:
        benchmark<> runs exec_fn on packed X, test/test_kernel.h:131-142);
      * w6_linear_us: the whole linear, dynamic activation quantization included;
      * fp16_us: torch F.linear fp16 (hipBLASLt / rocBLAS), the north-star denominator;
      * int8_us: the vendor int8 GEMM torch._int_mm (the reference's cuBLAS W8A8 baseline,
        engine/test_cublas_kernel.cu:122-133), at the smallest M >= 17 it accepts (one value per shape).
    Averages per M in README.md:189's form: the arithmetic mean of the per-shape speedups."""
    g = torch.Generator(device=dev).manual_seed(11)
    s = torch.cuda.Stream(dev)
    rows, by_m = [], {m: {"vs_int8": [], "vs_fp16": [], "linear_vs_int8": [], "fp16_TBps": [], "w6_frac": []}
                      for m in Ms}
    for (model, N, K, ab) in REFERENCE_SWEEP:
        c16 = max(2, -(-budget // (2 * N * K)))
        c6 = max(2, -(-budget // (N * K * 3 // 4)))
        w16 = [torch.randn((N, K), dtype=torch.float16, device=dev, generator=g) * 0.02 for _ in range(c16)]
        w6 = [ops.pack_w6(torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g),
                          (torch.rand((K // GROUP, N), device=dev, generator=g) * 0.02).half()) for _ in range(c6)]
        ti, mi = int8_vendor_us(N, K, 1, dev, g, s, reps)
        for M in Ms:
            x = torch.randn((M, K), dtype=torch.float16, device=dev, generator=g)
            xq, xs = ops.quantize_act(x, ab)
            y16 = torch.empty((M, N), dtype=torch.float16, device=dev)
            y6 = torch.empty((M, N), dtype=torch.float16, device=dev)
            with torch.cuda.stream(s):
                torch.nn.functional.linear(x, w16[0], out=y16)
                ops.linear_w6ax(x, w6[0], N, ab, out=y6)
                ops.gemm_w6ax(xq, xs, w6[0], N, ab, out=y6)
            torch.cuda.synchronize()
            t = {}
            for key, fn in (("fp16", lambda: [torch.nn.functional.linear(x, w16[i % c16], out=y16) for i in range(reps)]),
                            ("lin", lambda: [ops.linear_w6ax(x, w6[i % c6], N, ab, out=y6) for i in range(reps)]),
                            ("gemm", lambda: [ops.gemm_w6ax(xq, xs, w6[i % c6], N, ab, out=y6) for i in range(reps)])):
                gr = capture(fn, s)
                gr.replay()
                torch.cuda.synchronize()
                t[key] = time_graph(gr, 3, s) / (3 * reps)
                del gr
            row = {"model": model, "M": M, "N": N, "K": K, "abits": ab, "w6_gemm_us": round(t["gemm"] * 1e6, 2),
                   "w6_linear_us": round(t["lin"] * 1e6, 2), "fp16_us": round(t["fp16"] * 1e6, 2),
                   "speedup_vs_fp16": round(t["fp16"] / t["gemm"], 3),
                   "fp16_TBps": round(fp16_bytes(M, N, K) / t["fp16"] / 1e12, 3),
                   "w6_gemm_hbm_frac": round(alg_bytes(M, N, K, ab, False) / t["gemm"] / 1e9 / HBM_PEAK_GBS, 4)}
            by_m[M]["vs_fp16"].append(t["fp16"] / t["gemm"])
            by_m[M]["fp16_TBps"].append(row["fp16_TBps"])
            by_m[M]["w6_frac"].append(row["w6_gemm_hbm_frac"])
            if ti is not None:
                row.update(int8_us=round(ti * 1e6, 2), int8_M=mi, speedup_vs_int8=round(ti / t["gemm"], 3),
                           linear_speedup_vs_int8=round(ti / t["lin"], 3))
                by_m[M]["vs_int8"].append(ti / t["gemm"])
                by_m[M]["linear_vs_int8"].append(ti / t["lin"])
            rows.append(row)
        del w16, w6
        torch.cuda.empty_cache()
    mean = lambda v: round(float(np.mean(v)), 3) if v else None  # noqa: E731
    return {"what": "README.md:189's comparison over the reference's own kernel sweep (engine/test_flexq_kernel.sh:"
                    "7-39: LLaMA-7B, LLaMA-30B, LLaMA-2-13B, LLaMA-2-70B, OPT-30B; W6A8 down shapes) at M = 1, 2, 4, "
                    "8: the W6Ax GEMM on pre-quantized activations (as test_bgemm_kernel times it) vs the vendor "
                    "int8 GEMM torch._int_mm (the reference's cuBLAS W8A8 baseline; run at the smallest M it "
                    "accepts, int8_M) and vs hipBLASLt fp16 F.linear; graph-timed over rotating weight copies",
            "reference_published": {"vs_cublas_w8a8_avg": {"1": 1.78, "4": 1.81, "8": 1.82},
                                    "hardware": "NVIDIA A6000-class (sm_86), README.md:189"},
            "avg_speedup_vs_int8_by_M": {str(m): mean(v["vs_int8"]) for m, v in by_m.items()},
            "avg_linear_speedup_vs_int8_by_M": {str(m): mean(v["linear_vs_int8"]) for m, v in by_m.items()},
            "avg_speedup_vs_fp16_by_M": {str(m): mean(v["vs_fp16"]) for m, v in by_m.items()},
            "avg_fp16_TBps_by_M": {str(m): mean(v["fp16_TBps"]) for m, v in by_m.items()},
            "avg_w6_gemm_hbm_frac_by_M": {str(m): mean(v["w6_frac"]) for m, v in by_m.items()},
            "shapes": rows}


def pmc_traffic(config, merge):
    """HBM bytes per launch of the dominant kernel from the newest committed rocprofv3 FETCH_SIZE
    pass for this workload (profiles/rNN_pmc_summary.json, written by tools/pmc_summary.py, with
    the gfx950 x2 correction applied).  None when no pass matches."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_summary.json")), reverse=True):
        d = json.load(open(path))
        if d.get("config") == config and d.get("merged_gate_up", False) == merge:
            return d["hbm_read_bytes_per_launch"], os.path.relpath(path, ROOT)
    return None, None


def calibrate_peaks(dev, hbm_bytes=4 << 30, mfma_iters=20000):
    """Measured on this box: HBM streaming-read GB/s of a 16 B/lane
    non-temporal read over 4 GiB, and dense int8 MFMA TOPS of 4 independent
    v_mfma_i32_16x16x64_i8 chains per wave, 2 waves per SIMD (tools/fq_calib.hip)."""
    import ctypes
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libfq_calib.so"))
    lib.fqc_hbm_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    lib.fqc_mfma_i8.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    buf = torch.ones(hbm_bytes // 4, dtype=torch.int32, device=dev)
    sink = torch.zeros(8 * cus, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev)
    h = ctypes.c_void_p(s.cuda_stream)

    def timed(fn, reps):
        fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(reps):
            fn()
        b.record(s)
        b.synchronize()
        return a.elapsed_time(b) / 1e3 / reps

    t_hbm = timed(lambda: lib.fqc_hbm_read(ctypes.c_void_p(buf.data_ptr()), ctypes.c_size_t(hbm_bytes),
                                           ctypes.c_void_p(sink.data_ptr()), 8 * cus, h), 5)
    t_mfma = timed(lambda: lib.fqc_mfma_i8(mfma_iters, cus, ctypes.c_void_p(sink.data_ptr()), h), 3)
    del buf
    ops_mfma = cus * 8 * 4 * mfma_iters * (16 * 16 * 64 * 2)
    return {"hbm_read_GBps": round(hbm_bytes / t_hbm / 1e9, 1), "int8_mfma_TOPS": round(ops_mfma / t_mfma / 1e12, 1),
            "method": "tools/fq_calib.hip: 4 GiB 16 B/lane non-temporal streaming read; 4 independent "
                      "16x16x64 i8 MFMA chains per wave, 8 waves per CU"}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(budget_s=15.0, lins=None, M=1):
    """The reference's CPU fake-quant QuantLinear forward (oracle restatement, torch CPU ops) on a
    bounded sample of the workload's linear shapes, fp16, in BASELINE.md §3's two variants, half
    the budget each:
      * pre-quantized weights (weight_quant_inplace once, flexq_quantize/utils.py:116-123, then
        only the dynamic activation quantizer + F.linear per forward) -- the primary `value`;
      * re-quantized weights per forward: the reference eval flow (flexqllm.py:106-108 leaves
        use_weight_quant on, int_linear.py:60-61).
    At prefill sizes a 64-row slice of the M activation rows (the rate is per FLOP, so it scales)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import fq_oracle as oracle  # bench's cpu_baseline leg only
    # the GPU box exports OMP_NUM_THREADS = its CPU share (os.cpu_count() reports the whole host)
    quota = int(os.environ.get("OMP_NUM_THREADS", "0"))
    threads = quota or (os.cpu_count() or 1)
    torch.set_num_threads(threads)
    lins = lins or CONFIGS["llama2-7b-m1"][2]
    rows = min(M, 64)
    gen = torch.Generator().manual_seed(0)
    ws = [torch.randn((N, K), generator=gen).mul_(0.02).half() for (_, N, K, _) in lins]
    xs = [torch.randn((rows, K), generator=gen).half() for (_, N, K, _) in lins]
    what = [oracle.fake_quant_per_group(w, 6)[0] for w in ws]  # weight_quant_inplace, once

    def run(requant, budget):
        flops, layers = 0.0, 0
        t0 = time.perf_counter()
        while True:
            for (_, N, K, ab), w, wh, x in zip(lins, ws, what, xs):
                oracle.quant_linear_forward(x, w, 6, ab, requant_weight=requant, w_hat=wh)
                flops += 2.0 * rows * N * K
            layers += 1
            if time.perf_counter() - t0 > budget:
                break
        dt = time.perf_counter() - t0
        return flops / dt / 1e12, layers, dt

    pre, pre_layers, pre_dt = run(False, budget_s / 2)
    req, req_layers, req_dt = run(True, budget_s / 2)
    sample = (f"{len(lins)} linears per layer at M={rows} rows{' of ' + str(M) if rows < M else ''}, fp16, "
              f"through the fake-quant QuantLinear forward")
    return dict(value=pre, unit="TFLOPS-equiv", cores=threads, kind="port",
                sample=f"{sample}: {pre_layers} layers in {pre_dt:.1f} s with pre-quantized weights",
                tok_per_s=rows * pre_layers / pre_dt / 32,
                cpu_model=cpu_model(), os_cpu_count=os.cpu_count(), torch_threads=torch.get_num_threads(),
                cores_reason=("all of this process's CPU share: the GPU lease exports OMP_NUM_THREADS=%d (its CPU "
                              "quota; os.cpu_count() reports the whole %s-CPU host, shared with other leases)"
                              % (quota, os.cpu_count()) if quota else "os.cpu_count(): no CPU quota exported"),
                variants={
                    "prequantized_weights": dict(value=pre, tok_per_s=rows * pre_layers / pre_dt / 32,
                                                 layers=pre_layers, seconds=round(pre_dt, 2)),
                    "requant_weights_per_forward": dict(value=req, tok_per_s=rows * req_layers / req_dt / 32,
                                                        layers=req_layers, seconds=round(req_dt, 2),
                                                        note="the reference eval flow (flexqllm.py:106-108)"),
                })


# ---- the driver's line: the driver keeps a ~8 KB tail of stdout, so the final line must stay short
# (round 4's 28 KB line was unparseable).  The full result goes to a detail file; the line keeps the
# headline, the rooflines, the CPU baseline and per-section summaries.
LINE_MAX = 6000
ESSENTIAL = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
             "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline")
# N > 1: the same workload's one-GPU point and the collectives' world / backend, never dropped either
KEEP = ESSENTIAL + ("same_workload_1gpu", "comm")
# optional sections, dropped from the line in this order while it is too long (all stay in the detail file)
DROP_ORDER = ("vs_reference_sweep", "decoder_layers_e2e", "tp_llama2_7b_peer_gather", "tp_peer_gather",
              "c4_llama2_70b_tp_peer_gather", "replicas", "vs_rocblas_fp16", "tp_llama2_7b", "c4_llama2_70b_tp",
              "c4_llama2_70b_1gpu", "c3_llama2_7b_m16", "c5_llama3_8b_prefill", "tp", "decode_chain")
_TEXT_KEYS = {"what", "method", "traffic_vs", "note", "cores_reason", "hardware"}
_ROW = ("N", "K", "M", "fp16_us", "w6_us", "speedup", "fp16_TBps", "w6_hbm_frac")


def _slim(v):
    """Drop explanatory text (it is in the detail file and DESIGN.md) and round floats."""
    if isinstance(v, dict):
        return {k: _slim(x) for k, x in v.items() if k not in _TEXT_KEYS}
    if isinstance(v, list):
        return [_slim(x) for x in v]
    if isinstance(v, float):
        return round(v, 4)
    return v


def compact_line(res, detail=None, limit=LINE_MAX):
    """The one JSON object bench.py prints last: every ESSENTIAL key, then the optional sections with
    their per-shape rows folded into summaries (vs_reference_sweep: the per-M averages only;
    vs_rocblas_fp16: one short row per shape), dropping whole sections in DROP_ORDER while the line is
    longer than `limit` characters."""
    out = {}
    for k, v in res.items():
        if k == "vs_reference_sweep" and isinstance(v, dict) and "shapes" in v:
            v = {kk: vv for kk, vv in v.items() if kk != "shapes"}
            v["shapes_count"] = len(res[k]["shapes"])
        elif k == "vs_rocblas_fp16" and isinstance(v, dict):
            v = dict(v)
            for kk in ("config_shapes", "llama2_70b_m1"):
                if isinstance(v.get(kk), list):
                    v[kk] = [[r.get(f) for f in _ROW] for r in v[kk]]
            v["row_fields"] = list(_ROW)
        elif k == "cpu_baseline" and isinstance(v, dict):
            req = v.get("variants", {}).get("requant_weights_per_forward", {})
            v = {kk: vv for kk, vv in v.items() if kk != "variants"}
            if req:
                v["requant_weights_per_forward_value"] = req.get("value")
        out[k] = _slim(v)
    if detail:
        out["detail_file"] = detail
    for k in DROP_ORDER:
        if len(json.dumps(out)) <= limit:
            break
        if k in out:
            out[k] = "in detail_file"
    if len(json.dumps(out)) > limit:  # last resort: the essentials alone
        out = {k: out[k] for k in KEEP if k in out}
        if detail:
            out["detail_file"] = detail
    return out


def write_detail(res, path):
    """The full result as JSON (every row of every comparison); returns the path written, or None."""
    if not path:
        return None
    try:
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        with open(path, "w") as f:
            json.dump(res, f)
        return os.path.relpath(path, ROOT) if os.path.abspath(path).startswith(ROOT) else path
    except OSError as e:
        print(f"[bench] could not write {path}: {e}", file=sys.stderr)
        return None


def visible_gpus():
    """GPUs this process may use, counted WITHOUT touching the HIP runtime (which any HIP call,
    and torch's device count when amdsmi is unusable, would initialise before the spawn): KFD
    topology nodes with SIMDs, narrowed by the *_VISIBLE_DEVICES lists.  None if unknown."""
    import glob
    try:
        n = 0
        for prop in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
            with open(prop) as f:
                kv = dict(line.split() for line in f if len(line.split()) == 2)
            n += int(kv.get("simd_count", "0")) > 0
    except (OSError, ValueError):
        return None
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([d for d in v.split(",") if d.strip() != ""]))
    return n if n > 0 else None


def spawn_ranks(a):
    """`bench.py --gpus N` outside torchrun: start N ranks as a child torchrun (one process per GPU,
    127.0.0.1 rendezvous) and return its exit code.  Runs before anything touches the GPU
    (visible_gpus() reads the KFD topology, no HIP call), and the child is a separate
    process: nothing is exec'd over a process that has used the GPU."""
    import socket
    import subprocess
    n_dev = visible_gpus()
    if n_dev is not None and n_dev < a.gpus and not a.share_gpu:
        print(f"[bench] --gpus {a.gpus} but only {n_dev} GPU(s) visible", file=sys.stderr)
        return 2
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


class Ctx:
    """Rank context: device, world, the timing helpers shared by every measured stack."""

    def __init__(self, a, rank, world, dev, staged):
        self.a, self.rank, self.world, self.dev, self.staged = a, rank, world, dev, staged
        self.stream = torch.cuda.Stream(dev)

    def sync_all(self):
        torch.cuda.synchronize()
        if self.world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(self, v):
        if self.world == 1:
            return v
        t = torch.tensor([v], dtype=torch.float64, device=self.dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def prepare(self, step, use_graph):
        """Warm `step` eagerly on the capture stream (workspaces, communicators), then capture it
        into one HIP graph when allowed; returns replay()."""
        with torch.cuda.stream(self.stream):
            step()
        self.sync_all()
        graph = None
        if use_graph:
            try:
                graph = capture(step, self.stream)
            except RuntimeError as e:  # (an RCCL build that cannot be captured: time eager launches)
                if self.world == 1:
                    raise
                print(f"[bench] rank {self.rank}: graph capture with RCCL failed ({e}); eager launches",
                      file=sys.stderr)
                torch.cuda.synchronize()
        if graph is None:
            def replay():
                with torch.cuda.stream(self.stream):
                    step()
        else:
            def replay():
                graph.replay()
        replay.graph = graph
        return replay

    def timed(self, replay, steps, warmup):
        """W untimed + K timed replays, barrier + synchronize on both sides; the max over ranks of
        the wall time, and this rank's HIP-event time on the launch stream."""
        with torch.cuda.stream(self.stream):
            for _ in range(warmup):
                replay()
        self.sync_all()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        with torch.cuda.stream(self.stream):
            ev0.record(self.stream)
            for _ in range(steps):
                replay()
            ev1.record(self.stream)
        self.sync_all()
        elapsed = time.perf_counter() - t0
        return self.max_over_ranks(elapsed), ev0.elapsed_time(ev1) / 1e3

    def graph_time(self, fn, launches, reps):
        """Seconds per replay and per launch of a graph of fn (HIP events on its stream)."""
        g2 = capture(fn, self.stream)
        for _ in range(2):
            g2.replay()
        torch.cuda.synchronize()
        t = time_graph(g2, reps, self.stream)
        del g2
        return t / reps, t / (reps * launches)


def measure_tp(ctx, cfg, merge, tp, steps, warmup, peer=False):
    """Column-parallel N-shard of every linear of cfg over tp ranks: each rank
    streams its N/tp rows, ONE all-gather per linear assembles the fp16 output.  Returns ms/step
    with and without the gathers (max over ranks), the per-rank roofline of the GEMM launches and
    the gather bytes."""
    layers, M, lins, _ = cfg
    launch_lins = launch_list(lins, merge)
    stack = build_stack(cfg, ctx.rank, tp, ctx.dev, merge, peer=peer)
    use_graph = not ctx.a.no_graph and (peer or not ctx.staged)
    replay = ctx.prepare(lambda: run_step(stack, M, tp, staged=ctx.staged), use_graph)

    def peer_check(when):  # a timed-out peer wait on any rank fails the section on every rank
        pgs = {id(p["pg"]): p["pg"] for _, p in linears(stack) if "pg" in p}.values() if peer else ()
        if peer and ctx.max_over_ranks(float(any(pg.error() for pg in pgs))) > 0:
            raise RuntimeError(f"peer-store gather: a wait timed out ({when})")
    peer_check("warm-up")
    elapsed, _ = ctx.timed(replay, steps, warmup)
    peer_check("timed steps")
    n_lin = layers * len(launch_lins)
    gemm_step, per_launch = ctx.graph_time(lambda: run_step(stack, M, tp, gather=False), n_lin,
                                           ctx.a.roofline_reps)
    last_full = linears(stack)[-1][1]["full"]
    finite = bool(torch.isfinite(last_full.float()).all().item())
    final = last_full.view(-1)[:M * linears(stack)[-1][1]["N"]].cpu().numpy().copy()  # the step's output
    gemm_ms = ctx.max_over_ranks(gemm_step) * 1e3
    per_launch = ctx.max_over_ranks(per_launch)
    fused = {(N, K): ops.act_scratch_bytes(M, N // tp, K) == 0 for (_, N, K, _) in launch_lins}
    bytes_launch = layers * sum(alg_bytes(M, N // tp, K, ab, fused[(N, K)]) for (_, N, K, ab) in launch_lins) / n_lin
    flops_step = layers * sum(2.0 * M * N * K for (_, N, K, _) in lins)
    del stack, replay
    torch.cuda.empty_cache()
    return dict(ms_per_step=elapsed / steps * 1e3, elapsed=elapsed, flops_step=flops_step,
                gemm_only_ms_per_step=gemm_ms, allgather_ms_per_step=max(0.0, elapsed / steps * 1e3 - gemm_ms),
                per_launch_us=per_launch * 1e6, alg_bytes_per_launch=int(bytes_launch),
                hbm_GBps_per_rank=bytes_launch / per_launch / 1e9,
                allgather_bytes_per_step_per_rank=int(layers * sum(2 * M * (N // tp) * (tp - 1)
                                                                   for (_, N, K, _) in launch_lins)),
                launches_per_step=n_lin, fused_launches=all(fused.values()), graph=use_graph, finite=finite,
                final=final)


def measure_alone(ctx, cfg, merge, steps, warmup):
    """The same workload on ONE GPU, measured inside an N-rank run: rank 0 builds the
    whole (unsharded) stack and times it as one HIP graph of its per-linear launches -- the form the
    column-parallel step runs on every rank, minus the split and the gathers -- while the other ranks wait;
    ms per step broadcast to every rank.  The denominator of the line's strong-scaling efficiency, taken on
    the same node and in the same run as the split it is compared with."""
    layers, M, lins, _ = cfg
    ms = torch.zeros(1, dtype=torch.float64, device=ctx.dev)
    if ctx.rank == 0:
        stack = build_stack(cfg, 0, 1, ctx.dev, merge)
        step = lambda: run_step(stack, M, 1)  # noqa: E731
        with torch.cuda.stream(ctx.stream):
            step()
        torch.cuda.synchronize()
        g = capture(step, ctx.stream) if not ctx.a.no_graph else None
        with torch.cuda.stream(ctx.stream):
            for _ in range(warmup):
                g.replay() if g is not None else step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(ctx.stream):
            for _ in range(steps):
                g.replay() if g is not None else step()
        torch.cuda.synchronize()
        ms[0] = (time.perf_counter() - t0) / steps * 1e3
        del stack, g
        torch.cuda.empty_cache()
    if ctx.world > 1:
        dist.broadcast(ms, src=0)  # (the other ranks wait here while rank 0 measures)
    return float(ms.item())


def scaling_vs_1gpu(ms_n, ms_1, world, what):
    """Strong scaling against the same workload on one GPU: speedup ms_1 / ms_N, efficiency / N."""
    return {"what": what, "ms_per_step_1gpu": round(ms_1, 4), "ms_per_step": round(ms_n, 4),
            "speedup_vs_1gpu": round(ms_1 / ms_n, 4), "strong_scaling_efficiency": round(ms_1 / ms_n / world, 4)}


def measure_single(ctx, name, merge, steps, warmup):
    """Another BASELINE config on this one GPU, measured in the same run as the headline (C3's
    batch-16 step, C5's prefill step): the whole step as one HIP graph of its launches (quantize +
    GEMM per linear where they are separate), and for prefill the GEMM launches alone on
    pre-quantized codes (the MFMA roofline)."""
    cfg = CONFIGS[name]
    layers, M, lins, desc = cfg
    launch_lins = launch_list(lins, merge)
    n_lin = layers * len(launch_lins)
    stack = build_stack(cfg, ctx.rank, 1, ctx.dev, merge)
    replay = ctx.prepare(lambda: run_step(stack, M, 1), not ctx.a.no_graph)
    elapsed, ev_s = ctx.timed(replay, steps, warmup)
    chain = None
    if M <= 4 and not ctx.a.no_chain:  # the decode chains, as for the headline (taken when identical + faster)
        last_out = linears(stack)[-1][1]["out"]
        ref_bits = last_out.cpu().numpy().view(np.uint16).copy()
        runs = chain_runs(stack)
        replay_c = ctx.prepare(lambda: run_chains(runs), not ctx.a.no_graph)
        el_c, ev_c = ctx.timed(replay_c, steps, warmup)
        same = bool(np.array_equal(last_out.cpu().numpy().view(np.uint16), ref_bits))
        err = ops.chain_error(ctx.dev, stream=ctx.stream)
        chain = {"launches_per_step": len(runs), "ms_per_step": round(el_c / steps * 1e3, 4),
                 "launches_ms_per_step": round(elapsed / steps * 1e3, 4), "bit_identical_to_launches": same,
                 "wait_timed_out": bool(err)}
        if same and not err and el_c < elapsed:
            elapsed, ev_s = el_c, ev_c
            chain["taken"] = True
        del replay_c
    qo = None
    if (M >= ops.PREFILL_U8_MIN_M or 4 < M <= 16) and not ctx.a.no_qo:  # quantize in the producer's epilogue
        last_out = linears(stack)[-1][1]["out"]
        ref = last_out.clone()
        replay_q = ctx.prepare(lambda: run_step_qo(stack, M), not ctx.a.no_graph)
        el_q, ev_q = ctx.timed(replay_q, steps, warmup)
        same = bool(torch.equal(last_out.view(torch.int16), ref.view(torch.int16)))
        del ref
        qo = {"what": "each linear's activation quantize in the previous GEMM's epilogue "
                      "(fq_gemm_w6ax_u8_q / fq_gemm_w6ax_q; the step's first input quantized by its own launch)",
              "ms_per_step": round(el_q / steps * 1e3, 4),
              "separate_quantize_ms_per_step": round(elapsed / steps * 1e3, 4),
              "last_output_identical": same}
        if same and el_q < elapsed:
            elapsed, ev_s = el_q, ev_q
            qo["taken"] = True
        del replay_q
    flops_step = layers * sum(2.0 * M * N * K for (_, N, K, _) in lins)
    out = {"what": f"BASELINE config: {desc}, the dependent linear stack of every layer, one HIP graph" +
                   (" (weights: the fq6 image + its int8 MFMA operands unpacked once at load, "
                    "ops.prepare_prefill_weights; per linear the activation quantize + the prefill GEMM)"
                    if M >= ops.PREFILL_U8_MIN_M else ""),
           "ms_per_step": round(elapsed / steps * 1e3, 4),
           "value": round(flops_step * steps / elapsed / 1e12, 4), "unit": "TFLOPS-equiv",
           "tok_per_s": round(M * steps / elapsed, 2), "steps": steps, "warmup": warmup,
           "finite": bool(torch.isfinite(linears(stack)[-1][1]["out"].float()).all().item())}
    if chain is not None:
        out["decode_chain"] = chain
    if qo is not None:
        out["epilogue_quantize"] = qo
    if M > PREFILL_M:
        codes = {}
        for nm, p in linears(stack):
            if nm not in codes:
                codes[nm] = ops.quantize_act(p["x"], p["abits"])

        def gemms():
            for nm, p in linears(stack):
                ops.gemm_w6ax(codes[nm][0], codes[nm][1], p["pk"], p["Nl"], p["abits"], out=p["out"],
                              w_u8=p.get("w_u8"))
        _, per_gemm_s = ctx.graph_time(gemms, n_lin, 2)
        ops_launch = layers * sum(2.0 * M * N * K for (_, N, K, _) in launch_lins) / n_lin
        ach = ops_launch / per_gemm_s / 1e12
        out["roofline"] = {"kernel": "fq_gemm_prefill_big_kernel" if M >= 2048 else "fq_gemm_prefill_kernel",
                           "bound": "mfma", "achieved": round(ach, 1), "peak": I8_MFMA_PEAK_TOPS,
                           "unit": "TFLOP/s", "frac": round(ach / I8_MFMA_PEAK_TOPS, 4),
                           "per_launch_us": round(per_gemm_s * 1e6, 3)}
        del codes
    else:
        per_launch = ev_s / (steps * n_lin)
        fused = {(N, K): ops.act_scratch_bytes(M, N, K) == 0 for (_, N, K, _) in launch_lins}
        bytes_launch = layers * sum(alg_bytes(M, N, K, ab, fused[(N, K)]) for (_, N, K, ab) in launch_lins) / n_lin
        qtaken = qo is not None and qo.get("taken", False)
        out["roofline"] = {"kernel": "fq_gemm_decode_kernel" + ("<FUSE>" if all(fused.values()) else
                                                                 " with the next input's quantizer in its epilogue"
                                                                 if qtaken else " + the separate quantize launch"),
                           "bound": "hbm", "achieved": round(bytes_launch / per_launch / 1e9, 1),
                           "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": round(bytes_launch / per_launch / 1e9 / HBM_PEAK_GBS, 4),
                           "per_launch_us_incl_quantize": round(per_launch * 1e6, 3)}
    del stack, replay
    torch.cuda.empty_cache()
    return out


def decoder_layers_e2e(ctx, M, layers=32, H=4096, F=11008, reps=5, seed=77):
    """SURVEY.md §8(f)3 / README.md:193: LLaMA-2-7B decoder layers end to end (norms, SiLU*up,
    the four linears, residuals; the attention core is out of scope and stands in as ctx = v,
    exact attention over a single position) in FT's tensor-parallel layout over the ranks --
    qkv and gate_up column-parallel, o_proj and down_proj row-parallel + one all-reduce each
    (flexq_amd.layers.FlexQDecoderLayer) -- against the same layers in fp16 torch ops (F.rms_norm,
    hipBLASLt F.linear, F.silu, the same all-reduces), both as one HIP graph over `layers` layers.
    Returns ms per token step for both and, with several ranks, the W6 step without its
    all-reduces."""
    from flexq_amd import convert
    from flexq_amd.layers import FlexQDecoderLayer, FlexQFfn, W6Linear, run_layers
    dev, tp, rank = ctx.dev, ctx.world, ctx.rank
    g = torch.Generator(device=dev).manual_seed(seed)  # the same full weights on every rank
    sq, sf = H ** -0.5, F ** -0.5
    w6, w16 = [], []
    for _ in range(layers):
        q, k, v, o = (torch.randn((H, H), device=dev, generator=g) * sq for _ in range(4))
        gate, up = (torch.randn((F, H), device=dev, generator=g) * sq for _ in range(2))
        down = torch.randn((H, F), device=dev, generator=g) * sf
        qkv_p = convert.shard_parts([q.half(), k.half(), v.half()], tp, rank)
        o_p, _ = convert.shard_columns(o.half(), tp, rank)
        gu_p = convert.shard_parts([gate.half(), up.half()], tp, rank, by_group=True)
        down_p, _ = convert.shard_columns(down.half(), tp, rank)
        del q, k, v, o, gate, up, down
        ga = torch.ones(H, dtype=torch.float16, device=dev)
        lin = lambda w, ab, row: W6Linear(ops.quantize_pack_w6(w)[0], w.shape[0], w.shape[1], ab,  # noqa: E731
                                          row_parallel=row and tp > 1)
        w6.append(FlexQDecoderLayer(lin(qkv_p, 6, False), lin(o_p, 6, True),
                                    FlexQFfn(lin(gu_p, 6, False), lin(down_p, 8, True), ga), ga,
                                    lambda qkv: qkv[:, 2 * qkv.shape[1] // 3:]))
        w16.append(dict(qkv=qkv_p, o=o_p, gu=gu_p, down=down_p, ga=ga, Fp=down_p.shape[1]))
    torch.cuda.synchronize()

    def allreduce(t):  # the same all-reduces as the W6 layers' (gloo in the --share-gpu rehearsal)
        if tp > 1:
            dist.all_reduce(t)

    def step_w6(h):  # each layer's last residual add fused into the next one's norm (FT)
        run_layers(w6, h)

    def step_w6_noreduce(h):  # tp > 1, timing only: the same launches on the same buffers with the two
        # all-reduces per layer left out (every rank's partial sums feed its next norm: not a model output;
        # run_layers refuses reduce=False at tp > 1 for exactly that reason, so this bypasses it on purpose)
        pending, cur, spare = None, h, torch.empty_like(h)
        for L in w6:
            pending, cur, spare = L.step(cur, pending, spare, reduce=False)
        if pending is not None:
            torch.add(cur, pending, out=h)

    def step_16(h):
        F_ = torch.nn.functional
        for W in w16:
            x = F_.rms_norm(h, (H,), W["ga"], 1e-6)
            qkv = F_.linear(x, W["qkv"])
            a = F_.linear(qkv[:, 2 * qkv.shape[1] // 3:], W["o"])
            allreduce(a)
            h += a
            x = F_.rms_norm(h, (H,), W["ga"], 1e-6)
            gu = F_.linear(x, W["gu"])
            y = F_.linear(F_.silu(gu[:, :W["Fp"]]) * gu[:, W["Fp"]:], W["down"])
            allreduce(y)
            h += y

    out = {}
    h0 = torch.randn((M, H), dtype=torch.float16, device=dev, generator=g)
    hs = {k: h0.clone() for k in ("w6", "w6_noreduce", "fp16")}
    fns = {"w6": lambda: step_w6(hs["w6"]), "fp16": lambda: step_16(hs["fp16"])}
    if tp > 1:
        fns["w6_noreduce"] = lambda: step_w6_noreduce(hs["w6_noreduce"])
    for name, fn in fns.items():
        replay = ctx.prepare(fn, not ctx.a.no_graph and not ctx.staged)
        hs[name].copy_(h0)
        replay()
        torch.cuda.synchronize()
        el, _ = ctx.timed(replay, reps, 2)
        out[name] = el / reps * 1e3
        hs[name].copy_(h0)
    res = {"w6_ms_per_step": round(out["w6"], 4), "fp16_ms_per_step": round(out["fp16"], 4),
           "speedup_vs_fp16": round(out["fp16"] / out["w6"], 3), "tok_per_s": round(M * 1e3 / out["w6"], 2),
           "fp16_tok_per_s": round(M * 1e3 / out["fp16"], 2)}
    if tp > 1:
        res["w6_no_allreduce_ms_per_step"] = round(out["w6_noreduce"], 4)
        res["allreduce_share"] = round(max(0.0, 1 - out["w6_noreduce"] / out["w6"]), 4)
    del w6, w16
    torch.cuda.empty_cache()
    return res


def optional(res, key, fn, ctx=None, need_bytes=0):
    """An optional section of the line (the replicas, C4, the decoder layers): an exception there
    is recorded under `key` instead of costing the headline line.  With several ranks the ranks
    agree before (every rank must have `need_bytes` of device memory free -- all ranks' share
    under --share-gpu -- or the section is skipped on all) and after (a failure on any rank is a
    failure on every rank), so no rank goes on to the next section's collectives alone."""
    multi = ctx is not None and ctx.world > 1
    if need_bytes:
        free = torch.cuda.mem_get_info(ctx.dev if ctx is not None else None)[0]
        want = 1.15 * need_bytes * (ctx.world if multi and ctx.staged else 1)
        short = 1.0 if free < want else 0.0
        if (ctx.max_over_ranks(short) if multi else short) > 0:
            res[key] = {"skipped": f"needs ~{want / 1e9:.1f} GB of free device memory per GPU "
                                   f"({free / 1e9:.1f} GB free on this rank)"}
            print(f"[bench] optional section {key} skipped: {res[key]['skipped']}", file=sys.stderr, flush=True)
            return
    err = None
    try:
        out = fn()
    except Exception as e:  # noqa: BLE001
        err = f"{type(e).__name__}: {e}"[:500]
        print(f"[bench] optional section {key} failed: {e}", file=sys.stderr, flush=True)
        torch.cuda.empty_cache()
    if multi and ctx.max_over_ranks(1.0 if err else 0.0) > 0 and err is None:
        err = "failed on another rank"
    res[key] = {"error": err} if err else out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one process per GPU); outside torchrun, N > 1 starts them itself")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="llama2-7b-m1", choices=sorted(CONFIGS))
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of one HIP graph")
    ap.add_argument("--no-merge", action="store_true",
                    help="launch gate and up separately (default: one linear over their concatenated weights)")
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of CPU baseline (0 = skip)")
    ap.add_argument("--roofline-reps", type=int, default=10)
    ap.add_argument("--no-fp16-compare", action="store_true", help="skip the rocBLAS fp16 comparison")
    ap.add_argument("--no-calibrate", action="store_true", help="skip the on-box HBM / MFMA peak calibration")
    ap.add_argument("--parallel", choices=["c4", "tp", "dp"], default="c4",
                    help="N > 1, what `value` measures: c4 (default) = BASELINE config C4, the LLaMA-2-70B stack "
                         "with every linear column-sharded over the N GPUs + one all-gather per linear (RCCL, or "
                         "the peer-store gather when bit-identical and faster), total work fixed (strong scaling, "
                         "SURVEY.md §8(e)); tp = the same split of the --config stack (LLaMA-2-7B); dp = "
                         "independent replicas of the --config stack, one token stream per GPU (weak scaling).  "
                         "The others are measured beside it in the same line (`tp_llama2_7b`, `replicas`)")
    ap.add_argument("--no-replicas", action="store_true", help="N > 1, tp: skip the replica (dp) measurement")
    ap.add_argument("--no-tp", action="store_true", help="N > 1, dp: skip the column-parallel (tp) measurement")
    ap.add_argument("--no-peer", action="store_true",
                    help="N > 1, tp: skip the peer-store gather variant (all-gather fused into the GEMM epilogue)")
    ap.add_argument("--no-c4", action="store_true",
                    help="N > 1: skip the LLaMA-2-70B column-parallel measurement (BASELINE config C4)")
    ap.add_argument("--no-extra-configs", action="store_true",
                    help="N = 1: skip the C3 (batch 16) and C5 (prefill) steps measured beside the headline")
    ap.add_argument("--no-reference-sweep", action="store_true",
                    help="N = 1: skip the reference's kernel sweep (engine/test_flexq_kernel.sh, README.md:189's form)")
    ap.add_argument("--no-layers", action="store_true",
                    help="skip the end-to-end decoder-layer comparison against fp16 (M = 1 and 16)")
    ap.add_argument("--no-qo", action="store_true",
                    help="prefill steps: skip the form with each quantize in the previous GEMM's epilogue")
    ap.add_argument("--no-chain", action="store_true",
                    help="N = 1 decode: time only one launch per linear (default: also the decode chains, "
                         "fq_linear_chain_w6ax, taken for `value` when bit-identical and faster)")
    ap.add_argument("--detail-out", default=os.path.join(ROOT, "gpurun_out", "bench_detail.json"),
                    help="file for the full result (every comparison row); the printed line is its summary "
                         "(<= %d chars, what the driver parses); '' = none" % LINE_MAX)
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal only: every rank on cuda:0, gloo with host-staged gathers, no graph")
    a = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(spawn_ranks(a))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        print(f"[bench] --gpus {a.gpus} but WORLD_SIZE={world}: launch N ranks with torchrun "
              f"--nproc-per-node N, or run bench.py --gpus N without torchrun", file=sys.stderr)
        sys.exit(2)
    staged = a.share_gpu and world > 1
    dev = torch.device("cuda", 0 if a.share_gpu else local)
    torch.cuda.set_device(dev)
    if world > 1:
        if staged:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    ctx = Ctx(a, rank, world, dev, staged)

    cfg = CONFIGS[a.config]
    # N > 1 headline: BASELINE config C4 (the 70B column split) unless --parallel tp / dp; at N = 1 the
    # --config stack (BASELINE configs[1] by default) with C4's one-GPU point measured beside it
    c4_head = world > 1 and a.parallel == "c4" and CONFIGS[a.config][1] <= PREFILL_M
    hcfg = CONFIGS["llama2-70b-m1"] if c4_head else cfg
    layers, M, lins, desc = hcfg
    merge = not a.no_merge
    launch_lins = launch_list(lins, merge)
    tp = world if (a.parallel == "tp" or c4_head) else 1  # ranks one linear is sharded over
    prefill = M > PREFILL_M
    n_lin = layers * len(launch_lins)
    flops_step = layers * sum(2.0 * M * N * K for (_, N, K, _) in lins)  # whole model, counted once

    decode_form, chain_sec = "one fq_linear_w6ax launch per linear", None
    if tp > 1:
        r = measure_tp(ctx, hcfg, merge, tp, a.steps, a.warmup)
        # The column-parallel step's all-gather has two implementations: RCCL's all_gather and the
        # peer-store gather fused into the GEMM epilogue.  Both run; the peer one is
        # taken for `value` only when every rank's step output is bit-identical to the RCCL run's,
        # no wait timed out and it is faster (never in the --share-gpu rehearsal).
        gather_impl, r_rccl, peer_sec = "rccl all_gather_into_tensor", r, {}
        if not a.no_peer and M <= PREFILL_M:
            optional(peer_sec, "p", lambda: measure_tp(ctx, hcfg, merge, tp, a.steps, a.warmup, peer=True), ctx)
            rp = peer_sec["p"]
            if "final" in rp:
                bad = 0.0 if (rp["finite"] and np.array_equal(rp["final"].view(np.uint16),
                                                              r["final"].view(np.uint16))) else 1.0
                rp["bit_identical_to_rccl"] = ctx.max_over_ranks(bad) == 0.0
                if rp["bit_identical_to_rccl"] and rp["elapsed"] < r["elapsed"] and not staged:
                    r, gather_impl = rp, "peer-store gather in the GEMM epilogue (fq_linear_w6ax_gather)"
        elapsed = r["elapsed"]
        value = flops_step * a.steps / elapsed / 1e12
        tok_s = M * a.steps / elapsed
        per_launch_s = r["per_launch_us"] / 1e6
        bytes_launch = r["alg_bytes_per_launch"]
        read_launch = bytes_launch
        fused_all = r["fused_launches"]
        use_graph = r["graph"]
        finite = r["finite"]
    else:
        stack = build_stack(cfg, rank, 1, dev, merge)
        use_graph = not a.no_graph
        replay = ctx.prepare(lambda: run_step(stack, M, 1), use_graph)
        elapsed, ev_s = ctx.timed(replay, a.steps, a.warmup)
        if M <= 4 and not prefill and not a.no_chain:
            # the same step as decode chains: one persistent launch per run of linears between attention
            # cores, each linear waiting in-kernel for its input; taken for `value` only
            # when the step's output is bit-identical, no in-kernel wait timed out, and it is faster
            last_out = linears(stack)[-1][1]["out"]
            ref_bits = last_out.cpu().numpy().view(np.uint16).copy()
            runs = chain_runs(stack)
            replay_c = ctx.prepare(lambda: run_chains(runs), use_graph)
            el_c, ev_c = ctx.timed(replay_c, a.steps, a.warmup)
            same = bool(np.array_equal(last_out.cpu().numpy().view(np.uint16), ref_bits))
            err = ops.chain_error(dev, stream=ctx.stream)
            chain_sec = {"what": "the same step as decode chains (fq_linear_chain_w6ax): qkv_0 | o_i, gate_up_i, "
                                 "down_i, qkv_i+1 | ... -- one persistent launch per run between attention cores, "
                                 "each linear's weight stream issued before it waits in-kernel for its input "
                                 "(tagged hand-off granules)",
                         "launches_per_step": len(runs), "ms_per_step": round(el_c / a.steps * 1e3, 4),
                         "launches_ms_per_step": round(elapsed / a.steps * 1e3, 4),
                         "bit_identical_to_launches": same, "wait_timed_out": bool(err)}
            if same and not err and el_c < elapsed:
                elapsed, ev_s = el_c, ev_c
                decode_form = f"decode chains: {len(runs)} persistent launches per step (fq_linear_chain_w6ax)"
            del replay_c
        replicas = world  # independent token streams (dp), each through the whole model
        value = replicas * flops_step * a.steps / elapsed / 1e12
        tok_s = replicas * M * a.steps / elapsed
        # roofline of the dominant kernel: the timed region itself (only the linear launches run
        # in it), HIP events on the launch stream
        per_launch_s = ev_s / (a.steps * n_lin)
        fused = {(N, K): ops.act_scratch_bytes(M, N, K) == 0 for (_, N, K, _) in launch_lins}
        fused_all = all(fused.values())
        bytes_launch = layers * sum(alg_bytes(M, N, K, ab, fused[(N, K)]) for (_, N, K, ab) in launch_lins) / n_lin
        read_launch = layers * sum(alg_read_bytes(M, N, K, ab, fused[(N, K)]) for (_, N, K, ab) in launch_lins) / n_lin
        last = linears(stack)[-1][1]["out"]
        finite = bool(torch.isfinite(last.float()).all().item())
        if prefill:  # MFMA-bound: the dominant kernel is the prefill GEMM; time its launches alone
            codes = {}
            for name, p in linears(stack):
                if name not in codes:
                    codes[name] = ops.quantize_act(p["x"], p["abits"])

            def gemms():
                for name, p in linears(stack):
                    ops.gemm_w6ax(codes[name][0], codes[name][1], p["pk"], p["Nl"], p["abits"], out=p["out"],
                                  w_u8=p.get("w_u8"))

            _, per_gemm_s = ctx.graph_time(gemms, n_lin, a.roofline_reps)
            ops_launch = layers * sum(2.0 * M * N * K for (_, N, K, _) in launch_lins) / n_lin
            del codes
        del stack, replay
        torch.cuda.empty_cache()

    achieved = bytes_launch / per_launch_s / 1e9
    traffic, traffic_src = pmc_traffic(a.config, merge) if tp == 1 else (None, None)
    res = {
        "metric": "W6A6 GEMM TFLOPS-equiv + tok/s on LLaMA-2-7B linear shapes, 1/2/4/8 GPU",
        "value": round(value, 4),
        "unit": "TFLOPS-equiv",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(elapsed / a.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if tp > 1 else "weak",
        "vs_baseline": None,
        "dtype": "int8-mfma(w6a%d)->fp16" % max(ab for (_, _, _, ab) in lins) if prefill else "int8-mfma(w6a6)->fp16",
        "data": "synthetic (random-init int6 weights of the architecture with unit-gain scales; N(0,1) fp16 "
                "token, each linear reading the previous linear's output)",
        "outputs_finite": finite,
        "tok_per_s": round(tok_s, 2),
        "config": {
            "workload": ("BASELINE config C4: " if c4_head else "") + desc +
                        ", dependent linear stack of every decoder layer per step",
            "layers": layers, "batch_M": M,
            "shapes_NxK": [[N, K, ab] for (_, N, K, ab) in lins],
            "parallelism": (f"tp{world}: every linear column-parallel (N/{world} rows per rank) + one "
                            f"all-gather of its fp16 output per linear ({gather_impl})" if tp > 1 else
                            f"dp{world}: independent replicas, one token stream per GPU, no data-path collective"),
            "graph": use_graph,
            "launches_per_layer": [[name, N // tp, K, ab] for (name, N, K, ab) in launch_lins],
            "decode_form": decode_form if tp == 1 else "one launch per linear",
        },
        "roofline": {
            "kernel": ("fq_gemm_decode_chain_kernel (per linear: step time / linears)" if
                       (tp == 1 and decode_form.startswith("decode chains")) else
                       "fq_gemm_decode_kernel<FUSE>" if fused_all else
                       "fq_gemm_decode_kernel (+ quantize where unfused)"),
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "traffic_over_alg": round(traffic / read_launch, 4) if traffic else None,
            "traffic_vs": "algorithmic READ bytes per launch (FETCH_SIZE counts reads only)",
            "per_launch_us": round(per_launch_s * 1e6, 3),
            "alg_bytes_per_launch": int(bytes_launch),
            "fused_launches": fused_all,
            "method": ("HIP events on the launch stream around the timed steps (only the linear launches run)"
                       if tp == 1 else "per rank: graph of the step's linear launches only (no all-gather), "
                                       "HIP events on the capture stream; max over ranks"),
        },
    }
    if tp == 1 and chain_sec is not None:
        res["decode_chain"] = chain_sec
    if staged:
        res["rehearsal"] = "--share-gpu: all ranks on one GPU, gloo with host-staged gathers (not a valid result)"
    if world > 1:  # what the collectives actually ran on
        res["comm"] = {"world_size": dist.get_world_size(), "backend": str(dist.get_backend()),
                       "rccl_version": ".".join(str(v) for v in torch.cuda.nccl.version())
                       if dist.get_backend() == "nccl" else None}
    if tp > 1:  # the same workload on one GPU, same node, same run: the curve's like-for-like point
        def same_1gpu():
            ms1 = measure_alone(ctx, hcfg, merge, max(2, a.steps // 2), max(1, a.warmup // 2))
            return scaling_vs_1gpu(elapsed / a.steps * 1e3, ms1, world,
                                   f"`value`'s workload ({'C4' if c4_head else a.config}) unsharded on one GPU "
                                   "(rank 0 alone, per-linear launches in one graph) vs its column split over the "
                                   f"{world} GPUs; vs_baseline stays null (BASELINE.md publishes no number)")
        optional(res, "same_workload_1gpu", same_1gpu, ctx)  # (rank 0 alone holds the unsharded weights)
    if prefill and tp == 1:
        ach = ops_launch / per_gemm_s / 1e12
        bytes_pf = int(layers * sum(alg_bytes(M, N, K, ab, False) for (_, N, K, ab) in launch_lins) / n_lin)
        read_pf = int(layers * sum(alg_read_bytes(M, N, K, ab, False) for (_, N, K, ab) in launch_lins) / n_lin)
        res["roofline"] = {
            "kernel": "fq_gemm_prefill_big_kernel" if M >= 2048 else "fq_gemm_prefill_kernel",
            "bound": "mfma",
            "achieved": round(ach, 1),
            "peak": I8_MFMA_PEAK_TOPS,
            "unit": "TFLOP/s",
            "frac": round(ach / I8_MFMA_PEAK_TOPS, 4),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "traffic_over_alg": round(traffic / read_pf, 4) if traffic else None,
            "traffic_vs": "algorithmic READ bytes per GEMM launch (FETCH_SIZE counts reads only)",
            "per_launch_us": round(per_gemm_s * 1e6, 3),
            "alg_ops_per_launch": ops_launch,
            "alg_bytes_per_launch": bytes_pf,
            "step_ms_linears_incl_quantize": round(elapsed / a.steps * 1e3, 4),
            "method": "graph of the step's prefill GEMM launches on pre-quantized codes (the quantize "
                      "launches excluded), HIP events on the capture stream; TOPS = 2*M*N*K / launch time",
        }
    def tp_summary(rr):
        return {k: (round(v, 4) if isinstance(v, float) else v) for k, v in rr.items()
                if k not in ("elapsed", "flops_step", "finite", "final")}
    if world > 1 and (tp == 1 or c4_head) and not a.no_tp:
        # the north-star split of the same stack, measured beside the replicas: every
        # linear column-parallel over the N GPUs + one RCCL all-gather per linear (strong scaling)
        def tp_rccl():
            rr = measure_tp(ctx, cfg, merge, world, a.steps, a.warmup)
            ms1 = measure_alone(ctx, cfg, merge, max(2, a.steps // 2), max(1, a.warmup // 2))
            sc = scaling_vs_1gpu(rr["ms_per_step"], ms1, world, "")
            return {"what": f"tp{world}: the same stack, every linear column-parallel (N/{world} rows per rank) "
                            "+ one RCCL all_gather_into_tensor of its fp16 output per linear (strong scaling)",
                    "value": round(rr["flops_step"] * a.steps / rr["elapsed"] / 1e12, 4), "unit": "TFLOPS-equiv",
                    "tok_per_s": round(M * a.steps / rr["elapsed"], 2), **tp_summary(rr),
                    "finite": rr["finite"], "hbm_frac_per_rank": round(rr["hbm_GBps_per_rank"] / HBM_PEAK_GBS, 4),
                    **{k: v for k, v in sc.items() if k not in ("what", "ms_per_step")}}
        optional(res, "tp_llama2_7b" if c4_head else "tp", tp_rccl, ctx)
    if tp > 1:
        res["tp"] = tp_summary(r)
        res["tp"]["gather"] = gather_impl
        res["tp"]["rccl_ms_per_step"] = round(r_rccl["ms_per_step"], 4)
        res["tp"]["hbm_frac_per_rank"] = round(r["hbm_GBps_per_rank"] / HBM_PEAK_GBS, 4)
        if not a.no_replicas:  # the --config model as independent replicas, one token stream per GPU
            # (the replicas run the --config stack, 7B by default)
            flops_step_r = cfg[0] * sum(2.0 * cfg[1] * N * K for (_, N, K, _) in cfg[2])

            def replicas():
                stack = build_stack(cfg, rank, 1, dev, merge)
                replay = ctx.prepare(lambda: run_step(stack, cfg[1], 1), not a.no_graph)
                el_dp, _ = ctx.timed(replay, a.steps, a.warmup)
                del stack, replay
                torch.cuda.empty_cache()
                return {"what": f"dp{world}: the whole {a.config} model on every GPU, independent token streams, "
                                "no data-path collective (weak scaling)",
                        "value": round(world * flops_step_r * a.steps / el_dp / 1e12, 4),
                        "tok_per_s": round(world * cfg[1] * a.steps / el_dp, 2),
                        "ms_per_step": round(el_dp / a.steps * 1e3, 4)}
            need = cfg[0] * sum(ops.packed_w_bytes(N, K) for (_, N, K, _) in launch_list(cfg[2], merge))
            optional(res, "replicas", replicas, ctx, need_bytes=need)
    if world > 1:
        if not a.no_peer and M <= 32:  # the all-gather fused into the GEMM epilogue
            def tp_peer(c):
                rp = measure_tp(ctx, c, merge, world, max(2, a.steps // 2), max(1, a.warmup // 2), peer=True)
                return {"what": "the same column-parallel stack, each all-gather fused into its GEMM's epilogue: "
                                "peer stores into IPC-mapped gather buffers + one wait launch per linear "
                                "(fq_linear_w6ax_gather / fq_gather_wait) instead of an RCCL all_gather",
                        "value": round(rp["flops_step"] / (rp["ms_per_step"] / 1e3) / 1e12, 4),
                        "unit": "TFLOPS-equiv", "tok_per_s": round(M * 1e3 / rp["ms_per_step"], 2),
                        "ms_per_step": round(rp["ms_per_step"], 4),
                        "gemm_only_ms_per_step": round(rp["gemm_only_ms_per_step"], 4),
                        "finite": rp["finite"], "graph": rp["graph"]}
            rp = peer_sec.get("p") if tp > 1 else None
            if (tp == 1 or c4_head) and not a.no_tp:
                optional(res, "tp_llama2_7b_peer_gather" if c4_head else "tp_peer_gather", lambda: tp_peer(cfg), ctx)
            if rp is not None and "final" in rp:
                res["tp_peer_gather"] = {
                    "what": "the same column-parallel stack, each all-gather fused into its GEMM's epilogue: peer "
                            "stores into IPC-mapped gather buffers + one wait launch per linear "
                            "(fq_linear_w6ax_gather / fq_gather_wait) instead of an RCCL all_gather",
                    "value": round(rp["flops_step"] / (rp["ms_per_step"] / 1e3) / 1e12, 4), "unit": "TFLOPS-equiv",
                    "tok_per_s": round(M * 1e3 / rp["ms_per_step"], 2), "ms_per_step": round(rp["ms_per_step"], 4),
                    "gemm_only_ms_per_step": round(rp["gemm_only_ms_per_step"], 4), "finite": rp["finite"],
                    "bit_identical_to_rccl": rp["bit_identical_to_rccl"], "graph": rp["graph"]}
            elif rp is not None:
                res["tp_peer_gather"] = rp
            if not a.no_c4 and a.config != "llama2-70b-m1" and not c4_head:
                optional(res, "c4_llama2_70b_tp_peer_gather", lambda: tp_peer(CONFIGS["llama2-70b-m1"]), ctx)
        if not a.no_c4 and a.config != "llama2-70b-m1" and not prefill and not c4_head:
            def c4_tp():
                c4 = CONFIGS["llama2-70b-m1"]
                rc = measure_tp(ctx, c4, merge, world, max(2, a.steps // 2), max(1, a.warmup // 2))
                ms1 = measure_alone(ctx, c4, merge, max(2, a.steps // 2), max(1, a.warmup // 2))
                sc = scaling_vs_1gpu(rc["ms_per_step"], ms1, world, "")
                return {**{k: v for k, v in sc.items() if k not in ("what", "ms_per_step")},
                    "what": f"BASELINE config C4: {c4[3]}, column-parallel over {world} GPUs + one RCCL "
                            f"all-gather per linear ({c4[0]} layers, {len(launch_list(c4[2], merge))} launches each)",
                    "value": round(rc["flops_step"] / (rc["ms_per_step"] / 1e3) / 1e12, 4),
                    "unit": "TFLOPS-equiv", "tok_per_s": round(1e3 / rc["ms_per_step"], 2),
                    **{k: (round(v, 4) if isinstance(v, float) else v) for k, v in rc.items()
                       if k not in ("elapsed", "flops_step", "final")},
                    "hbm_frac_per_rank": round(rc["hbm_GBps_per_rank"] / HBM_PEAK_GBS, 4)}
            optional(res, "c4_llama2_70b_tp", c4_tp, ctx)
    if world == 1 and not a.no_extra_configs:  # the other single-GPU BASELINE configs, same run
        for key, name, st, wu in (("c3_llama2_7b_m16", "llama2-7b-m16", 10, 3),
                                  ("c5_llama3_8b_prefill", "llama3-8b-prefill", 2, 1),
                                  ("c4_llama2_70b_1gpu", "llama2-70b-m1", 10, 3)):
            if name != a.config:
                need = CONFIGS[name][0] * sum(ops.packed_w_bytes(N, K) for (_, N, K, _) in
                                              launch_list(CONFIGS[name][2], merge))
                optional(res, key, lambda name=name, st=st, wu=wu: measure_single(ctx, name, merge, st, wu), ctx,
                         need_bytes=need)
        if res.get("c4_llama2_70b_1gpu", {}).get("value"):
            res["c4_llama2_70b_1gpu"]["note"] = ("C4's one-GPU point: bench.py --gpus N (N > 1) reports C4 split "
                                                 "over the N GPUs as `value`")
            res["c4_llama2_70b_1gpu"]["baseline_for"] = "--gpus N --parallel c4 (the N > 1 default): value"
    if not a.no_layers and not prefill and a.config.startswith("llama2-7b"):
        optional(res, "decoder_layers_e2e", lambda: {
            "what": f"LLaMA-2-7B decoder layers end to end (32 layers; RMSNorm, qkv, o, gate_up, SiLU*up, down, "
                    f"residuals; attention core out of scope: ctx = v), FT's TP layout over {world} rank(s) "
                    f"(row-parallel o/down + one all-reduce each), W6A6 (down W6A8) engine vs fp16 torch "
                    f"(F.rms_norm, hipBLASLt F.linear, F.silu), one HIP graph each; README.md:193's comparison",
            "tp": world,
            **{f"M{m}": decoder_layers_e2e(ctx, m) for m in (1, 16)}}, ctx)
    if world == 1 and not a.no_calibrate:
        res["roofline"]["peak_measured"] = calibrate_peaks(dev)
        pm = res["roofline"]["peak_measured"]
        res["roofline"]["frac_of_measured"] = round(
            (ach / pm["int8_mfma_TOPS"]) if prefill else (achieved / pm["hbm_read_GBps"]), 4)
    if world == 1 and not a.no_fp16_compare:
        torch.cuda.empty_cache()
        shapes = sorted({(N, K) for (_, N, K, _) in lins})
        ab_cfg = max(ab for (_, _, _, ab) in lins)
        cmp_cfg = fp16_compare(shapes, M, ab_cfg, dev, reps=20 if not prefill else 4, int8=True)
        geo = lambda rows: round(float(np.exp(np.mean([np.log(r["speedup"]) for r in rows]))), 3)  # noqa: E731
        res["vs_rocblas_fp16"] = {
            "what": f"W6A{ab_cfg} linear (quantize+GEMM, one launch where fused) vs torch F.linear fp16 "
                    "(hipBLASLt/rocBLAS), same M,N,K, graph-timed; config shapes also vs the vendor int8 "
                    "GEMM torch._int_mm (context only: int8 x int8 -> int32, no quantize or dequant, "
                    "int8_vendor_M = the smallest M it accepts)",
            "config_shapes": cmp_cfg, "config_geomean_speedup": geo(cmp_cfg),
        }
        i8 = [r["speedup_vs_int8"] for r in cmp_cfg if "speedup_vs_int8" in r]
        if i8:
            res["vs_rocblas_fp16"]["config_geomean_speedup_vs_int8"] = round(float(np.exp(np.mean(np.log(i8)))), 3)
        if not prefill:
            cmp_ns = {m: fp16_compare(NORTH_STAR_SHAPES, m, 6, dev) for m in (1, 2, 4, 8)}
            res["vs_rocblas_fp16"].update({
                "llama2_70b_m1": cmp_ns[1], "llama2_70b_m1_geomean_speedup": geo(cmp_ns[1]),
                "llama2_70b_geomean_speedup_by_M": {str(m): geo(r) for m, r in cmp_ns.items()},
                "north_star_target": 1.3})
    if world == 1 and not a.no_reference_sweep and not prefill:
        optional(res, "vs_reference_sweep", lambda: reference_sweep(dev), ctx)
    if rank == 0 and world == 1 and a.cpu_budget > 0:
        res["cpu_baseline"] = cpu_baseline(a.cpu_budget, lins, M)
    if rank == 0:
        print(json.dumps(compact_line(res, write_detail(res, a.detail_out))), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
