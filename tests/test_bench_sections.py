"""bench.py's optional sections with several ranks (CPU, gloo, world size 2): a section that fails on
ONE rank is recorded as failed on every rank, and the ranks stay in step for the next section's
collectives (the driver's 8-GPU run must never diverge into mismatched collectives and hang)."""
import os
import socket
import sys
import types

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, q):
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import bench
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        ctx = types.SimpleNamespace(world=world, rank=rank, staged=False, dev=torch.device("cpu"))
        ctx.max_over_ranks = lambda v: bench.Ctx.max_over_ranks(ctx, v)
        res = {}

        def flaky():
            if rank == 1:
                raise RuntimeError("out of memory on this rank only")
            return {"ok": True}
        bench.optional(res, "first", flaky, ctx)

        def fine():
            t = torch.tensor([float(rank + 1)])
            dist.all_reduce(t)  # a collective inside the next section: both ranks must reach it
            return {"sum": float(t.item())}
        bench.optional(res, "second", fine, ctx)
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_optional_section_failure_is_agreed_across_ranks():
    import torch.multiprocessing as mp
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p_ in procs:
        p_.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p_ in procs:
        p_.join(timeout=60)
        assert p_.exitcode == 0
    for r in range(2):
        assert "error" in res[r]["first"], res[r]
        assert res[r]["second"] == {"sum": 3.0}
    assert "another rank" in res[0]["first"]["error"] and "out of memory" in res[1]["first"]["error"]


def _r04_result():
    """Round 4's full N = 1 result (28,196 characters as one line: the driver could not parse it)."""
    import json
    with open(os.path.join(ROOT, "profiles", "r04_bench_final.json")) as f:
        return json.loads(f.readline())


def test_driver_line_fits_and_keeps_the_headline():
    """The printed line stays under the driver's limit on a full N = 1 result, keeps every essential key
    (value, roofline, cpu_baseline, ...) and the per-M averages of the reference sweep, and folds the
    per-shape rows away (they are in the detail file)."""
    import json
    sys.path.insert(0, ROOT)
    import bench
    res = _r04_result()
    assert len(json.dumps(res)) > 20000  # the representative input really is the oversized one
    line = bench.compact_line(res, "gpurun_out/bench_detail.json")
    text = json.dumps(line)
    assert len(text) < 6000, len(text)
    for k in bench.ESSENTIAL:
        assert k in line, k
    assert line["value"] == res["value"] and line["ms_per_step"] == res["ms_per_step"]
    assert line["roofline"]["frac"] == res["roofline"]["frac"] and line["roofline"]["bound"] == "hbm"
    assert line["cpu_baseline"]["cores"] == 16 and line["cpu_baseline"]["kind"] == "port"
    for k in ("c3_llama2_7b_m16", "c5_llama3_8b_prefill", "c4_llama2_70b_1gpu", "decode_chain"):
        assert isinstance(line[k], dict) and "roofline" in line[k] or k == "decode_chain", k
    sweep = line["vs_reference_sweep"]
    assert "shapes" not in sweep and sweep["avg_speedup_vs_int8_by_M"] == res["vs_reference_sweep"]["avg_speedup_vs_int8_by_M"]
    assert line["detail_file"] == "gpurun_out/bench_detail.json"


def test_driver_line_drops_sections_rather_than_overflow():
    """Even with every multi-GPU section present and oversized, the line stays under the limit: whole
    optional sections give way (in DROP_ORDER), never the essentials."""
    import json
    sys.path.insert(0, ROOT)
    import bench
    res = _r04_result()
    big = {"what": "x" * 3000, "ms_per_step": 1.0, "rows": [{"a": i, "b": float(i)} for i in range(200)]}
    for k in ("tp", "tp_llama2_7b", "tp_peer_gather", "tp_llama2_7b_peer_gather", "c4_llama2_70b_tp",
              "c4_llama2_70b_tp_peer_gather", "replicas"):
        res[k] = dict(big)
    line = bench.compact_line(res, "d.json")
    assert len(json.dumps(line)) < 6000
    for k in bench.ESSENTIAL:
        assert k in line, k
    assert bench.compact_line({k: res[k] for k in bench.ESSENTIAL if k in res})["value"] == res["value"]


def test_chain_runs_cut_at_the_attention_cores():
    """bench.chain_runs: the step's linears in order, cut before every o_proj (the attention core sits
    between qkv and o), so 32 LLaMA layers give qkv_0 | (o, gate_up, down, qkv) x 31 | o, gate_up, down."""
    sys.path.insert(0, ROOT)
    import bench
    layer = lambda i: {n: dict(x=f"x{n}{i}", pk=f"w{n}{i}", Nl=1, abits=6, out=f"d{n}{i}")  # noqa: E731
                       for n in ("qkv", "o", "gate_up", "down")}
    runs = bench.chain_runs([layer(i) for i in range(32)])
    assert len(runs) == 33
    assert [r[1] for r in runs[0]] == ["wqkv0"]
    assert [r[1] for r in runs[1]] == ["wo0", "wgate_up0", "wdown0", "wqkv1"]
    assert [r[1] for r in runs[-1]] == ["wo31", "wgate_up31", "wdown31"]
    assert sum(len(r) for r in runs) == 128


def test_multi_gpu_line_is_like_for_like():
    """an N > 1 line carries the same workload's one-GPU point measured in the same run
    (same_workload_1gpu: ms per step, speedup, strong-scaling efficiency), the 7B split's and C4's own
    one-GPU points, and the world size / backend the collectives ran on -- and keeps them, under the
    driver's 6,000-character limit, on a synthetic N = 8 result padded with every optional section."""
    import json
    sys.path.insert(0, ROOT)
    import bench
    with open(os.path.join(ROOT, "profiles", "r05_final_share2_rehearsal.json")) as f:
        res = json.loads(f.readline())
    res.pop("rehearsal", None)
    res["n_gpus"] = 8
    res["comm"] = {"world_size": 8, "backend": "nccl", "rccl_version": "2.26.6"}
    res["same_workload_1gpu"] = bench.scaling_vs_1gpu(1.60, 8.83, 8, "C4 unsharded on one GPU vs its split")
    res["tp_llama2_7b"].update({k: v for k, v in bench.scaling_vs_1gpu(0.70, 1.16, 8, "").items()
                                if k not in ("what", "ms_per_step")})
    res["c4_llama2_70b_tp"] = dict(res["tp"], **{k: v for k, v in bench.scaling_vs_1gpu(1.6, 8.83, 8, "").items()
                                                 if k not in ("what", "ms_per_step")})
    big = _r04_result()  # the N = 1 sections, as if a run had them all
    for k in ("vs_reference_sweep", "vs_rocblas_fp16", "c3_llama2_7b_m16", "c5_llama3_8b_prefill"):
        res[k] = big[k]
    line = bench.compact_line(res, "gpurun_out/bench_detail.json")
    text = json.dumps(line)
    assert len(text) <= bench.LINE_MAX, len(text)
    sw = line["same_workload_1gpu"]
    assert sw["ms_per_step_1gpu"] == 8.83 and sw["speedup_vs_1gpu"] == round(8.83 / 1.60, 4)
    assert sw["strong_scaling_efficiency"] == round(8.83 / 1.60 / 8, 4)
    assert line["comm"] == {"world_size": 8, "backend": "nccl", "rccl_version": "2.26.6"}
    assert line["vs_baseline"] is None  # BASELINE.md publishes no number for this metric
    for k in bench.ESSENTIAL:
        assert k in line or k == "cpu_baseline", k  # (the CPU baseline is timed at N = 1 only)
    # last resort (a line that would not fit even without the optional sections) keeps them too
    tiny = bench.compact_line(res, None, limit=10)
    assert "same_workload_1gpu" in tiny and "comm" in tiny


def test_round6_detail_file_folds_into_the_driver_line():
    """Round 6's full N = 1 result (the detail file of the final check: C3 with both quantize forms timed,
    C5 and C4 with theirs, the decoder layers, the reference sweep's per-shape rows) folds into a line
    under the limit with every essential key and the C3 epilogue-form record kept."""
    import json
    sys.path.insert(0, ROOT)
    import bench
    with open(os.path.join(ROOT, "profiles", "r06c_bench_detail.json")) as f:
        res = json.load(f)
    line = bench.compact_line(res, "d.json")
    assert len(json.dumps(line)) < 6000
    for k in bench.ESSENTIAL:
        assert k in line, k
    eq = line["c3_llama2_7b_m16"]["epilogue_quantize"]
    assert eq["last_output_identical"] and "taken" not in eq  # (slower in a graph: not taken)
    assert line["roofline"]["traffic_source"].startswith("profiles/r06")
