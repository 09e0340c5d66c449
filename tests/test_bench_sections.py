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
