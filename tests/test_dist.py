"""Column-parallel sharding + the one all-gather, and row-parallel sharding (128-group column
split) + the one all-reduce, world_size 2 over gloo on CPU (the same code runs over RCCL on GPUs:
bench.py --gpus N --parallel tp, flexq_amd.layers with converter files)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from flexq_amd.dist import (all_reduce_sum, gather_columns, group_shard_range, shard_range, shard_scales,
                            shard_weight, shard_weight_k)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, M, N, K, q):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(0)
        w = torch.randn(N, K, generator=g)
        ws = torch.rand(K // 128, N, generator=g)
        x = torch.randn(M, K, generator=g)
        w_p, ws_p = shard_weight(w, world, rank), shard_scales(ws, world, rank)
        lo, hi = shard_range(N, world, rank)
        assert torch.equal(w_p, w[lo:hi]) and torch.equal(ws_p, ws[:, lo:hi])
        local = x @ w_p.t()                    # stands in for this rank's linear output
        full = gather_columns(local)
        pre = torch.full((M, N), float("nan"))  # caller-owned output (M = 1: gathered in place)
        got = gather_columns(local, out=pre)
        ok = torch.allclose(full, x @ w.t(), atol=1e-5) and got is pre and torch.equal(pre, full)
        q.put((rank, ok, tuple(full.shape)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("M", [1, 5])
def test_column_parallel_gather_world2(M):
    world, N, K = 2, 96, 256
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, M, N, K, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok, shape in res:
        assert ok and shape == (M, N), (rank, shape)


def test_shard_range_rules():
    assert shard_range(4096, 8, 3) == (1536, 2048)
    with pytest.raises(ValueError):
        shard_range(100, 2, 0)  # 50-column shards are not whole 16-column tiles


def _row_worker(rank, world, port, M, N, K, q):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(0)
        w = torch.randn(N, K, generator=g, dtype=torch.float64)
        x = torch.randn(M, K, generator=g, dtype=torch.float64)
        lo, hi = group_shard_range(K, world, rank)
        w_p = shard_weight_k(w, world, rank)
        assert torch.equal(w_p, w[:, lo:hi])
        part = x[:, lo:hi] @ w_p.t()           # this rank's partial output (its K slice)
        full = all_reduce_sum(part)
        q.put((rank, torch.allclose(full, x @ w.t(), atol=1e-9), tuple(full.shape)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("K", [512, 640])  # 640 = 5 groups: uneven 3 + 2 split
def test_row_parallel_all_reduce_world2(K):
    world, M, N = 2, 3, 48
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_row_worker, args=(r, world, port, M, N, K, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok, shape in res:
        assert ok and shape == (M, N), (rank, shape)


def test_group_shard_range_rules():
    # LLaMA-2-7B FFN width: 86 groups -> 22, 22, 21, 21 at P = 4; whole groups, contiguous, covering
    spans = [group_shard_range(11008, 4, r) for r in range(4)]
    assert spans == [(0, 2816), (2816, 5632), (5632, 8320), (8320, 11008)]
    for P in (1, 2, 3, 8):
        s = [group_shard_range(4096, P, r) for r in range(P)]
        assert s[0][0] == 0 and s[-1][1] == 4096 and all(a[1] == b[0] for a, b in zip(s, s[1:]))
        assert all((hi - lo) % 128 == 0 for lo, hi in s)
    assert group_shard_range(4096, 8, 3) == shard_range(4096, 8, 3)  # even case = the column rule
    with pytest.raises(ValueError):
        group_shard_range(100, 2, 0)
    with pytest.raises(ValueError):
        group_shard_range(256, 4, 0)  # 2 groups over 4 ranks
