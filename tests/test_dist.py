"""Column-parallel sharding + the one all-gather, world_size 2 over gloo on CPU (the same code
runs over RCCL on GPUs, bench.py --gpus N)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from flexq_amd.dist import gather_columns, shard_range, shard_scales, shard_weight


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
        q.put((rank, torch.allclose(full, x @ w.t(), atol=1e-5), tuple(full.shape)))
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
