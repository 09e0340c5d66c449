"""BASELINE config C4 as the reference runs it: the LLaMA-2-70B linears of
engine/test_flexq_kernel.sh:25-28 (24576x8192, 8192x8192, 28672x8192, 8192x28672) split 8 ways
column-parallel and gathered (the reference's ftNcclAllGather, e2e/src/fastertransformer/utils/
nccl_utils.cc:70-82).  Eight real processes share the box's one GPU (gloo carries the all-gather;
RCCL over xGMI on an 8-GPU node runs the same ColumnParallelW6Linear code).  Each rank builds ONLY
its shard of every weight (deterministic integer codes and exactly representable scales, a function
of the global row, so the oracle can rebuild any column), packs it into its weight image and runs
the HIP linear at M = 1 (fused) and M = 8 (separate quantize launch).  The gathered [M, N] is held
against the CPU oracle on 96 sampled columns spanning all eight shards, and the ranks agree bit for
bit on the whole output."""
import socket

import numpy as np
import pytest
import torch

from common import assert_gemm_close, oracle
from inputs import act_input

WORLD = 8
SHAPES = [(24576, 8192), (8192, 8192), (28672, 8192), (8192, 28672)]
MS = (1, 8)
PER_RANK = 12  # sampled columns per shard -> 96


def _mix(v, xp):
    """32-bit integer hash (identical in torch and numpy int64 arithmetic)."""
    m = 0xFFFFFFFF
    v = v & m
    v = v ^ (v >> 13)
    v = (v * 0x5BD1E995) & m
    v = v ^ (v >> 15)
    return v


def weight_codes(rows, K, xp):
    """int6 codes [len(rows), K] of global weight rows `rows` (xp = torch or numpy)."""
    if xp is torch:
        n = rows.to(torch.int64)[:, None]
        k = torch.arange(K, dtype=torch.int64, device=rows.device)[None, :]
    else:
        n = rows.astype(np.int64)[:, None]
        k = np.arange(K, dtype=np.int64)[None, :]
    h = _mix(n * 1000003 + k * 7919 + 12345, xp)
    c = ((h >> 8) & 63) - 32
    return c.to(torch.int8) if xp is torch else c.astype(np.int8)


def weight_scales(rows, K, xp):
    """fp16 [K/128, len(rows)] in [2^-10, 2^-9): exactly representable, a function of (row, group)."""
    G = K // 128
    if xp is torch:
        n = rows.to(torch.int64)[None, :]
        g = torch.arange(G, dtype=torch.int64, device=rows.device)[:, None]
        h = _mix(n * 31337 + g * 977 + 7, xp)
        return (((h & 1023) + 1024).to(torch.float32) * 2.0 ** -20).to(torch.float16)
    n = rows.astype(np.int64)[None, :]
    g = np.arange(G, dtype=np.int64)[:, None]
    h = _mix(n * 31337 + g * 977 + 7, xp)
    return (((h & 1023) + 1024).astype(np.float32) * np.float32(2.0 ** -20)).astype(np.float16)


def sampled_columns(N):
    n = N // WORLD
    return np.concatenate([r * n + np.linspace(0, n - 1, PER_RANK).astype(np.int64) for r in range(WORLD)])


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from flexq_amd import dist as fqd
    from flexq_amd import ops
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda:0")
        for (N, K) in SHAPES:
            lo, hi = fqd.shard_range(N, world, rank)
            rows = torch.arange(lo, hi, device=dev)
            img = ops.pack_w6(weight_codes(rows, K, torch), weight_scales(rows, K, torch))
            lin = fqd.ColumnParallelW6Linear(img, N, K, 6)
            for M in MS:
                x = torch.from_numpy(act_input(M, K, seed=40 + M).astype(np.float16)).to(dev)
                y = lin(x)
                torch.cuda.synchronize()
                q.put(((N, K, M, rank), y.cpu().numpy()))  # by value: the worker may exit first
            del img, lin
            torch.cuda.empty_cache()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_llama2_70b_column_parallel_world8(dev):
    import torch.multiprocessing as mp
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, q)) for r in range(WORLD)]
    for p_ in procs:
        p_.start()
    res = dict(q.get(timeout=110) for _ in range(WORLD * len(SHAPES) * len(MS)))
    for p_ in procs:
        p_.join(timeout=60)
        assert p_.exitcode == 0
    for (N, K) in SHAPES:
        cols = sampled_columns(N)
        wq = weight_codes(cols, K, np)
        ws = weight_scales(cols, K, np)
        for M in MS:
            x = act_input(M, K, seed=40 + M).astype(np.float16)
            xq, xs = oracle.quantize_engine(x, 6)
            ref, _, mag = oracle.gemm(xq, xs, wq, ws)
            y0 = res[(N, K, M, 0)]
            assert y0.shape == (M, N)
            assert_gemm_close(y0[:, cols], ref, mag, f"C4 {N}x{K} M={M} (8-way column-parallel)")
            for r in range(1, WORLD):
                np.testing.assert_array_equal(res[(N, K, M, r)].view(np.uint16), y0.view(np.uint16))


def test_weight_hash_torch_numpy_agree():
    """The per-rank GPU generator and the oracle's CPU rebuild give the same codes and scales
    (runs on the CPU device too)."""
    rows = np.array([0, 1, 17, 3583, 28671])
    for K in (128, 8192):
        tq = weight_codes(torch.from_numpy(rows), K, torch).numpy()
        nq = weight_codes(rows, K, np)
        np.testing.assert_array_equal(tq, nq)
        assert tq.min() >= -32 and tq.max() <= 31
        np.testing.assert_array_equal(weight_scales(torch.from_numpy(rows), K, torch).numpy().view(np.uint16),
                                      weight_scales(rows, K, np).view(np.uint16))
