"""The column-parallel N-shard (BASELINE config C4's scheme) on the GPU through
real processes: two ranks share the box's one GPU (gloo carries the all-gather here; RCCL over
xGMI on an 8-GPU node runs the same ColumnParallelW6Linear code), each packs ITS shard of the
weight into a weight image, runs the HIP linear on it and all-gathers the fp16 outputs.  The
gathered [M, N] is checked against the CPU oracle over the full N on every rank, and the ranks
agree bit for bit.  bench.py's --share-gpu rehearsal runs its multi-rank path the same way."""
import socket

import numpy as np
import pytest
import torch

from common import assert_gemm_close, oracle
from inputs import act_input, weight_input

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, M, N, K, abits, q):
    import torch.distributed as dist
    from flexq_amd import dist as fqd
    from flexq_amd import ops
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda:0")
        w = torch.from_numpy(weight_input(N, K, seed=21).astype(np.float16))
        x = torch.from_numpy(act_input(M, K, seed=22).astype(np.float16)).to(dev)
        img, _ = ops.quantize_pack_w6(fqd.shard_weight(w, world, rank).to(dev))
        lin = fqd.ColumnParallelW6Linear(img, N, K, abits)
        y = lin(x)
        torch.cuda.synchronize()
        q.put((rank, y.cpu()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("M,N,K,abits,world", [(1, 4096, 4096, 6, 2), (4, 1024, 2048, 8, 2), (1, 2560, 8192, 6, 4)])
def test_column_parallel_linear_multi_process(dev, M, N, K, abits, world):
    import torch.multiprocessing as mp
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, M, N, K, abits, q)) for r in range(world)]
    for p_ in procs:
        p_.start()
    res = dict(q.get(timeout=100) for _ in range(world))
    for p_ in procs:
        p_.join(timeout=60)
        assert p_.exitcode == 0
    w = weight_input(N, K, seed=21).astype(np.float16)
    x = act_input(M, K, seed=22).astype(np.float16)
    xq, xs = oracle.quantize_engine(x, abits)
    wq, ws = oracle.quantize_engine(w, 6)  # per-(row, group) codes: the same whether sharded or not
    ref, _, mag = oracle.gemm(xq, xs, wq, ws)
    for r in range(world):
        assert tuple(res[r].shape) == (M, N)
        assert_gemm_close(res[r].numpy(), ref, mag, f"column-parallel rank {r} of {world}")
        np.testing.assert_array_equal(res[r].numpy().view(np.uint16), res[0].numpy().view(np.uint16))


def _peer_worker(rank, world, port, cases, q):
    import torch.distributed as dist
    from flexq_amd import dist as fqd
    from flexq_amd import ops
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        out = {}
        for (M, N, K, abits, chain) in cases:
            w = torch.from_numpy(weight_input(N, K, seed=31).astype(np.float16))
            img, _ = ops.quantize_pack_w6(fqd.shard_weight(w, world, rank).to(dev))
            ref_lin = fqd.ColumnParallelW6Linear(img, N, K, abits)
            pg = fqd.PeerGather(M, N, device=dev)
            x = torch.from_numpy(act_input(M, K, seed=32).astype(np.float16)).to(dev)
            got, want = [], []
            for step in range(chain):
                y = pg.linear(x, img, abits)          # peer-store gather fused into the GEMM epilogue
                torch.cuda.synchronize()
                yr = ref_lin(x)                       # the RCCL/gloo all_gather path
                got.append(y.cpu().numpy().copy())
                want.append(yr.cpu().numpy())
                if K == N:
                    x = y.clone()                     # a dependent chain (next input = this output)
            # the folded form (K == N): every call reads the previous call's gather buffer in place and
            # waits for it inside its own launch (fq_linear_w6ax_gather_after), no wait launches, no
            # host synchronisation inside the chain; only the last output is waited for
            folded = []
            if K == N:
                x0 = torch.from_numpy(act_input(M, K, seed=32).astype(np.float16)).to(dev)
                pg2 = fqd.PeerGather(M, N, device=dev)
                y = pg2.linear(x0, img, abits, parity=0, wait=False)
                for step in range(1, chain):
                    y = pg2.linear(y, img, abits, parity=step & 1, after=(pg2, (step - 1) & 1), wait=False)
                pg2.wait((chain - 1) & 1, y)
                torch.cuda.synchronize()
                folded = [y.cpu().numpy().copy(), pg2.error()]
                pg2.close()
            out[(M, N, K, abits)] = (got, want, pg.error(), pg.uncached, folded)
            pg.close()
        q.put((rank, out))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_peer_store_gather_matches_all_gather(dev, world):
    """fq_linear_w6ax_gather + fq_gather_wait (the all-gather fused into the decode GEMM epilogue
    through IPC-mapped peer buffers) against ColumnParallelW6Linear's all_gather: every rank's full
    output bit-identical to the collective's, over dependent chains of calls that alternate the two
    gather buffers, at M = 1 (fused quantizer), M = 4 (split-K shard) and M = 16 (separate quantize);
    and the same chains with each wait folded into the next call (fq_linear_w6ax_gather_after: one
    launch per linear where the quantizer is fused, the wait launch first elsewhere) bit-identical
    to the two-launch chain's last output."""
    import torch.multiprocessing as mp
    cases = [(1, 2048, 2048, 6, 6), (4, 512, 8192, 8, 3), (16, 4096, 4096, 6, 4)]
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_peer_worker, args=(r, world, port, cases, q)) for r in range(world)]
    for p_ in procs:
        p_.start()
    res = dict(q.get(timeout=100) for _ in range(world))
    for p_ in procs:
        p_.join(timeout=60)
        assert p_.exitcode == 0
    for (M, N, K, abits, chain) in cases:
        for r in range(world):
            got, want, err, uncached, folded = res[r][(M, N, K, abits)]
            assert err == 0, f"rank {r}: a gather wait timed out"
            assert uncached, f"rank {r}: the gather buffers are not in uncached device memory"
            if folded:  # the folded chain ends where the two-launch chain ends, bit for bit
                assert folded[1] == 0, f"rank {r}: a folded gather wait timed out"
                np.testing.assert_array_equal(folded[0].view(np.uint16), got[-1].view(np.uint16),
                                              err_msg=f"rank {r}: folded chain")
            assert len(got) == chain
            for i, (g, w) in enumerate(zip(got, want)):
                np.testing.assert_array_equal(g.view(np.uint16), w.view(np.uint16), err_msg=f"rank {r} call {i}")
            np.testing.assert_array_equal(got[-1].view(np.uint16), res[0][(M, N, K, abits)][0][-1].view(np.uint16))


def test_gather_wait_times_out_once_then_fails_fast(dev):
    """fq_gather_wait is bounded: with a flag that never arrives it sets the error word after about
    a second and returns (never a hang), and every later wait with the error word set returns at
    once (a broken peer path costs one timeout, not one per linear)."""
    import ctypes
    import time
    from flexq_amd import _lib, ops
    P8, I4 = ctypes.c_uint64 * 8, ctypes.c_int32 * 4

    class Desc(ctypes.Structure):  # fq_gather (include/flexq_hip.h)
        _fields_ = [("out", P8), ("flags", P8), ("done", ctypes.c_uint64), ("gen", ctypes.c_uint64), ("ints", I4)]
    buf = torch.zeros((1, 16), dtype=torch.float16, device=dev)
    flags = torch.zeros(8, dtype=torch.int32, device=dev)  # never raised
    state = torch.tensor([0, 1], dtype=torch.int32, device=dev)  # generation 1 was published by this rank
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    d = Desc()
    d.out[0], d.flags[0] = buf.data_ptr(), flags.data_ptr()
    d.done, d.gen = state.data_ptr(), state.data_ptr() + 4
    d.ints = I4(1, 0, 0, 16)
    desc = torch.frombuffer(bytearray(bytes(d)), dtype=torch.uint8).to(dev)
    s = ops._stream(buf)
    torch.cuda.synchronize()
    t0 = time.time()
    _lib.call("fq_gather_wait", ops._ptr(desc), ops._ptr(err), s)
    torch.cuda.synchronize()
    t1 = time.time()
    assert int(err.item()) == 1 and int(state[1].item()) == 1  # timed out; the wait never moves the generation
    assert 0.05 < t1 - t0 < 30, t1 - t0
    for _ in range(20):
        _lib.call("fq_gather_wait", ops._ptr(desc), ops._ptr(err), s)
    torch.cuda.synchronize()
    assert time.time() - t1 < 0.5 * (t1 - t0) + 0.05, "waits with the error word set must return at once"
