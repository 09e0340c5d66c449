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
