"""bench.py's decoder-layer section at tp = 2: two real processes share the
box's GPU (gloo carries the all-reduces, as in bench.py --share-gpu; RCCL on a node runs the same code),
each calls bench.decoder_layers_e2e, and the section must come back numeric on both ranks -- including
the "no all-reduce" timing, whose run_layers(reduce=False) form the tp > 1 guard rejects."""
import os
import socket
import sys
import types

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, q):
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import bench
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        a = types.SimpleNamespace(no_graph=True)
        ctx = bench.Ctx(a, rank, world, dev, staged=True)
        res = {}
        bench.optional(res, "decoder_layers_e2e", lambda: {"tp": world, "M1": bench.decoder_layers_e2e(ctx, 1, layers=2)},
                       ctx)
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_decoder_layers_section_at_tp2():
    import torch.multiprocessing as mp
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p_ in procs:
        p_.start()
    res = dict(q.get(timeout=110) for _ in range(2))
    for p_ in procs:
        p_.join(timeout=60)
        assert p_.exitcode == 0
    for r in range(2):
        sec = res[r]["decoder_layers_e2e"]
        assert "error" not in sec, sec
        m1 = sec["M1"]
        for k in ("w6_ms_per_step", "fp16_ms_per_step", "w6_no_allreduce_ms_per_step", "allreduce_share"):
            assert isinstance(m1[k], float) and m1[k] >= 0.0, (k, m1)
