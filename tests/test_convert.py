"""On-disk packed-weight format (flexq_amd.convert): header round trip,
corruption detection, and the per-rank shard layout of fused linears.  CPU only (no packing)."""
import os

import numpy as np
import pytest
import torch

from flexq_amd import convert


def test_header_round_trip(tmp_path):
    N, K = 48, 256
    nb = convert.packed_bytes(N, K)
    img = torch.from_numpy(np.random.default_rng(0).integers(0, 256, nb, dtype=np.uint8))
    p = str(tmp_path / "x.fqw6")
    convert.save_image(p, img, N, K, 8, N_full=96, row_offset=48, tp_rank=1, tp_size=2)
    back, meta = convert.load_image(p)
    assert torch.equal(back, img)
    assert meta == dict(N=N, K=K, N_full=96, row_offset=48, tp_rank=1, tp_size=2, abits=8,
                        crc32=meta["crc32"], image_bytes=nb)
    assert os.path.getsize(p) == convert.HEADER + nb


def test_corruption_is_detected(tmp_path):
    N, K = 16, 128
    img = torch.zeros(convert.packed_bytes(N, K), dtype=torch.uint8)
    p = str(tmp_path / "y.fqw6")
    convert.save_image(p, img, N, K, 6)
    raw = bytearray(open(p, "rb").read())
    raw[convert.HEADER + 5] ^= 1
    open(p, "wb").write(raw)
    with pytest.raises(ValueError, match="CRC"):
        convert.load_image(p)
    open(p, "wb").write(raw[:-1])
    with pytest.raises(ValueError, match="truncated"):
        convert.load_image(p)
    open(p, "wb").write(b"NOTFQW6!" + bytes(raw[8:]))
    with pytest.raises(ValueError, match="fqw6"):
        convert.load_image(p)
    with pytest.raises(ValueError):
        convert.save_image(p, img[:-1], N, K, 6)


def test_fused_shards_stack_parts_per_rank():
    q = torch.arange(64).view(64, 1).expand(64, 2)
    k = 100 + torch.arange(32).view(32, 1).expand(32, 2)
    r1 = convert.shard_parts([q, k], 2, 1)
    assert r1[:, 0].tolist() == list(range(32, 64)) + list(range(116, 132))
