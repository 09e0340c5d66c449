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
                        crc32=meta["crc32"], image_bytes=nb, k_offset=0, split=convert.COLUMN)
    convert.save_image(p, img, N, K, 6, N_full=N, tp_rank=1, tp_size=3, k_offset=384, split=convert.ROW)
    meta = convert.read_header(p)
    assert (meta["k_offset"], meta["split"], meta["row_offset"]) == (384, convert.ROW, 0)
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


def test_row_parallel_columns_and_matching_gate_rows():
    """down_proj columns and gate/up rows use the same 128-group split, so rank p's SiLU*up
    output is exactly down_proj's rank-local input."""
    F, H, P = 640, 32, 2
    down = torch.arange(H * F).view(H, F)
    gate = torch.arange(F).view(F, 1).expand(F, 4)
    for r in range(P):
        cols, k_off = convert.shard_columns(down, P, r)
        rows = convert.shard_parts([gate, gate], P, r, by_group=True)
        assert rows.shape[0] == 2 * cols.shape[1]
        assert rows[:cols.shape[1], 0].tolist() == list(range(k_off, k_off + cols.shape[1]))
        assert torch.equal(cols, down[:, k_off:k_off + cols.shape[1]])


def test_uneven_group_shards_have_cumulative_row_offsets():
    """LLaMA-2-7B gate/up at TP 4: 11008 = 86 groups -> 22/22/21/21 groups per rank.  Each rank's
    stacked [gate_p; up_p] file starts where the lower ranks' files end."""
    F, P = 11008, 4
    gate = torch.arange(F).view(F, 1)
    up = F + torch.arange(F).view(F, 1)
    offs, sizes = [], []
    for r in range(P):
        rows, off = convert.shard_parts([gate, up], P, r, by_group=True, return_offset=True)
        offs.append(off)
        sizes.append(rows.shape[0])
    assert sizes == [2 * 22 * 128, 2 * 22 * 128, 2 * 21 * 128, 2 * 21 * 128]
    assert offs == [0, sizes[0], sizes[0] + sizes[1], sizes[0] + sizes[1] + sizes[2]]
    assert sum(sizes) == 2 * F
