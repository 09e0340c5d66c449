"""GEMM straight from the reference's bit-plane activations (fq_gemm_w6ax_planes): the X / X_SCALE
operands of FQBMMAExecFn_t (engine/src/bgemm/flexq_bmma_op.h:187-188) and of
FLEXQGEMMWrapper::gemm(const int* A ...) (flexq_gemm_wrapper.cu:21-97), which FT's decoder
attention calls with its fused RMSNorm's packed output (LlamaV2DecoderSelfAttentionLayer.cc:653).

At decode sizes the planes are unpacked inside the GEMM's prologue (one launch); elsewhere they are
imported first.  Either way the output must be bit-identical to fq_import_ref_x + fq_gemm_w6ax
and within the oracle's tolerance (oracle.gemm_tolerance: 1e-3 relative + the fp32 floor).  The
planes come from the oracle's restatement of the reference packer (bit_packing.cu:76-133), pinned
by the packing KAT (tests/test_oracle.py).
"""
import numpy as np
import pytest
import torch

from common import assert_gemm_close, kat_operands, oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops(dev):
    from flexq_amd import ops as _ops
    return _ops


def to_dev(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def planes_case(ops, dev, M, N, K, abits, seed, xraw=None):
    kat_xraw, _, _, wq, xs, ws = kat_operands(M, N, K, abits, seed)
    if xraw is None:
        xraw = kat_xraw
    xq = ((xraw ^ (1 << (abits - 1))) - (1 << (abits - 1))).astype(np.int8)
    X = to_dev(oracle.pack_bitplanes(xraw, abits), dev)
    XS = to_dev(oracle.xs_to_ref_dup(xs, M, K), dev)
    pk = ops.pack_w6(to_dev(wq, dev), to_dev(ws, dev))
    d = ops.gemm_w6ax_planes(X, XS, pk, M, N, K, abits)
    xq2, xs2 = ops.import_ref_x(X, XS, M, K, abits)
    d2 = ops.gemm_w6ax(xq2, xs2, pk, N, abits)
    np.testing.assert_array_equal(host(xq2), xq)
    np.testing.assert_array_equal(host(d).view(np.uint16), host(d2).view(np.uint16))
    ref, _, mag = oracle.gemm(xq, xs, wq, ws)
    assert_gemm_close(host(d), ref, mag, f"planes M={M} N={N} K={K} a{abits}")


# decode sizes (fused unpack: M <= 32 where the quantizer would fuse), the split-K decode plan
# (1 x 512 x 8192), the long-K shape whose linear splits (8192 x 28672), batched rows on the
# import path (M = 16, 24, 64) and a prefill size
SHAPES = [(1, 4096, 4096, 6), (1, 12288, 4096, 6), (1, 4096, 11008, 8), (2, 512, 1024, 6), (3, 256, 384, 8),
          (4, 1024, 4096, 6), (5, 96, 512, 6), (7, 200, 640, 8), (8, 4096, 4096, 8), (1, 512, 8192, 8),
          (1, 8192, 28672, 6), (16, 512, 2048, 6), (24, 256, 1024, 8), (32, 256, 1024, 6), (64, 256, 512, 6),
          (2048, 256, 512, 8)]


@pytest.mark.parametrize("M,N,K,abits", SHAPES)
def test_planes_gemm_matches_import_then_gemm(ops, dev, M, N, K, abits):
    planes_case(ops, dev, M, N, K, abits, seed=M * 131 + N + K + abits)


@pytest.mark.parametrize("abits", [6, 8])
@pytest.mark.parametrize("pattern", ["min", "max", "alternate", "zero"])
def test_planes_gemm_extreme_codes(ops, dev, abits, pattern):
    """Sign extension of the top plane: every code at -2^(b-1), at 2^(b-1)-1, alternating, zero."""
    M, N, K = 2, 256, 1024
    lo, hi = 1 << (abits - 1), (1 << (abits - 1)) - 1  # raw patterns of the extremes
    if pattern == "min":
        xraw = np.full((M, K), lo, dtype=np.int32)
    elif pattern == "max":
        xraw = np.full((M, K), hi, dtype=np.int32)
    elif pattern == "alternate":
        xraw = np.where(np.arange(K)[None, :] % 2 == 0, lo, hi).astype(np.int32).repeat(M, 0).reshape(M, K)
    else:
        xraw = np.zeros((M, K), dtype=np.int32)
    planes_case(ops, dev, M, N, K, abits, seed=abits, xraw=xraw)


def test_planes_fuse_at_decode_sizes(ops):
    """The LLaMA decode shapes take the one-launch path (no activation scratch); a linear whose
    quantizer would not fuse imports instead."""
    from flexq_amd import _lib
    L = _lib.load()
    for (N, K) in [(12288, 4096), (4096, 4096), (22016, 4096), (4096, 11008), (28672, 8192), (8192, 8192)]:
        assert L.fq_planes_act_scratch_bytes(1, N, K) == 0, (N, K)
    assert L.fq_planes_act_scratch_bytes(4, 4096, 4096) == 0  # 16 pairs per wave: still one launch
    assert L.fq_planes_act_scratch_bytes(1, 8192, 28672) == 28672 + 2 * (28672 // 128)
    assert L.fq_planes_act_scratch_bytes(8, 4096, 4096) == 8 * 4096 + 2 * 8 * 32
    assert L.fq_planes_act_scratch_bytes(64, 4096, 4096) == 64 * 4096 + 2 * 64 * 32


def test_planes_gemm_in_graph_replay(ops, dev):
    """Captured once, replayed with new plane contents: the fused path reads its operands at run time."""
    M, N, K, abits = 1, 4096, 4096, 6
    xraw0, wraw, xq0, wq, xs, ws = kat_operands(M, N, K, abits, seed=5)
    pk = ops.pack_w6(to_dev(wq, dev), to_dev(ws, dev))
    X = to_dev(oracle.pack_bitplanes(xraw0, abits), dev)
    XS = to_dev(oracle.xs_to_ref_dup(xs, M, K), dev)
    out = torch.empty((M, N), dtype=torch.float16, device=dev)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        ops.gemm_w6ax_planes(X, XS, pk, M, N, K, abits, out=out)  # warm-up (workspace, module load)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            ops.gemm_w6ax_planes(X, XS, pk, M, N, K, abits, out=out)
    for seed in (6, 7):
        xraw = kat_operands(M, N, K, abits, seed=seed)[0]
        X.copy_(to_dev(oracle.pack_bitplanes(xraw, abits), dev))
        g.replay()
        xq = ((xraw ^ (1 << (abits - 1))) - (1 << (abits - 1))).astype(np.int8)
        ref, _, mag = oracle.gemm(xq, xs, wq, ws)
        assert_gemm_close(host(out), ref, mag, f"planes graph replay seed={seed}")
