"""GPU parity across the M dispatch boundaries (README "Which kernel runs"): every GEMM path --
decode (fused and split), the decode kernel in row chunks, the 128 x 128 prefill kernel with and
without split-K, the 128 x 128 and 256 x 256 kernels over once-unpacked weights -- on shapes on
both sides of each threshold, ragged M and N included.  The whole GEMM runs on the GPU; the
oracle checks a seeded sample of rows x columns: int32 group accumulators bit-exact, fp16
outputs within oracle.gemm_tolerance.  The fused linear (quantize inside) is checked against the
quantize-then-GEMM path bit-exactly where it applies."""
import numpy as np
import pytest
import torch

from common import assert_gemm_close, oracle, rng

pytestmark = pytest.mark.gpu

# (M, N, K, abits): boundaries 32/33 (decode -> chunks/prefill), 64/65 (chunks -> prefill),
# few-tile split-K, 2047/2048 (per-WG unpack -> unpacked weights), tile selection at M >= 2048
CASES = [
    (1, 4096, 4096, 6), (31, 1000, 1280, 6), (32, 4096, 4096, 8), (33, 4096, 4096, 6), (33, 4104, 2048, 8),
    (64, 4096, 4096, 6), (65, 4096, 4096, 8), (64, 12288, 4096, 6), (96, 1000, 4096, 6), (127, 4096, 11008, 8),
    # the 64-row decode tile (33 <= M <= 64): activation rows per ring slot, x-scales staged or per slot,
    # several tiles per workgroup, ragged M
    (48, 22016, 4096, 6), (64, 4096, 11008, 8), (40, 1000, 1280, 8), (57, 4104, 14336, 6),
    (200, 2048, 1280, 6), (257, 768, 2048, 8), (511, 4096, 4096, 6), (1023, 1004, 1280, 8), (2047, 512, 1024, 6),
    (2048, 4096, 1024, 8), (2049, 1000, 1280, 6), (3072, 6144, 512, 8), (4096, 28672, 256, 6),
]


@pytest.fixture(scope="module")
def ops(dev):
    from flexq_amd import ops as _ops
    return _ops


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


@pytest.mark.parametrize("M,N,K,abits", CASES)
def test_gemm_across_dispatch_boundaries(ops, dev, M, N, K, abits):
    g = torch.Generator(device=dev).manual_seed(M * 7 + N + K)
    lo, hi = -(1 << (abits - 1)), 1 << (abits - 1)
    xq_d = torch.randint(lo, hi, (M, K), dtype=torch.int8, device=dev, generator=g)
    wq_d = torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g)
    xs_d = (torch.rand((K // 128, M), device=dev, generator=g) * 0.05).half()
    ws_d = (torch.rand((K // 128, N), device=dev, generator=g) * 0.05).half()
    pk = ops.pack_w6(wq_d, ws_d)
    d, acc = ops.gemm_w6ax(xq_d, xs_d, pk, N, abits, return_acc=True)
    d_prod = ops.gemm_w6ax(xq_d, xs_d, pk, N, abits)  # the production (no debug output) variant
    assert torch.equal(d.view(torch.int16), d_prod.view(torch.int16))
    r = rng(M + N + K)
    rows = np.unique(np.concatenate([r.choice(M, size=min(M, 24), replace=False), [0, M - 1]]))
    cols = np.unique(np.concatenate([r.choice(N, size=min(N, 48), replace=False), [0, N - 1]]))
    rows_t, cols_t = torch.from_numpy(rows).to(dev), torch.from_numpy(cols).to(dev)
    xq, xs = host(xq_d.index_select(0, rows_t)), host(xs_d.index_select(1, rows_t))
    wq, ws = host(wq_d.index_select(0, cols_t)), host(ws_d.index_select(1, cols_t))
    ref, acc_ref, mag = oracle.gemm(np.ascontiguousarray(xq), np.ascontiguousarray(xs), wq,
                                    np.ascontiguousarray(ws), want_acc=True)
    np.testing.assert_array_equal(host(acc.index_select(0, rows_t).index_select(1, cols_t)), acc_ref)
    assert_gemm_close(host(d.index_select(0, rows_t).index_select(1, cols_t)), ref, mag,
                      f"dispatch M={M} N={N} K={K} a{abits}")


@pytest.mark.parametrize("M,N,K", [(1, 4096, 4096), (32, 1000, 1280), (33, 4096, 2048), (64, 4096, 4096), (300, 2048, 1024)])
def test_linear_equals_quantize_then_gemm_across_boundaries(ops, dev, M, N, K):
    g = torch.Generator(device=dev).manual_seed(M + N + K)
    x = torch.randn((M, K), dtype=torch.float16, device=dev, generator=g)
    wq = torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g)
    pk = ops.pack_w6(wq, (torch.rand((K // 128, N), device=dev, generator=g) * 0.05).half())
    y = ops.linear_w6ax(x, pk, N, 6)
    xq, xs = ops.quantize_act(x, 6)
    y2 = ops.gemm_w6ax(xq, xs, pk, N, 6)
    assert torch.equal(y.view(torch.int16), y2.view(torch.int16))
