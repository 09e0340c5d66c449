"""100 seeded random shapes across every GEMM path (a fuzz complement to the curated dispatch sweep):
M from 1 to 3000 (weighted towards decode sizes), N any multiple of 16 up to 30000, K any multiple of
128 up to 16384, A6 or A8.  Per shape the whole GEMM runs on the GPU and the oracle checks a seeded
sample of rows x columns -- int32 group accumulators bit-exact, fp16 outputs within
oracle.gemm_tolerance; the production (no debug output) variant equals the debug one bit for bit; the
one-launch linear equals quantize-then-GEMM; and the next-input form (fq_gemm_w6ax_q) gives
fq_quantize_act's codes of the output.  The shape list is fixed by the seed, so a failure names a
reproducible case."""
import numpy as np
import pytest
import torch

from common import assert_gemm_close, oracle, rng

pytestmark = pytest.mark.gpu


def _shapes(n=100, seed=2026):
    r = np.random.default_rng(seed)
    out = []
    while len(out) < n:
        M = int(r.choice([r.integers(1, 5), r.integers(5, 33), r.integers(33, 129), r.integers(129, 3001)],
                         p=[0.3, 0.3, 0.2, 0.2]))
        N = 16 * int(r.integers(1, 1876))
        K = 128 * int(r.integers(1, 129))
        ab = int(r.choice([6, 8]))
        if M * N * (K // 128) > (1 << 26) or M * K > (1 << 24):  # (the debug accumulators stay <= 256 MB)
            continue
        out.append((M, N, K, ab))
    return out


SHAPES = _shapes()


@pytest.fixture(scope="module")
def ops(dev):
    from flexq_amd import ops as _ops
    return _ops


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


@pytest.mark.parametrize("M,N,K,abits", SHAPES)
def test_random_shape_against_the_oracle(ops, dev, M, N, K, abits):
    g = torch.Generator(device=dev).manual_seed(M * 131 + N * 7 + K + abits)
    lo, hi = -(1 << (abits - 1)), 1 << (abits - 1)
    xq_d = torch.randint(lo, hi, (M, K), dtype=torch.int8, device=dev, generator=g)
    wq_d = torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g)
    xs_d = (torch.rand((K // 128, M), device=dev, generator=g) * 0.05).half()
    ws_d = (torch.rand((K // 128, N), device=dev, generator=g) * 0.05).half()
    pk = ops.pack_w6(wq_d, ws_d)
    d, acc = ops.gemm_w6ax(xq_d, xs_d, pk, N, abits, return_acc=True)
    d_prod = ops.gemm_w6ax(xq_d, xs_d, pk, N, abits)
    assert torch.equal(d.view(torch.int16), d_prod.view(torch.int16))
    r = rng(M * 3 + N + K)
    rows = np.unique(np.concatenate([r.choice(M, size=min(M, 12), replace=False), [0, M - 1]]))
    cols = np.unique(np.concatenate([r.choice(N, size=min(N, 40), replace=False), [0, N - 1]]))
    rows_t, cols_t = torch.from_numpy(rows).to(dev), torch.from_numpy(cols).to(dev)
    xq, xs = host(xq_d.index_select(0, rows_t)), host(xs_d.index_select(1, rows_t))
    wq, ws = host(wq_d.index_select(0, cols_t)), host(ws_d.index_select(1, cols_t))
    ref, acc_ref, mag = oracle.gemm(np.ascontiguousarray(xq), np.ascontiguousarray(xs), wq,
                                    np.ascontiguousarray(ws), want_acc=True)
    np.testing.assert_array_equal(host(acc.index_select(0, rows_t).index_select(1, cols_t)), acc_ref)
    assert_gemm_close(host(d.index_select(0, rows_t).index_select(1, cols_t)), ref, mag,
                      f"fuzz M={M} N={N} K={K} a{abits}")
    del acc
    # the next-input form: fq_quantize_act's codes of the output's leading rows (a [qM, qK] prefix)
    qK = 128 * max(1, min(N, 4096) // 128)
    qM = max(1, min(M * N // qK, 64))
    if qM * qK > M * N:
        return
    _, qxq, qxs = ops.gemm_w6ax_q(xq_d, xs_d, pk, N, abits, None, (qM, qK), 8)
    rq, rs = ops.quantize_act(d_prod.view(-1)[:qM * qK].view(qM, qK), 8)
    assert torch.equal(qxq, rq) and torch.equal(qxs.view(torch.int16), rs.view(torch.int16))


@pytest.mark.parametrize("M,N,K,abits", [s for s in SHAPES if s[0] <= 300][:32])
def test_random_shape_linear_equals_quantize_then_gemm(ops, dev, M, N, K, abits):
    g = torch.Generator(device=dev).manual_seed(M + 3 * N + K)
    x = torch.randn((M, K), dtype=torch.float16, device=dev, generator=g)
    wq = torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g)
    pk = ops.pack_w6(wq, (torch.rand((K // 128, N), device=dev, generator=g) * 0.05).half())
    y = ops.linear_w6ax(x, pk, N, abits)
    xq, xs = ops.quantize_act(x, abits)
    y2 = ops.gemm_w6ax(xq, xs, pk, N, abits)
    assert torch.equal(y.view(torch.int16), y2.view(torch.int16))
