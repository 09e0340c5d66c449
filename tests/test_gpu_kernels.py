"""GPU parity tests: every HIP kernel through the C ABI against the CPU oracle.

Bit-exact: activation codes + scales, fq6 packing, reference bit planes, imports, the int32
group accumulators.  fp16 outputs: within 1e-3 relative + the fp32-accumulation floor
(oracle.gemm_tolerance).  Shapes cover the reference's edge cases: M in {1,2,4,8} (the wrapper's
buckets, flexq_gemm_wrapper.cu:53-84) and the ragged ones the reference gets wrong (3, 5-7,
M % 8 != 0), N not a multiple of 16, K = 128 (minimum) and K = 11008 (86 groups, odd split),
all-zero groups, tiny/huge groups, and the A8 range.
"""
import numpy as np
import pytest
import torch

from common import assert_gemm_close, kat_operands, model_operands, oracle, rng
from inputs import act_input, edge_inputs

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


# ------------------------------------------------------------------ activation quantizer

@pytest.mark.parametrize("M,K", [(1, 128), (1, 4096), (3, 384), (16, 4096), (17, 11008), (64, 1024), (1000, 256)])
@pytest.mark.parametrize("bits", [6, 8])
def test_quantize_act_bit_exact(ops, dev, M, K, bits):
    x = act_input(M, K, seed=M + K + bits).astype(np.float16)
    xq, xs = ops.quantize_act(to_dev(x, dev), bits)
    q_ref, xs_ref = oracle.quantize_engine(x, bits)
    np.testing.assert_array_equal(host(xq), q_ref)
    np.testing.assert_array_equal(host(xs).view(np.uint16), xs_ref.view(np.uint16))


@pytest.mark.parametrize("bits", [6, 8])
def test_quantize_act_edge_cases(ops, dev, bits):
    for name, arr in edge_inputs().items():
        x = arr.reshape(-1, arr.shape[-1]).astype(np.float16)
        xq, xs = ops.quantize_act(to_dev(x, dev), bits)
        q_ref, xs_ref = oracle.quantize_engine(x, bits)
        np.testing.assert_array_equal(host(xq), q_ref, err_msg=name)
        np.testing.assert_array_equal(host(xs).view(np.uint16), xs_ref.view(np.uint16), err_msg=name)
    # ties at exactly .5: roundf goes away from zero (e2e bit_packing.cu:160)
    x = np.zeros((1, 128), np.float16)
    x[0, 0] = 31.0
    x[0, 1:9] = [0.5, 1.5, 2.5, -0.5, -1.5, -2.5, 30.5, -30.5]  # absmax 31 -> scale exactly 1
    xq, _ = ops.quantize_act(to_dev(x, dev), 6)
    assert list(host(xq)[0, :9]) == [31, 1, 2, 3, -1, -2, -3, 31, -31]
    np.testing.assert_array_equal(host(xq), oracle.quantize_engine(x, 6)[0])


def special_value_input():
    """Rows of 8 groups mixing NaN (alone, beside inf, in every lane position), +-inf, -0, all-
    subnormal groups, fp16 max and ordinary values: the quantizer's integer absmax fast path and its
    NaN fallback (a wave where any group holds a NaN) against the oracle."""
    r = rng(77)
    K = 1024
    x = (r.standard_normal((12, K)) * 2.0).astype(np.float16)
    nan, inf = np.float16(np.nan), np.float16(np.inf)
    x[0, 5] = nan                                       # one NaN, the rest of the row ordinary
    x[1, 128:256:7] = nan                               # many NaNs in one group
    x[2, 300] = inf
    x[3, 400], x[3, 401] = -inf, nan                    # NaN and inf in one group
    x[4, :128] = -0.0
    x[4, 128:256] = 0.0
    x[4, 256:384] = np.ldexp(r.integers(-1023, 1024, 128).astype(np.float64), -24).astype(np.float16)
    x[5, :] = np.float16(65504.0) * np.where(r.random(K) < 0.5, 1, -1).astype(np.float16)
    x[6, 700] = -inf
    x[6, 900] = nan
    x[7, ::128] = nan                                   # a NaN leading every group
    x[8, 127::128] = inf                                # an inf closing every group
    x[9] = np.ldexp(r.integers(-1023, 1024, K).astype(np.float64), -24).astype(np.float16)  # subnormals
    x[10, 0] = np.float16(6.1e-5)                       # smallest normal beside subnormals
    x[10, 1:128] = np.ldexp(r.integers(-1023, 1024, 127).astype(np.float64), -24).astype(np.float16)
    x[11, 640:768] = np.frombuffer(np.uint16(0x7e01).tobytes() * 128, np.float16)  # NaN payloads only
    return x


@pytest.mark.parametrize("bits", [6, 8])
def test_quantize_act_special_values(ops, dev, bits):
    x = special_value_input()
    q_ref, xs_ref = oracle.quantize_engine(x, bits)
    xq, xs = ops.quantize_act(to_dev(x, dev), bits)
    np.testing.assert_array_equal(host(xq), q_ref)
    np.testing.assert_array_equal(host(xs).view(np.uint16), xs_ref.view(np.uint16))
    # NaN-free rows alone (every wave on the fast path) give the same codes as beside the NaN rows
    clean = [i for i in range(x.shape[0]) if not np.isnan(x[i]).any()]
    xq2, xs2 = ops.quantize_act(to_dev(x[clean], dev), bits)
    np.testing.assert_array_equal(host(xq2), q_ref[clean])
    # the fused decode quantizer (M = 1 linear) is the same code: same outputs as the separate
    # quantize + GEMM on the oracle's codes (NaN/inf outputs where a scale is inf, in the same places)
    N = 64
    wq = rng(6).integers(-32, 32, size=(N, x.shape[1])).astype(np.int8)
    ws = (rng(7).random((x.shape[1] // 128, N)) * 0.05).astype(np.float16)
    pk = ops.pack_w6(to_dev(wq, dev), to_dev(ws, dev))
    for i in range(x.shape[0]):
        d = ops.linear_w6ax(to_dev(x[i:i + 1], dev), pk, N, bits)
        d2 = ops.gemm_w6ax(to_dev(q_ref[i:i + 1], dev), to_dev(np.ascontiguousarray(xs_ref[:, i:i + 1]), dev),
                           pk, N, bits)
        np.testing.assert_array_equal(host(d), host(d2), err_msg=f"row {i}")


def tie_heavy_input(M, K, bits, seed):
    """Groups whose scale is exactly a power of two s (absmax = (2^(b-1)-1) s), every other value
    an integer multiple of s/2: about half the quotients are exact .5 ties, the rest exact
    integers -- the cases where a division shortcut could round differently."""
    r = rng(seed)
    hi = (1 << (bits - 1)) - 1
    e = r.integers(-20, 9, size=(M, K // 128, 1))
    s = np.ldexp(1.0, e)
    m = r.integers(-2 * hi, 2 * hi + 1, size=(M, K // 128, 128)).astype(np.float64)
    x = m * s / 2
    x[:, :, 0] = hi * s[:, :, 0] * np.where(r.random((M, K // 128)) < 0.5, 1, -1)
    # plus non-tie values in some groups: odd multiples of s/1024
    noisy = r.random((M, K // 128)) < 0.25
    x[noisy, 1:] += (r.integers(-5, 6, size=(int(noisy.sum()), 127)) * 2 + 1) * s[noisy][:, :1] / 1024
    out = x.reshape(M, K).astype(np.float16)
    return out


@pytest.mark.parametrize("bits", [6, 8])
def test_quantize_act_tie_stress(ops, dev, bits):
    """Quotient-rounding stress: exact ties and exact integers across scales 2^-20 .. 2^8."""
    x = tie_heavy_input(64, 2048, bits, seed=bits)
    xq, xs = ops.quantize_act(to_dev(x, dev), bits)
    q_ref, xs_ref = oracle.quantize_engine(x, bits)
    np.testing.assert_array_equal(host(xs).view(np.uint16), xs_ref.view(np.uint16))
    np.testing.assert_array_equal(host(xq), q_ref)
    # the fused decode quantizer is the same code path: same codes through the GEMM result
    N = 64
    r = rng(5)
    wq = r.integers(-32, 32, size=(N, 2048)).astype(np.int8)
    ws = (r.random((16, N)) * 0.05).astype(np.float16)
    pk = ops.pack_w6(to_dev(wq, dev), to_dev(ws, dev))
    for M in (1, 4, 16):
        d = ops.linear_w6ax(to_dev(x[:M], dev), pk, N, bits)
        d2 = ops.gemm_w6ax(to_dev(q_ref[:M], dev), to_dev(np.ascontiguousarray(xs_ref[:, :M]), dev), pk, N, bits)
        np.testing.assert_array_equal(host(d).view(np.uint16), host(d2).view(np.uint16))


# ------------------------------------------------------------------ packers and importers

@pytest.mark.parametrize("N,K", [(32, 128), (64, 4096), (40, 384), (4096, 256), (17, 128), (8, 256)])
def test_pack_w6_bit_exact(ops, dev, N, K):
    """Weight image (codes + blocked scales) byte-identical to the oracle's, and it round-trips."""
    r = rng(N * 7 + K)
    wq = r.integers(-32, 32, size=(N, K)).astype(np.int8)
    ws = (r.random((K // 128, N)) * 0.05).astype(np.float16)
    pk = ops.pack_w6(to_dev(wq, dev), to_dev(ws, dev))
    np.testing.assert_array_equal(host(pk), oracle.pack_fq6(wq, ws))
    wq2, ws2 = ops.unpack_w6(pk, N, K)
    np.testing.assert_array_equal(host(wq2), wq)
    np.testing.assert_array_equal(host(ws2).view(np.uint16), ws.view(np.uint16))


@pytest.mark.parametrize("N,K", [(32, 128), (96, 1024), (40, 256)])
def test_quantize_pack_w6(ops, dev, N, K):
    w = (rng(N + K).standard_normal((N, K)) * 0.02).astype(np.float16)
    pk, ws, wq = ops.quantize_pack_w6(to_dev(w, dev), return_codes=True)
    wq_ref, ws_ref = oracle.quantize_engine(w, 6)
    np.testing.assert_array_equal(host(wq), wq_ref)
    np.testing.assert_array_equal(host(ws).view(np.uint16), ws_ref.view(np.uint16))
    np.testing.assert_array_equal(host(pk), oracle.pack_fq6(wq_ref, ws_ref))


@pytest.mark.parametrize("R,K,bits", [(1, 128, 6), (4, 512, 8), (8, 256, 6), (24, 384, 6), (16, 128, 8)])
def test_ref_bit_packing_bit_exact(ops, dev, R, K, bits):
    vals = rng(R + K + bits).integers(0, 1 << bits, size=(R, K), dtype=np.int32)
    planes = ops.ref_bit_packing(to_dev(vals, dev), bits)
    np.testing.assert_array_equal(host(planes), oracle.pack_bitplanes(vals, bits))


@pytest.mark.parametrize("M,K,bits", [(1, 4096, 6), (2, 256, 8), (4, 384, 6), (8, 1024, 8), (16, 512, 6)])
def test_ref_quantize_bit_packing(ops, dev, M, K, bits):
    """The drop-in for e2e flexq_bit_packing(const half*...) + FLEXQGEMMWrapper::pack."""
    x = act_input(M, K, seed=3 * M + K).astype(np.float16)
    planes, dup = ops.ref_quantize_bit_packing(to_dev(x, dev), bits)
    q_ref, xs_ref = oracle.quantize_engine(x, bits)
    np.testing.assert_array_equal(host(planes), oracle.pack_bitplanes(q_ref.astype(np.int32), bits))
    np.testing.assert_array_equal(host(dup).view(np.uint16), oracle.xs_to_ref_dup(xs_ref, M, K).view(np.uint16))
    xq2, xs2 = ops.import_ref_x(planes, dup, M, K, bits)
    np.testing.assert_array_equal(host(xq2), q_ref)
    np.testing.assert_array_equal(host(xs2).view(np.uint16), xs_ref.view(np.uint16))


@pytest.mark.parametrize("N,K", [(8, 128), (64, 384), (48, 256)])
def test_import_ref_w(ops, dev, N, K):
    wraw = rng(N + K).integers(0, 64, size=(N, K), dtype=np.int32)
    wq = ((wraw ^ 32) - 32).astype(np.int8)
    ws = (rng(K).random((K // 128, N)) * 0.1).astype(np.float16)
    planes = oracle.pack_bitplanes(wraw, 6)
    pk = ops.import_ref_w(to_dev(planes, dev), to_dev(ws, dev), N, K)
    np.testing.assert_array_equal(host(pk), oracle.pack_fq6(wq, ws))


# ------------------------------------------------------------------ GEMM

def run_gemm(ops, dev, xq, xs, wq, ws, abits):
    N = wq.shape[0]
    pk = ops.pack_w6(to_dev(wq, dev), to_dev(ws, dev))
    args = (to_dev(xq, dev), to_dev(xs, dev), pk, N, abits)
    d, acc = ops.gemm_w6ax(*args, return_acc=True)
    d_prod = ops.gemm_w6ax(*args)  # the production (no debug output) kernel variant
    np.testing.assert_array_equal(host(d).view(np.uint16), host(d_prod).view(np.uint16))
    return host(d), host(acc)


GEMM_KAT = [
    (1, 32, 128, 6), (1, 64, 256, 6), (2, 96, 384, 6), (3, 64, 256, 8), (4, 4096, 4096, 6),
    (5, 40, 256, 6), (8, 64, 11008, 6), (9, 128, 512, 8), (16, 4096, 1024, 8), (17, 100, 384, 6),
    (31, 64, 256, 6), (32, 256, 512, 8), (33, 96, 256, 6), (64, 128, 256, 6), (130, 200, 384, 8),
    (257, 256, 1024, 6), (512, 512, 512, 8),
]


@pytest.mark.parametrize("M,N,K,abits", GEMM_KAT)
def test_gemm_kat(ops, dev, M, N, K, abits):
    """Reference-test-style operands: raw uniform bit patterns, scales U[0, 0.1)."""
    _, _, xq, wq, xs, ws = kat_operands(M, N, K, abits, seed=M * 31 + N * 7 + K)
    d, acc = run_gemm(ops, dev, xq, xs, wq, ws, abits)
    ref, acc_ref, mag = oracle.gemm(xq, xs, wq, ws, want_acc=True)
    np.testing.assert_array_equal(acc, acc_ref)  # int32 group accumulators, bit-exact
    assert_gemm_close(d, ref, mag, f"gemm M={M} N={N} K={K} a{abits}")


@pytest.mark.parametrize("M,N,K,abits", [(1, 4096, 4096, 6), (16, 4096, 11008, 8), (16, 11008, 4096, 6), (256, 1024, 4096, 8),
                                         (48, 4096, 4096, 6), (64, 2048, 4096, 8)])  # (row-chunked decode)
def test_gemm_model_like(ops, dev, M, N, K, abits):
    _, _, xq, wq, xs, ws = model_operands(M, N, K, abits, seed=M + N + K)
    d, acc = run_gemm(ops, dev, xq, xs, wq, ws, abits)
    ref, acc_ref, mag = oracle.gemm(xq, xs, wq, ws, want_acc=True)
    np.testing.assert_array_equal(acc, acc_ref)
    assert_gemm_close(d, ref, mag, f"model-like M={M} N={N} K={K}")


def test_gemm_zero_groups_and_extremes(ops, dev):
    M, N, K = 4, 64, 512
    xq = np.full((M, K), -128, np.int8)
    xq[1, :128] = 0  # an all-zero group
    wq = np.full((N, K), -32, np.int8)
    wq[:, 128:256] = 31
    xs = np.full((K // 128, M), 0.0999, np.float16)
    ws = np.full((K // 128, N), 0.0999, np.float16)
    d, acc = run_gemm(ops, dev, xq, xs, wq, ws, 8)
    ref, acc_ref, mag = oracle.gemm(xq, xs, wq, ws, want_acc=True)
    np.testing.assert_array_equal(acc, acc_ref)
    assert acc.max() == 524288  # 128 * (-128) * (-32): the largest W6A8 group sum
    assert_gemm_close(d, ref, mag, "extremes")


def test_gemm_deterministic(ops, dev):
    _, _, xq, wq, xs, ws = kat_operands(1, 4096, 4096, 6, seed=5)
    pk = ops.pack_w6(to_dev(wq, dev), to_dev(ws, dev))
    a = [host(ops.gemm_w6ax(to_dev(xq, dev), to_dev(xs, dev), pk, 4096, 6)) for _ in range(3)]
    for b in a[1:]:
        np.testing.assert_array_equal(a[0].view(np.uint16), b.view(np.uint16))


@pytest.mark.parametrize("M,N,K,abits", [
    (1, 28672, 8192, 6), (8, 8192, 28672, 6), (16, 24576, 8192, 6),  # LLaMA-2-70B (BASELINE C4)
    # long K / many tiles per CU: the staging variants (activations, then scales, in the ring)
    (16, 8192, 28672, 6), (32, 28672, 8192, 8), (4, 8192, 65536, 6), (12, 16384, 16384, 8), (1, 57344, 8192, 6),
    # 32 < M < 2048 with few 128 x 128 tiles: split-K prefill (fp32 slabs + reduce launch)
    (64, 4096, 11008, 8), (100, 12288, 4096, 6), (33, 4096, 4096, 6),
])
def test_gemm_full_size_sampled_columns(ops, dev, M, N, K, abits):
    """Full sizes: the whole GEMM runs on the GPU, the oracle checks a seeded sample of 96
    columns exactly (accumulators) and within tolerance (outputs)."""
    r = rng(N + K)
    xq = r.integers(-(1 << (abits - 1)), 1 << (abits - 1), size=(M, K)).astype(np.int8)
    wq_dev = torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev,
                           generator=torch.Generator(device=dev).manual_seed(7))
    xs = (r.random((K // 128, M)) * 0.05).astype(np.float16)
    ws = (r.random((K // 128, N)) * 0.05).astype(np.float16)
    pk = ops.pack_w6(wq_dev, to_dev(ws, dev))
    d, acc = ops.gemm_w6ax(to_dev(xq, dev), to_dev(xs, dev), pk, N, abits, return_acc=True)
    cols = np.sort(r.choice(N, size=96, replace=False))
    cols_t = torch.from_numpy(cols).to(dev)
    wq_s = host(wq_dev.index_select(0, cols_t))
    ref, acc_ref, mag = oracle.gemm(xq, xs, wq_s, np.ascontiguousarray(ws[:, cols]), want_acc=True)
    np.testing.assert_array_equal(host(acc.index_select(1, cols_t)), acc_ref)
    assert_gemm_close(host(d)[:, cols], ref, mag, f"full-size M={M} N={N} K={K}")
    # the packed weight round-trips at full size
    assert torch.equal(ops.unpack_w6(pk, N, K)[0], wq_dev)


LINEAR_SHAPES = [
    # (M, N, K, abits): decode sizes run fused (one launch), the rest quantize separately
    (1, 4096, 4096, 6), (1, 12288, 4096, 6), (1, 100, 384, 6), (1, 4096, 11008, 8), (2, 33, 128, 6),
    (3, 512, 1024, 8), (4, 11008, 4096, 6), (5, 64, 256, 6), (8, 1024, 4096, 6), (9, 96, 1280, 8),
    (16, 4096, 4096, 6), (16, 11008, 4096, 6), (16, 4096, 11008, 8), (17, 256, 1024, 6),
    (32, 4096, 4096, 8), (33, 128, 512, 6), (64, 256, 1024, 8),
]


@pytest.mark.parametrize("M,N,K,abits", LINEAR_SHAPES)
def test_linear_matches_quantize_then_gemm(ops, dev, M, N, K, abits):
    """fq_linear_w6ax (FLEXQGEMMWrapper::gemm(const half* A ...)): bit-identical to the two-launch
    quantize + GEMM path, whichever of the two it takes, and within tolerance of the oracle."""
    x, w, xq, wq, xs, ws = model_operands(M, N, K, abits, seed=M * 7 + N + K)
    pk = ops.pack_w6(to_dev(wq, dev), to_dev(ws, dev))
    xd = to_dev(x, dev)
    d = ops.linear_w6ax(xd, pk, N, abits)
    xq_d, xs_d = ops.quantize_act(xd, abits)
    d2 = ops.gemm_w6ax(xq_d, xs_d, pk, N, abits)
    np.testing.assert_array_equal(host(d).view(np.uint16), host(d2).view(np.uint16))
    ref, _, mag = oracle.gemm(xq, xs, wq, ws)
    assert_gemm_close(host(d), ref, mag, f"linear M={M} N={N} K={K}")


def test_linear_fuses_at_decode_sizes(ops):
    """Single-token decode shapes run as one launch (no activation scratch); where the in-kernel
    quantizer's redundancy outweighs a separate quantize launch the linear splits in two."""
    for (N, K) in [(12288, 4096), (4096, 4096), (11008, 4096), (22016, 4096), (4096, 11008),
                   (28672, 8192), (8192, 8192), (10240, 8192)]:
        assert ops.act_scratch_bytes(1, N, K) == 0, (N, K)
    split = lambda M, K: M * K + M * (K // 128) * 2  # noqa: E731
    assert ops.act_scratch_bytes(1, 8192, 28672) == split(1, 28672)  # 28 pairs per wave
    assert ops.act_scratch_bytes(16, 11008, 4096) == split(16, 4096)
    assert ops.act_scratch_bytes(33, 4096, 4096) == split(33, 4096)


def test_linear_edge_inputs(ops, dev):
    """Fused quantizer on the edge groups (zeros, ties, outliers, tiny values)."""
    for name, x in edge_inputs().items():
        x = np.ascontiguousarray(x.reshape(-1, x.shape[-1]).astype(np.float16))
        M, K = x.shape
        if K % 128 or M > 32:
            continue
        N = 96
        r = rng(M + K)
        wq = r.integers(-32, 32, size=(N, K)).astype(np.int8)
        ws = (r.random((K // 128, N)) * 0.05).astype(np.float16)
        pk = ops.pack_w6(to_dev(wq, dev), to_dev(ws, dev))
        for abits in (6, 8):
            d = ops.linear_w6ax(to_dev(x, dev), pk, N, abits)
            xq, xs = oracle.quantize_engine(x, abits)
            ref, _, mag = oracle.gemm(xq, xs, wq, ws)
            assert_gemm_close(host(d), ref, mag, f"linear edge {name} a{abits}")


@pytest.mark.parametrize("M,N,K,abits", [(4, 256, 1024, 6), (1, 512, 8192, 8), (16, 200, 512, 6)])
def test_bmma_state_api_reference_layout(ops, dev, M, N, K, abits):
    """FQBMMAInitFn/ExecFn-style calls (flexq_bmma_op.h:163-188) on the reference's own operands:
    bit-plane X and W plus X_SCALE (duplicated layout) and W_SCALE, into UNinitialised scratch
    (torch.empty; the first exec zeroes its ticket region and imports W).  (1, 512, 8192) plans a
    split-K decode (S > 1), so garbage tickets would show; N = 200 is ragged (bit-plane rows 8k).
    The image fast path (fq_bmma_init_image) gives the same bits, and repeated execs are stable."""
    import ctypes
    from flexq_amd import _lib
    L = _lib.load()
    if M == 1:
        assert L.fq_gemm_workspace_bytes(M, N, K) > 0  # the split-K plan
    xraw, wraw, xq, wq, xs, ws = kat_operands(M, N, K, abits, seed=77 + M)
    X = to_dev(oracle.pack_bitplanes(xraw, abits), dev)
    W = to_dev(oracle.pack_bitplanes(wraw, 6), dev)
    XS = to_dev(oracle.xs_to_ref_dup(xs, M, K), dev)
    WS = to_dev(ws, dev)
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    ref, _, mag = oracle.gemm(xq, xs, wq, ws)
    outs = []
    for image in (False, True):
        D = torch.full((M, N), float("nan"), dtype=torch.float16, device=dev)
        nb = (L.fq_bmma_image_scratch_bytes if image else L.fq_bmma_scratch_bytes)(M, N, K)
        scratch = torch.empty(nb, dtype=torch.uint8, device=dev)
        scratch.fill_(0xA5)  # garbage everywhere, tickets included
        if image:
            img = ops.import_ref_w(W, WS, N, K)
            st = L.fq_bmma_init_image(X.data_ptr(), img.data_ptr(), XS.data_ptr(), M, N, K, D.data_ptr(), 128, 0,
                                      abits, 6, scratch.data_ptr(), nb)
        else:
            st = L.fq_bmma_init(X.data_ptr(), W.data_ptr(), XS.data_ptr(), WS.data_ptr(), M, N, K, D.data_ptr(),
                                128, 0, abits, 6, scratch.data_ptr(), nb)
        assert st.init_success == 1 and st.prepared == 0
        for _ in range(3):
            assert L.fq_bmma_exec(ctypes.byref(st), stream) == 0
            assert st.prepared == 1
            assert_gemm_close(host(D), ref, mag, f"bmma state api image={image}")
            outs.append(host(D).view(np.uint16).copy())
    for o in outs[1:]:
        np.testing.assert_array_equal(o, outs[0])


def test_bmma_init_rejections(ops, dev):
    """The rejections of FQBMMAOp::initialize (flexq_bmma_op.h:103-126) as init_success = 0."""
    from flexq_amd import _lib
    L = _lib.load()
    M, N, K = 4, 256, 1024
    nb = L.fq_bmma_scratch_bytes(M, N, K)
    buf = torch.empty(nb, dtype=torch.uint8, device=dev)
    p = buf.data_ptr()

    def init(**kw):
        a = dict(X=p, W=p, XS=p, WS=p, M=M, N=N, K=K, D=p, g=128, bias=0, xb=6, wb=6, s=p, nb=nb)
        a.update(kw)
        return L.fq_bmma_init(a["X"], a["W"], a["XS"], a["WS"], a["M"], a["N"], a["K"], a["D"], a["g"], a["bias"],
                              a["xb"], a["wb"], a["s"], a["nb"]).init_success
    assert init() == 1
    for kw in (dict(g=64), dict(bias=1), dict(K=1000), dict(xb=4), dict(wb=8), dict(WS=None), dict(W=None),
               dict(M=12), dict(N=20), dict(nb=nb - 1), dict(s=None)):
        assert init(**kw) == 0, kw
    assert L.fq_bmma_image_scratch_bytes(M, N, K) < nb  # no image region on the fast path


def test_split_k_after_prefill_on_shared_workspace(ops, dev):
    """One workspace per stream serves the large-M unpack buffer and the split-K decode tickets:
    a split-K decode launch right after a prefill launch on the same stream is still exact."""
    from flexq_amd import _lib
    L = _lib.load()
    Md, Nd, Kd = 1, 512, 8192  # split-K shape (workspace > 0 at M = 1)
    assert L.fq_gemm_workspace_bytes(Md, Nd, Kd) > 0
    g = torch.Generator(device=dev).manual_seed(3)
    xq = torch.randint(-32, 32, (Md, Kd), dtype=torch.int8, device=dev, generator=g)
    xs = (torch.rand((Kd // 128, Md), device=dev, generator=g) * 0.05).half()
    wq = torch.randint(-32, 32, (Nd, Kd), dtype=torch.int8, device=dev, generator=g)
    ws = (torch.rand((Kd // 128, Nd), device=dev, generator=g) * 0.05).half()
    pk = ops.pack_w6(wq, ws)
    d0 = ops.gemm_w6ax(xq, xs, pk, Nd, 6)
    Mp, Np, Kp = 2048, 2048, 4096  # prefill on the same stream: the unpack buffer is written
    xp = torch.randint(-128, 128, (Mp, Kp), dtype=torch.int8, device=dev, generator=g)
    xsp = (torch.rand((Kp // 128, Mp), device=dev, generator=g) * 0.05).half()
    pkp = ops.pack_w6(torch.randint(-32, 32, (Np, Kp), dtype=torch.int8, device=dev, generator=g),
                      (torch.rand((Kp // 128, Np), device=dev, generator=g) * 0.05).half())
    ops.gemm_w6ax(xp, xsp, pkp, Np, 8)
    for _ in range(3):
        d1 = ops.gemm_w6ax(xq, xs, pk, Nd, 6)
        torch.cuda.synchronize()
        assert torch.equal(d0.view(torch.int16), d1.view(torch.int16))
    ref, _, mag = oracle.gemm(host(xq), host(xs), host(wq), host(ws))
    assert_gemm_close(host(d1), ref, mag, "split-K after prefill")


def test_workspace_growth_keeps_captured_graphs_valid(ops, dev):
    """A graph captured with the stream's workspace bakes its address (split-K tickets + slabs)
    into the launch.  Growing the workspace afterwards (a prefill on the same stream) must not free
    it: the replay stays exact even after the allocator hands out and scribbles over new memory."""
    from flexq_amd import _lib
    L = _lib.load()
    M, N, K = 1, 512, 8192  # split-K decode (tickets + slabs in the workspace)
    assert 0 < L.fq_gemm_workspace_bytes(M, N, K) < L.fq_gemm_workspace_bytes(2048, 2048, 4096)
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn((M, K), dtype=torch.float16, device=dev, generator=g)
    pk = ops.pack_w6(torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g),
                     (torch.rand((K // 128, N), device=dev, generator=g) * 0.05).half())
    s = torch.cuda.Stream(dev)  # a fresh stream: its workspace is created by the first call
    out = torch.empty((M, N), dtype=torch.float16, device=dev)
    with torch.cuda.stream(s):
        ops.linear_w6ax(x, pk, N, 6, out=out)
    torch.cuda.synchronize()
    want = out.clone()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        ops.linear_w6ax(x, pk, N, 6, out=out)
    # grow the stream's workspace: the prefill U8 path wants the unpack buffer
    xp = torch.randint(-128, 128, (2048, 4096), dtype=torch.int8, device=dev, generator=g)
    xsp = (torch.rand((32, 2048), device=dev, generator=g) * 0.05).half()
    pkp = ops.pack_w6(torch.randint(-32, 32, (2048, 4096), dtype=torch.int8, device=dev, generator=g),
                      (torch.rand((32, 2048), device=dev, generator=g) * 0.05).half())
    with torch.cuda.stream(s):
        ops.gemm_w6ax(xp, xsp, pkp, 2048, 8)
    torch.cuda.synchronize()
    junk = [torch.full((1 << 20,), -1, dtype=torch.int32, device=dev) for _ in range(8)]  # reuse freed blocks
    for _ in range(3):
        out.zero_()
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(out.view(torch.int16), want.view(torch.int16))
    del junk


@pytest.mark.parametrize("M,N,K", [(1, 512, 8192), (4, 1024, 28672), (16, 2048, 28672)])
def test_split_k_back_to_back_graph_replay(ops, dev, M, N, K):
    """The cross-workgroup split-K hand-off (write-through slabs, one agent-scope ticket per tile,
    last arriver sums) under back-to-back launches: a graph of 48 launches over 4 inputs and 3
    weight images (tickets reused every launch, consumers on every XCD, uneven arrival), replayed
    4 times; every output bit-identical to its eager launch.  (A mid-stream ticket poll passed a few
    eager calls and hung under exactly this replay pattern)"""
    from flexq_amd import _lib
    assert _lib.load().fq_gemm_workspace_bytes(M, N, K) > 0  # the plan splits K
    g = torch.Generator(device=dev).manual_seed(M + N)
    xs = [torch.randn((M, K), dtype=torch.float16, device=dev, generator=g) for _ in range(4)]
    pks = [ops.pack_w6(torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g),
                       (torch.rand((K // 128, N), device=dev, generator=g) * 0.05).half()) for _ in range(3)]
    R = 48
    pairs = [(i % 4, i % 3) for i in range(R)]
    outs = [torch.empty((M, N), dtype=torch.float16, device=dev) for _ in range(R)]
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        for i, (a, b) in enumerate(pairs):
            ops.linear_w6ax(xs[a], pks[b], N, 6, out=outs[i])
    torch.cuda.synchronize()
    want = [o.clone() for o in outs]
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        for i, (a, b) in enumerate(pairs):
            ops.linear_w6ax(xs[a], pks[b], N, 6, out=outs[i])
    for _ in range(4):
        for o in outs:
            o.fill_(-1)
        graph.replay()
        torch.cuda.synchronize()
        for i in range(R):
            assert torch.equal(outs[i].view(torch.int16), want[i].view(torch.int16)), f"launch {i}"
    # and the eager results agree across inputs that share an (x, W) pair
    for i in range(R):
        j = pairs.index(pairs[i])
        assert torch.equal(want[i].view(torch.int16), want[j].view(torch.int16))


def test_split_k_handoff_under_uneven_load(ops, dev):
    """MI355X_MICROARCH.md "Test every hand-off under UNEVEN load, consumer L1-warm, checking every
    word": the split-K decode hand-off (write-through slabs, agent-scope ticket, last arriver sums
    with sc1 loads) runs while a second stream streams 1 GiB copies beside it, so its workgroups land
    on CUs that are busy to different degrees and arrive unevenly; each launch reuses the tickets and
    slabs of the one before it (the consumer CUs' caches warm with the previous launch's lines).
    Every output word of 3 x 64 launches equals the quiet-GPU result."""
    from flexq_amd import _lib
    L = _lib.load()
    cases = [(1, 512, 8192), (4, 1024, 28672), (16, 2048, 28672)]
    g = torch.Generator(device=dev).manual_seed(17)
    data = []
    for (M, N, K) in cases:
        assert L.fq_gemm_workspace_bytes(M, N, K) > 0  # the plan splits K
        x = torch.randn((M, K), dtype=torch.float16, device=dev, generator=g)
        pk = ops.pack_w6(torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g),
                         (torch.rand((K // 128, N), device=dev, generator=g) * 0.05).half())
        data.append((M, N, K, x, pk))
    main = torch.cuda.Stream(dev)
    with torch.cuda.stream(main):
        want = [ops.linear_w6ax(x, pk, N, 6) for (M, N, K, x, pk) in data]
    torch.cuda.synchronize()
    R = 64
    src = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    side = torch.cuda.Stream(dev)
    outs = [[torch.full((M, N), -1.0, dtype=torch.float16, device=dev) for _ in range(R)] for (M, N, K, x, pk) in data]
    with torch.cuda.stream(side):
        for _ in range(6):
            dst.copy_(src)
    with torch.cuda.stream(main):
        for i in range(R):
            for c, (M, N, K, x, pk) in enumerate(data):
                ops.linear_w6ax(x, pk, N, 6, out=outs[c][i])
    torch.cuda.synchronize()
    for c in range(len(data)):
        for i in range(R):
            assert torch.equal(outs[c][i].view(torch.int16), want[c].view(torch.int16)), f"case {c} launch {i}"
    del src, dst


# (2048, 1000) and (2304, 1004) run the 128 x 128 kernel over the unpacked weights (too few 256 x 256
# tiles to fill the chip), (16384, 1004) and (4096, 4096) the 256 x 256 kernel (ragged N: per-element stores)
@pytest.mark.parametrize("M,N,K", [(2048, 1000, 1280), (2304, 1004, 1280), (16384, 1004, 1280), (4096, 4096, 4096)])
def test_prefill_unpacked_path_bit_identical(ops, dev, M, N, K):
    """Large M with a workspace: the weights are unpacked once (fq_unpack_w8_kernel) and the GEMM
    streams int8 operands (fq_gemm_prefill_kernel<U8>); without a workspace the GEMM unpacks per
    workgroup.  Both paths: identical fp16 outputs and int32 accumulators."""
    import ctypes
    from flexq_amd import _lib
    L = _lib.load()
    assert L.fq_gemm_workspace_bytes(M, N, K) == 256 * 1024 + ((N + 15) // 16) * (K // 128) * 2048
    # below the unpack threshold a workspace holds at most split-K slabs (fp32 [S][M][Npad])
    Mh, npad = min(M // 2 - 1, 2047), (N + 15) // 16 * 16
    wsh = L.fq_gemm_workspace_bytes(Mh, N, K)
    assert wsh == 0 or (wsh - 256 * 1024) % (Mh * npad * 4) == 0
    g = torch.Generator(device=dev).manual_seed(M + N)
    xq = torch.randint(-128, 128, (M, K), dtype=torch.int8, device=dev, generator=g)
    wq = torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g)
    xs = (torch.rand((K // 128, M), device=dev, generator=g) * 0.05).half()
    ws = (torch.rand((K // 128, N), device=dev, generator=g) * 0.05).half()
    pk = ops.pack_w6(wq, ws)
    d1, a1 = ops.gemm_w6ax(xq, xs, pk, N, 8, return_acc=True)  # workspace: the unpacked path
    d2 = torch.empty_like(d1)
    a2 = torch.empty_like(a1)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = L.fq_gemm_w6ax(P(xq), P(xs), P(pk), M, N, K, 8, P(d2), P(a2), None, 0,
                        ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert st == 0
    torch.cuda.synchronize()
    assert torch.equal(a1, a2)
    assert torch.equal(d1.view(torch.int16), d2.view(torch.int16))


@pytest.mark.parametrize("M,N,K", [(2048, 1000, 1280), (16384, 1004, 1280), (4096, 4096, 4096), (1000, 512, 1280),
                                   (32, 4096, 4096)])
def test_prefill_resident_weights_bit_identical(ops, dev, M, N, K):
    """fq_prefill_unpack_weights once + fq_gemm_w6ax_u8 (the caller keeps the int8 operands) against
    fq_gemm_w6ax (unpacking per call in its workspace): identical fp16 outputs and int32
    accumulators; below M = 2048 (and at decode sizes) the _u8 entry is fq_gemm_w6ax itself.  The
    linear wrapper with w_u8 gives the same bits as without."""
    g = torch.Generator(device=dev).manual_seed(M + 3 * N)
    xq = torch.randint(-128, 128, (M, K), dtype=torch.int8, device=dev, generator=g)
    wq = torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g)
    xs = (torch.rand((K // 128, M), device=dev, generator=g) * 0.05).half()
    ws = (torch.rand((K // 128, N), device=dev, generator=g) * 0.05).half()
    pk = ops.pack_w6(wq, ws)
    w_u8 = ops.prepare_prefill_weights(pk, N, K)
    assert w_u8.numel() == ((N + 15) // 16) * (K // 128) * 2048
    d1, a1 = ops.gemm_w6ax(xq, xs, pk, N, 8, return_acc=True)
    d2, a2 = ops.gemm_w6ax(xq, xs, pk, N, 8, return_acc=True, w_u8=w_u8)
    torch.cuda.synchronize()
    assert torch.equal(a1, a2)
    assert torch.equal(d1.view(torch.int16), d2.view(torch.int16))
    x = (torch.randn((M, K), device=dev, generator=g)).half()
    y1 = ops.linear_w6ax(x, pk, N, 8)
    y2 = ops.linear_w6ax(x, pk, N, 8, w_u8=w_u8)
    torch.cuda.synchronize()
    assert torch.equal(y1.view(torch.int16), y2.view(torch.int16))


@pytest.mark.parametrize("M,N,K,qM,qK,qbits", [
    (8192, 6144, 1024, 8192, 4096, 8),     # qkv -> o: the next input a prefix of the output (256 x 256 epilogue)
    (4096, 28672, 1024, 8192, 14336, 8),   # gate_up -> down shape: the next rows straddle the output rows
    (4096, 4096, 1024, 4096, 4096, 6),     # A6 codes
    # ragged M (M % 256 != 0): the epilogue kernel's XSF = false form, partial last row tile
    (2404, 4096, 1024, 2404, 4096, 8),
    (2404, 4096, 1024, 7000, 1280, 6),     # qK != N, the next input ending mid-row of the output
    (2048, 4096, 1024, 2048, 4096, 8),     # 128 x 128 tiles (fill rule): the GEMM, then the quantizer
    (2048, 1000, 1280, 3200, 640, 8),      # N % 128 != 0: the GEMM, then the quantizer
    (32, 4096, 4096, 32, 4096, 8),         # decode sizes: the same
])
def test_prefill_quantized_output_bit_identical(ops, dev, M, N, K, qM, qK, qbits):
    """fq_gemm_w6ax_u8_q: the next linear's codes and scales from the prefill GEMM's epilogue are
    bit-identical to fq_quantize_act over the fp16 output's leading qM x qK values, and the fp16
    output is the plain GEMM's."""
    g = torch.Generator(device=dev).manual_seed(M + 5 * N + qK)
    xq = torch.randint(-128, 128, (M, K), dtype=torch.int8, device=dev, generator=g)
    wq = torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g)
    xs = (torch.rand((K // 128, M), device=dev, generator=g) * 0.05).half()
    ws = (torch.rand((K // 128, N), device=dev, generator=g) * 0.05).half()
    pk = ops.pack_w6(wq, ws)
    w_u8 = ops.prepare_prefill_weights(pk, N, K)
    d0 = ops.gemm_w6ax(xq, xs, pk, N, 8, w_u8=w_u8)
    d1, qxq, qxs = ops.gemm_w6ax_q(xq, xs, pk, N, 8, w_u8, (qM, qK), qbits)
    rq, rs = ops.quantize_act(d1.view(-1)[:qM * qK].view(qM, qK), qbits)
    torch.cuda.synchronize()
    assert torch.equal(d0.view(torch.int16), d1.view(torch.int16))
    assert torch.equal(qxs.view(torch.int16), rs.view(torch.int16))
    assert torch.equal(qxq, rq)


# The round-1 prefill kernel with VGPR-destination asm loads faulted on one shape of this list
# (not recorded which): every shape of that list stays here as the regression set.
@pytest.mark.parametrize("M,N,K,abits,with_acc", [
    (1000, 1000, 1280, 6, True),      # ragged M and N (partial WG tiles on both edges)
    (2048, 2048, 4096, 8, True),
    (16384, 4096, 4096, 8, False),    # LLaMA-3-8B prefill (BASELINE C5) o_proj shape
    # C5's own wide and long shapes at C5's M, accumulators included (acc_dbg is [M, N, K/128]
    # int32: 13-60 GB on the device, written by the debug kernel; the oracle sees the sample)
    pytest.param(16384, 6144, 4096, 8, True, marks=pytest.mark.timeout(300)),    # qkv (GQA)
    pytest.param(16384, 28672, 4096, 8, True, marks=pytest.mark.timeout(300)),   # gate_up merged
    pytest.param(16384, 4096, 14336, 8, True, marks=pytest.mark.timeout(300)),   # down_proj: 112 groups
    # activation codes just past 4 GiB (M x K > 2^32): the host leaves the buffer-addressed 256 x 256
    # kernel (32-bit offsets) for the 128 x 128 one with 64-bit addresses (launch_prefill_u8)
    pytest.param((1 << 20) + 64, 256, 4096, 8, False, marks=pytest.mark.timeout(300)),
])
def test_gemm_prefill_sampled(ops, dev, M, N, K, abits, with_acc):
    """Prefill sizes: the whole GEMM on the GPU, the oracle on a seeded sample of rows x columns."""
    g = torch.Generator(device=dev).manual_seed(M + N + K)
    lo, hi = -(1 << (abits - 1)), 1 << (abits - 1)
    xq_d = torch.randint(lo, hi, (M, K), dtype=torch.int8, device=dev, generator=g)
    wq_d = torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g)
    xs_d = (torch.rand((K // 128, M), device=dev, generator=g) * 0.05).half()
    ws_d = (torch.rand((K // 128, N), device=dev, generator=g) * 0.05).half()
    pk = ops.pack_w6(wq_d, ws_d)
    out = ops.gemm_w6ax(xq_d, xs_d, pk, N, abits, return_acc=with_acc)
    d, acc = out if with_acc else (out, None)
    r = rng(M + K)
    rows = np.sort(np.concatenate([r.choice(M, size=62, replace=False), [0, M - 1]]))
    cols = np.sort(np.concatenate([r.choice(N, size=94, replace=False), [0, N - 1]]))
    rows_t, cols_t = torch.from_numpy(rows).to(dev), torch.from_numpy(cols).to(dev)
    xq, xs = host(xq_d.index_select(0, rows_t)), host(xs_d.index_select(1, rows_t))
    wq, ws = host(wq_d.index_select(0, cols_t)), host(ws_d.index_select(1, cols_t))
    ref, acc_ref, mag = oracle.gemm(np.ascontiguousarray(xq), np.ascontiguousarray(xs), wq,
                                    np.ascontiguousarray(ws), want_acc=True)
    if with_acc:
        np.testing.assert_array_equal(host(acc.index_select(0, rows_t).index_select(1, cols_t)), acc_ref)
    assert_gemm_close(host(d.index_select(0, rows_t).index_select(1, cols_t)), ref, mag,
                      f"prefill M={M} N={N} K={K}")


# C5 (LLaMA-3-8B prefill, M = 16384, W6A8) through the PRODUCTION 256 x 256 kernel (no debug output:
# the fp16 result of the launch the bench times) on every C5 width, against the oracle on a sample
@pytest.mark.timeout(300)
@pytest.mark.parametrize("N,K", [(6144, 4096), (28672, 4096), (4096, 14336)])
def test_c5_production_kernel_sampled(ops, dev, N, K):
    M = 16384
    g = torch.Generator(device=dev).manual_seed(N + K)
    xq_d = torch.randint(-128, 128, (M, K), dtype=torch.int8, device=dev, generator=g)
    wq_d = torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g)
    xs_d = (torch.rand((K // 128, M), device=dev, generator=g) * 0.05).half()
    ws_d = (torch.rand((K // 128, N), device=dev, generator=g) * 0.05).half()
    pk = ops.pack_w6(wq_d, ws_d)
    w_u8 = ops.prepare_prefill_weights(pk, N, K)
    d = ops.gemm_w6ax(xq_d, xs_d, pk, N, 8, w_u8=w_u8)
    r = rng(N + 7 * K)
    rows = np.sort(np.concatenate([r.choice(M, size=62, replace=False), [0, M - 1]]))
    cols = np.sort(np.concatenate([r.choice(N, size=94, replace=False), [0, N - 1]]))
    rows_t, cols_t = torch.from_numpy(rows).to(dev), torch.from_numpy(cols).to(dev)
    ref, _, mag = oracle.gemm(host(xq_d.index_select(0, rows_t)), np.ascontiguousarray(host(xs_d.index_select(1, rows_t))),
                              host(wq_d.index_select(0, cols_t)), np.ascontiguousarray(host(ws_d.index_select(1, cols_t))))
    assert_gemm_close(host(d.index_select(0, rows_t).index_select(1, cols_t)), ref, mag, f"C5 production {N}x{K}")


@pytest.mark.timeout(300)
def test_c5_epilogue_quantized_codes_against_the_oracle(ops, dev):
    """C5's gate_up -> down hand-off as the bench runs it (fq_gemm_w6ax_u8_q: the next linear's A8 codes and
    scales from the 256 x 256 GEMM's epilogue; the next input [16384, 14336] is the output's leading
    values, rows straddling output rows): sampled rows of the codes and scales bit-exact against the
    oracle's engine quantizer applied to the GEMM's own fp16 output, and that output within the oracle's
    GEMM tolerance."""
    M, N, K, qM, qK = 16384, 28672, 4096, 16384, 14336
    g = torch.Generator(device=dev).manual_seed(31)
    xq = torch.randint(-128, 128, (M, K), dtype=torch.int8, device=dev, generator=g)
    wq = torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g)
    xs = (torch.rand((K // 128, M), device=dev, generator=g) * 0.05).half()
    ws = (torch.rand((K // 128, N), device=dev, generator=g) * 0.05).half()
    pk = ops.pack_w6(wq, ws)
    w_u8 = ops.prepare_prefill_weights(pk, N, K)
    d, qxq, qxs = ops.gemm_w6ax_q(xq, xs, pk, N, 8, w_u8, (qM, qK), 8)
    torch.cuda.synchronize()
    r = rng(11)
    qrows = np.sort(np.concatenate([r.choice(qM, size=30, replace=False), [0, qM - 1]]))
    qr_t = torch.from_numpy(qrows).to(dev)
    x_next = d.view(-1)[:qM * qK].view(qM, qK).index_select(0, qr_t)
    q_ref, s_ref = oracle.quantize_engine(host(x_next), 8)
    np.testing.assert_array_equal(host(qxq.index_select(0, qr_t)), q_ref)
    np.testing.assert_array_equal(host(qxs.index_select(1, qr_t)).view(np.uint16), s_ref.view(np.uint16))
    rows = np.sort(np.concatenate([r.choice(M, size=30, replace=False), [0, M - 1]]))
    cols = np.sort(np.concatenate([r.choice(N, size=62, replace=False), [0, N - 1]]))
    rows_t, cols_t = torch.from_numpy(rows).to(dev), torch.from_numpy(cols).to(dev)
    ref, _, mag = oracle.gemm(host(xq.index_select(0, rows_t)), np.ascontiguousarray(host(xs.index_select(1, rows_t))),
                              host(wq.index_select(0, cols_t)), np.ascontiguousarray(host(ws.index_select(1, cols_t))))
    assert_gemm_close(host(d.index_select(0, rows_t).index_select(1, cols_t)), ref, mag, "C5 gate_up (epilogue form)")


# M = 1 decode linears of the headline workload (every plan S = 1): the fused one-launch output bit for
# bit against the oracle's restatement of the decode kernel's summation order
@pytest.mark.parametrize("N,K", [(12288, 4096), (4096, 4096), (22016, 4096), (4096, 11008)])
def test_decode_linear_bit_exact_decode_order(ops, dev, N, K):
    g = torch.Generator(device=dev).manual_seed(N ^ K)
    x = torch.randn((1, K), dtype=torch.float16, device=dev, generator=g)
    wq = torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g)
    ws = ((torch.rand((K // 128, N), device=dev, generator=g) + 0.5) / (18.5 * K ** 0.5)).half()
    pk = ops.pack_w6(wq, ws)
    y = ops.linear_w6ax(x, pk, N, 6)
    torch.cuda.synchronize()
    q, s = oracle.quantize_engine(host(x), 6)
    exact = oracle.gemm_decode_order(q, s, host(wq), host(ws), nw=8)
    np.testing.assert_array_equal(host(y).view(np.uint16), exact.view(np.uint16))


@pytest.mark.timeout(300)
def test_quantize_act_past_4g_elements(ops, dev):
    """fq_quantize_act over M x K > 2^32 elements (its 64-bit index form): sampled rows bit-exact
    against the oracle, the rows on both sides of element 2^32 included."""
    M, K = (1 << 20) + 64, 4096
    g = torch.Generator(device=dev).manual_seed(7)
    x = torch.randn((M, K), device=dev, dtype=torch.float16, generator=g)
    xq, xs = ops.quantize_act(x, 8)
    edge = (1 << 32) // K
    rows = torch.tensor([0, 1, edge - 1, edge, edge + 1, M - 2, M - 1], device=dev)
    q_ref, s_ref = oracle.quantize_engine(host(x.index_select(0, rows)), 8)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(host(xq.index_select(0, rows)), q_ref)
    np.testing.assert_array_equal(host(xs.index_select(1, rows)).view(np.uint16), s_ref.view(np.uint16))
    del x, xq, xs


def test_workspace_growth_is_geometric(ops, dev):
    """rising M values (split-K slabs grow with M) must not leave a superseded buffer per
    new maximum: growth is x1.5 and a buffer no graph capture has seen is released."""
    from flexq_amd import _lib
    L = _lib.load()
    N, K = 4096, 4096
    s = torch.cuda.Stream(dev)
    g = torch.Generator(device=dev).manual_seed(9)
    pk = ops.pack_w6(torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g),
                     (torch.rand((K // 128, N), device=dev, generator=g) * 0.05).half())
    before = ops.workspace_device_bytes()
    needs = []
    with torch.cuda.stream(s):
        for M in range(33, 1024, 29):
            needs.append(L.fq_gemm_workspace_bytes(M, N, K))
            x = torch.randn((M, K), dtype=torch.float16, device=dev, generator=g)
            ops.linear_w6ax(x, pk, N, 6)
    torch.cuda.synchronize()
    held = ops.workspace_device_bytes() - before
    assert max(needs) > 0
    assert held <= 2 * max(max(needs), 1 << 20), (held, max(needs))


def test_prefill_split_k_without_workspace_is_an_error(ops, dev):
    """a split-K prefill shape without its slabs returns FQ_ERR_WORKSPACE (as the split-K
    decode does) instead of silently running S = 1, whose fp16 bits differ."""
    import ctypes
    from flexq_amd import _lib
    L = _lib.load()
    M, N, K = 200, 4096, 4096
    assert L.fq_gemm_workspace_bytes(M, N, K) > 256 * 1024  # the plan splits K
    xq = torch.zeros((M, K), dtype=torch.int8, device=dev)
    xs = torch.zeros((K // 128, M), dtype=torch.float16, device=dev)
    pk = torch.zeros(ops.packed_w_bytes(N, K), dtype=torch.uint8, device=dev)
    d = torch.empty((M, N), dtype=torch.float16, device=dev)
    P = ctypes.c_void_p
    rc = L.fq_gemm_w6ax(P(xq.data_ptr()), P(xs.data_ptr()), P(pk.data_ptr()), M, N, K, 8, P(d.data_ptr()), None,
                        None, 0, None)
    assert rc == 4  # FQ_ERR_WORKSPACE


# fq_gemm_w6ax_q at decode sizes: the next linear's codes from the decode GEMM's epilogue (group tickets,
# the last workgroup of each 128-column group quantizes it).  C3's four hand-offs (down's A8 input a prefix
# whose rows straddle gate_up's), M = 1 / 4 / 8 / ragged 13, and two shapes that take the two-launch form
# (N % 128 != 0; a k-split plan).
@pytest.mark.parametrize("M,N,K,qM,qK,qbits", [
    (16, 12288, 4096, 16, 4096, 6),    # qkv -> o: the output's leading third
    (16, 4096, 4096, 16, 4096, 6),     # o -> gate_up
    (16, 22016, 4096, 16, 11008, 8),   # gate_up -> down (A8)
    (16, 4096, 11008, 16, 4096, 6),    # down -> the next layer's qkv
    (1, 12288, 4096, 1, 4096, 6),
    (4, 4096, 4096, 4, 4096, 8),
    (8, 4224, 4096, 8, 4224, 6),       # 33 groups, 264 tiles: two items on 8 workgroups
    (13, 4096, 4096, 13, 4096, 6),     # ragged rows in the 16-row tile
    (16, 4112, 4096, 16, 4096, 6),     # N % 128 != 0: the GEMM, then the quantizer
    (16, 1024, 4096, 16, 1024, 6),     # narrow N: a k-split plan, the two-launch form
])
def test_decode_quantized_output_bit_identical(ops, dev, M, N, K, qM, qK, qbits):
    """fq_gemm_w6ax_q: codes and scales bit-identical to fq_quantize_act over the fp16 output's leading
    qM x qK values, the output the plain GEMM's, and the same again on a second call and on graph
    replays (the group tickets return to zero after every launch)."""
    g = torch.Generator(device=dev).manual_seed(M * 7 + N + qK)
    xq = torch.randint(-32, 32, (M, K), dtype=torch.int8, device=dev, generator=g)
    wq = torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g)
    xs = (torch.rand((K // 128, M), device=dev, generator=g) * 0.05).half()
    ws = (torch.rand((K // 128, N), device=dev, generator=g) * 0.05).half()
    pk = ops.pack_w6(wq, ws)
    d0 = ops.gemm_w6ax(xq, xs, pk, N, 6)
    rq, rs = ops.quantize_act(d0.view(-1)[:qM * qK].view(qM, qK), qbits)
    for _ in range(2):
        d1, qxq, qxs = ops.gemm_w6ax_q(xq, xs, pk, N, 6, None, (qM, qK), qbits)
        torch.cuda.synchronize()
        assert torch.equal(d0.view(torch.int16), d1.view(torch.int16))
        assert torch.equal(qxs.view(torch.int16), rs.view(torch.int16))
        assert torch.equal(qxq, rq)
    s = torch.cuda.Stream(dev)
    d2 = torch.empty_like(d0)
    with torch.cuda.stream(s):
        ops.gemm_w6ax_q(xq, xs, pk, N, 6, None, (qM, qK), qbits, out=d2)  # (sizes the stream's workspace)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        _, gq, gs = ops.gemm_w6ax_q(xq, xs, pk, N, 6, None, (qM, qK), qbits, out=d2)
    for _ in range(3):
        gq.zero_()
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(gq, rq) and torch.equal(gs.view(torch.int16), rs.view(torch.int16))


def test_c3_epilogue_quantized_codes_against_the_oracle(ops, dev):
    """C3's gate_up -> down hand-off in the decode epilogue form (M = 16, the next input [16, 11008] A8 is
    the output's leading values, its rows straddling gate_up's): the codes and scales bit-exact against
    the oracle's engine quantizer applied to the GEMM's own fp16 output, and that output within the
    oracle's GEMM tolerance."""
    M, N, K, qM, qK = 16, 22016, 4096, 16, 11008
    g = torch.Generator(device=dev).manual_seed(37)
    xq = torch.randint(-32, 32, (M, K), dtype=torch.int8, device=dev, generator=g)
    wq = torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g)
    xs = (torch.rand((K // 128, M), device=dev, generator=g) * 0.05).half()
    ws = (torch.rand((K // 128, N), device=dev, generator=g) * 0.05).half()
    pk = ops.pack_w6(wq, ws)
    d, qxq, qxs = ops.gemm_w6ax_q(xq, xs, pk, N, 6, None, (qM, qK), 8)
    torch.cuda.synchronize()
    q_ref, s_ref = oracle.quantize_engine(host(d.view(-1)[:qM * qK].view(qM, qK)), 8)
    np.testing.assert_array_equal(host(qxq), q_ref)
    np.testing.assert_array_equal(host(qxs).view(np.uint16), s_ref.view(np.uint16))
    r = rng(13)
    cols = np.sort(np.concatenate([r.choice(N, size=126, replace=False), [0, N - 1]]))
    cols_t = torch.from_numpy(cols).to(dev)
    ref, _, mag = oracle.gemm(host(xq), np.ascontiguousarray(host(xs)), host(wq.index_select(0, cols_t)),
                              np.ascontiguousarray(host(ws.index_select(1, cols_t))))
    assert_gemm_close(host(d.index_select(1, cols_t)), ref, mag, "C3 gate_up (epilogue form)")
