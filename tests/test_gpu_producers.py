"""GPU parity tests of the fused activation producers through the C ABI.

fq_rmsnorm_quantize (layernorm_kernels.cu:1851-2051): residual, normalised fp16 values, codes
and scales bit-exact against oracle.rmsnorm_quantize, which restates the kernel's arithmetic
order (IEEE add/mul/div/sqrt, a fixed reduction tree).

Against the REFERENCE's formula (not this build's order): the reference normalises with CUDA's
rsqrtf (layernorm_kernels.cu:1816, 1893), an approximation defined only to 2 ulp, so its bits are
not a target; its fp16 output is within one fp16 ulp of the float64 evaluation of
half(half(x + in) * rsqrt(mean(x^2) + eps) * gamma), and so is this kernel's
(test_rmsnorm_within_one_ulp_of_reference_formula): the two agree to one fp16 ulp per element.

fq_silu_mul_quantize (activation_kernels.cu:245-450): the fp16 product within one fp16 ulp of
the double-precision oracle (the kernel uses fp32 and the hardware's fast exp, as the reference
uses __expf); codes and scales bit-exact against the engine quantizer applied to the kernel's own
fp16 product, i.e. the quantization step is exact.
"""
import numpy as np
import pytest
import torch

from common import oracle, rng

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops(dev):
    from flexq_amd import ops as _ops
    return _ops


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def to_dev(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def hbits(a):
    return np.ascontiguousarray(a).view(np.uint16)


@pytest.mark.parametrize("M,K", [(1, 4096), (3, 4096), (16, 11008), (5, 128), (2, 32768), (64, 8192), (7, 384),
                                 (2048, 4096)])
@pytest.mark.parametrize("bits", [6, 8])
@pytest.mark.parametrize("with_input", [True, False])
def test_rmsnorm_quantize_bit_exact(ops, dev, M, K, bits, with_input):
    r = rng(M * 131 + K + bits + with_input)
    res = (r.standard_normal((M, K)) * 2.0).astype(np.float16)
    inp = (r.standard_normal((M, K)) * 0.5).astype(np.float16) if with_input else None
    gamma = (1.0 + 0.2 * r.standard_normal(K)).astype(np.float16)
    res[0, :7] = [0.0, -0.0, 6e-8, -3e4, 3e4, 1e-3, 65504.0]  # zeros, subnormal, clamp range
    eps = 1e-5
    res_d = to_dev(res, dev)
    xq, xs, normed = ops.rmsnorm_quantize(res_d, to_dev(gamma, dev), bits, eps=eps,
                                          input=None if inp is None else to_dev(inp, dev), return_normed=True)
    r_ref, n_ref, q_ref, xs_ref = oracle.rmsnorm_quantize(inp, res, gamma, eps, bits)
    np.testing.assert_array_equal(hbits(host(res_d)), hbits(r_ref), err_msg="residual")
    np.testing.assert_array_equal(hbits(host(normed)), hbits(n_ref), err_msg="normed")
    np.testing.assert_array_equal(host(xq), q_ref, err_msg="codes")
    np.testing.assert_array_equal(hbits(host(xs)), hbits(xs_ref), err_msg="scales")


def test_rmsnorm_zero_and_huge_rows(ops, dev):
    """An all-zero row (scale 0 -> codes 0, the reference's NaN path defined) and a row of
    near-fp16-max values."""
    K = 1024
    res = np.zeros((2, K), np.float16)
    res[1] = 6.0e4
    gamma = np.ones(K, np.float16)
    xq, xs, normed = ops.rmsnorm_quantize(to_dev(res, dev), to_dev(gamma, dev), 6, return_normed=True)
    _, n_ref, q_ref, xs_ref = oracle.rmsnorm_quantize(None, res, gamma, 1e-6, 6)
    np.testing.assert_array_equal(hbits(host(normed)), hbits(n_ref))
    np.testing.assert_array_equal(host(xq), q_ref)
    np.testing.assert_array_equal(hbits(host(xs)), hbits(xs_ref))
    assert not host(xq)[0].any()


def within_one_ulp(got, ref):
    g = got.astype(np.float64)
    f = ref.astype(np.float64)
    ulp = np.spacing(np.abs(ref).astype(np.float16)).astype(np.float64)
    return np.abs(g - f) <= ulp


@pytest.mark.parametrize("M,N", [(1, 11008), (16, 11008), (3, 128), (64, 14336), (5, 640), (2048, 14336)])
@pytest.mark.parametrize("bits", [8, 6])
def test_silu_mul_quantize(ops, dev, M, N, bits):
    """gate and up as the two column halves of one merged gate_up output [M, 2N] (the layout of
    bench.py's merged gate/up linear), row stride 2N."""
    r = rng(M * 7 + N + bits)
    gu = (r.standard_normal((M, 2 * N)) * 3.0).astype(np.float16)
    gu[0, :4] = [0.0, -20.0, 20.0, -0.0]
    gu_d = to_dev(gu, dev)
    gate, up = gu_d[:, :N], gu_d[:, N:]
    xq, xs, act = ops.silu_mul_quantize(gate, up, bits, return_act=True)
    act_h = host(act)
    ref = oracle.silu_mul_ref(gu[:, :N], gu[:, N:])
    ok = within_one_ulp(act_h, ref)
    assert ok.all(), f"{int((~ok).sum())} products more than one fp16 ulp off"
    q_ref, xs_ref = oracle.quantize_engine(act_h, bits)
    np.testing.assert_array_equal(host(xq), q_ref)
    np.testing.assert_array_equal(hbits(host(xs)), hbits(xs_ref))


def test_producer_feeds_gemm(ops, dev):
    """SiLU * up -> A8 codes -> W6A8 down_proj GEMM equals quantize(act) -> GEMM, bit for bit."""
    M, N, K = 4, 1024, 2048  # down_proj: K = the FFN width
    r = rng(3)
    gu = r.standard_normal((M, 2 * K)).astype(np.float16)
    gu_d = to_dev(gu, dev)
    xq, xs, act = ops.silu_mul_quantize(gu_d[:, :K], gu_d[:, K:], 8, return_act=True)
    w = (r.standard_normal((N, K)) / np.sqrt(K)).astype(np.float16)
    wpk, _ = ops.quantize_pack_w6(to_dev(w, dev))
    d1 = ops.gemm_w6ax(xq, xs, wpk, N, 8)
    xq2, xs2 = ops.quantize_act(act, 8)
    d2 = ops.gemm_w6ax(xq2, xs2, wpk, N, 8)
    np.testing.assert_array_equal(hbits(host(d1)), hbits(host(d2)))


def test_producer_status_codes(ops, dev):
    from flexq_amd import _lib
    lib = _lib.load()
    P = lambda n: torch.empty(n, dtype=torch.uint8, device=dev)  # noqa: E731
    a, b, c = P(1 << 16), P(1 << 16), P(1 << 16)
    s = ops._stream(a)
    ptr = ops._ptr
    assert lib.fq_rmsnorm_quantize(None, ptr(a), ptr(b), 1e-6, 1, 100, 6, ptr(c), ptr(c), None, s) == 2
    assert lib.fq_rmsnorm_quantize(None, ptr(a), ptr(b), 1e-6, 1, 128, 7, ptr(c), ptr(c), None, s) == 3
    assert lib.fq_rmsnorm_quantize(None, None, ptr(b), 1e-6, 1, 128, 6, ptr(c), ptr(c), None, s) == 1
    assert lib.fq_silu_mul_quantize(ptr(a), ptr(b), 100, 1, 200, 8, ptr(c), ptr(c), None, s) == 2
    assert lib.fq_silu_mul_quantize(ptr(a), ptr(b), 128, 1, 128, 5, ptr(c), ptr(c), None, s) == 3


@pytest.mark.parametrize("M,K", [(1, 4096), (16, 11008), (64, 8192)])
def test_rmsnorm_within_one_ulp_of_reference_formula(ops, dev, M, K):
    """The reference's T5 RMSNorm (layernorm_kernels.cu:1851-1900: residual add, variance =
    sum(x^2) / n, rsqrtf(variance + eps), x * s * gamma) evaluated in float64 and rounded once to
    fp16: the kernel's normalised output is within one fp16 ulp of it everywhere."""
    r = rng(M + K)
    res = (r.standard_normal((M, K)) * 2.0).astype(np.float16)
    inp = (r.standard_normal((M, K)) * 0.5).astype(np.float16)
    gamma = (1.0 + 0.2 * r.standard_normal(K)).astype(np.float16)
    eps = 1e-6
    res_d = to_dev(res, dev)
    _, _, normed = ops.rmsnorm_quantize(res_d, to_dev(gamma, dev), 6, eps=eps, input=to_dev(inp, dev),
                                        return_normed=True)
    h = (res.astype(np.float64) + inp.astype(np.float64)).astype(np.float16).astype(np.float64)
    ref = h / np.sqrt((h * h).mean(axis=1, keepdims=True) + eps) * gamma.astype(np.float64)
    ref16 = ref.astype(np.float16)
    got = host(normed).astype(np.float64)
    ulp = np.spacing(np.abs(ref16)).astype(np.float64)
    assert np.all(np.abs(got - ref) <= ulp), float((np.abs(got - ref) / ulp).max())


def _image(ops, dev, N, K, seed):
    w = (rng(seed).standard_normal((N, K)) / np.sqrt(K)).astype(np.float16)
    return ops.quantize_pack_w6(to_dev(w, dev))[0]


# (M, N, K): the fused one-launch forms (M = 1, K = 4096: qkv, gate_up, a narrow S = 1 width) and
# the two-launch fallbacks (K != 4096, M > 1, a split-K shard width)
@pytest.mark.parametrize("M,N,K", [(1, 4096, 4096), (1, 12288, 4096), (1, 22016, 4096), (1, 2048, 4096),
                                   (1, 256, 4096), (1, 4096, 2048), (4, 4096, 4096), (16, 1024, 8192)])
@pytest.mark.parametrize("with_input", [True, False])
def test_rmsnorm_linear_matches_producer_then_gemm(ops, dev, M, N, K, with_input):
    """fq_rmsnorm_linear_w6ax (the norm inside the decode GEMM's prologue at M = 1, K = 4096)
    against fq_rmsnorm_quantize + fq_gemm_w6ax: output and updated residual bit-identical, the
    input residual untouched; and the output against the CPU oracle (norm + quantize + GEMM)."""
    from common import assert_gemm_close
    r = rng(M * 17 + N + K + with_input)
    res = (r.standard_normal((M, K)) * 2.0).astype(np.float16)
    inp = (r.standard_normal((M, K)) * 0.5).astype(np.float16) if with_input else None
    gamma = (1.0 + 0.2 * r.standard_normal(K)).astype(np.float16)
    res[0, :5] = [0.0, -0.0, 6e-8, -3e4, 3e4]
    eps = 1e-5
    wpk = _image(ops, dev, N, K, 5)
    res_d, g_d = to_dev(res, dev), to_dev(gamma, dev)
    inp_d = None if inp is None else to_dev(inp, dev)
    fused_expected = M == 1 and K == 4096 and ops.gemm_workspace_bytes(M, N, K) == 0
    assert (int(ops._lib.load().fq_rmsnorm_linear_scratch_bytes(M, N, K)) == 0) == fused_expected
    y, h = ops.rmsnorm_linear_w6ax(res_d, g_d, wpk, N, 6, eps=eps, input=inp_d)
    res2 = res_d.clone()
    xq, xs = ops.rmsnorm_quantize(res2, g_d, 6, eps=eps, input=inp_d)
    y2 = ops.gemm_w6ax(xq, xs, wpk, N, 6)
    np.testing.assert_array_equal(hbits(host(y)), hbits(host(y2)), err_msg="output")
    np.testing.assert_array_equal(hbits(host(h)), hbits(host(res2)), err_msg="updated residual")
    np.testing.assert_array_equal(hbits(host(res_d)), hbits(res), err_msg="the residual must not change")
    _, _, q_ref, xs_ref = oracle.rmsnorm_quantize(inp, res, gamma, eps, 6)
    wq, ws = ops.unpack_w6(wpk, N, K)
    ref, _, mag = oracle.gemm(q_ref, xs_ref, host(wq), host(ws))
    assert_gemm_close(host(y), ref, mag, "rmsnorm_linear vs oracle")


@pytest.mark.parametrize("M,N,K,bits", [(1, 4096, 11008, 8), (1, 4096, 14336, 8), (4, 4096, 11008, 8),
                                        (16, 2048, 4096, 6), (32, 1024, 2048, 8), (1, 512, 11008, 8),
                                        (64, 1024, 2048, 8), (1, 8192, 28672, 8)])
def test_silu_linear_matches_producer_then_gemm(ops, dev, M, N, K, bits):
    """fq_silu_linear_w6ax (SiLU * up inside the decode GEMM's prologue where the quantizer is fused)
    against fq_silu_mul_quantize + fq_gemm_w6ax over a merged [gate | up] buffer: bit-identical;
    and against the oracle GEMM of the producer's codes."""
    from common import assert_gemm_close
    r = rng(M * 5 + N + K)
    gu = (r.standard_normal((M, 2 * K)) * 3.0).astype(np.float16)
    gu[0, :4] = [0.0, -20.0, 20.0, -0.0]
    gu_d = to_dev(gu, dev)
    wpk = _image(ops, dev, N, K, 6)
    y = ops.silu_linear_w6ax(gu_d[:, :K], gu_d[:, K:], wpk, N, bits)
    xq, xs = ops.silu_mul_quantize(gu_d[:, :K], gu_d[:, K:], bits)
    y2 = ops.gemm_w6ax(xq, xs, wpk, N, bits)
    np.testing.assert_array_equal(hbits(host(y)), hbits(host(y2)))
    wq, ws = ops.unpack_w6(wpk, N, K)
    ref, _, mag = oracle.gemm(host(xq), host(xs), host(wq), host(ws))
    assert_gemm_close(host(y), ref, mag, "silu_linear vs oracle")


def test_fused_producer_linear_status_codes(ops, dev):
    from flexq_amd import _lib
    lib = _lib.load()
    P = lambda n: torch.empty(n, dtype=torch.uint8, device=dev)  # noqa: E731
    a, b, c, d = P(1 << 16), P(1 << 16), P(1 << 16), P(1 << 16)
    wpk = _image(ops, dev, 64, 128, 7)
    s = ops._stream(a)
    ptr = ops._ptr
    z = ctypes_size(0)
    # residual_out == residual with an input: refused (other workgroups still read the residual)
    assert lib.fq_rmsnorm_linear_w6ax(ptr(b), ptr(a), ptr(a), ptr(c), 1e-6, 1, 64, 128, 6, ptr(wpk), ptr(d),
                                      None, None, None, z, s) == 2
    assert lib.fq_rmsnorm_linear_w6ax(ptr(b), ptr(a), None, ptr(c), 1e-6, 1, 64, 128, 6, ptr(wpk), ptr(d),
                                      None, None, None, z, s) == 1
    assert lib.fq_rmsnorm_linear_w6ax(None, ptr(a), None, ptr(c), 1e-6, 1, 64, 100, 6, ptr(wpk), ptr(d),
                                      None, None, None, z, s) == 2
    assert lib.fq_silu_linear_w6ax(ptr(a), ptr(b), 64, 1, 64, 128, 8, ptr(wpk), ptr(d), None, None, None, z,
                                   s) == 2  # ld < K
    assert lib.fq_silu_linear_w6ax(ptr(a), ptr(b), 128, 1, 64, 128, 7, ptr(wpk), ptr(d), None, None, None, z,
                                   s) == 3
    torch.cuda.synchronize()


def ctypes_size(n):
    import ctypes
    return ctypes.c_size_t(n)


# ---- OPT-family LayerNorm producer (generalAddBiasResidualLayerNormOpt2FlexQFusion,
# layernorm_kernels.cu:316-575): residual output, normalised fp16, codes and scales bit-exact against
# oracle.layernorm_quantize (the kernel's summation order; fp16 elementwise steps as the reference)
def _ln_inputs(M, K, seed, with_input, with_bias, with_beta):
    r = rng(seed)
    res = (r.standard_normal((M, K)) * 2.0 + 0.25).astype(np.float16)
    inp = (r.standard_normal((M, K)) * 0.5).astype(np.float16) if with_input else None
    bias = (0.1 * r.standard_normal(K)).astype(np.float16) if with_bias else None
    gamma = (1.0 + 0.2 * r.standard_normal(K)).astype(np.float16)
    beta = (0.05 * r.standard_normal(K)).astype(np.float16) if with_beta else None
    res[0, :6] = [0.0, -0.0, 6e-8, -3e4, 3e4, 1e-3]
    return res, inp, bias, gamma, beta


@pytest.mark.parametrize("M,K", [(1, 4096), (3, 7168), (16, 4096), (5, 128), (2, 32768), (64, 9216), (2048, 4096)])
@pytest.mark.parametrize("bits", [6, 8])
@pytest.mark.parametrize("form", ["pre", "post", "post_nobias", "nobeta"])
def test_layernorm_quantize_bit_exact(ops, dev, M, K, bits, form):
    """pre: invokeGeneralLayerNorm's FlexQ form (residual only); post: bias + residual + input (the
    post-attention add, layernorm_kernels.cu:357-385); without bias; without beta."""
    with_input, with_bias, with_beta = {"pre": (False, False, True), "post": (True, True, True),
                                        "post_nobias": (True, False, True), "nobeta": (True, True, False)}[form]
    res, inp, bias, gamma, beta = _ln_inputs(M, K, M * 31 + K + bits, with_input, with_bias, with_beta)
    eps = 1e-5
    d = lambda a: None if a is None else to_dev(a, dev)  # noqa: E731
    res_d = d(res)
    rout = torch.empty_like(res_d)
    xq, xs, normed = ops.layernorm_quantize(res_d, d(gamma), bits, beta=d(beta), eps=eps, input=d(inp),
                                            bias=d(bias), residual_out=rout, return_normed=True)
    r_ref, n_ref, q_ref, xs_ref = oracle.layernorm_quantize(inp, res, gamma, beta, eps, bits, bias=bias)
    np.testing.assert_array_equal(hbits(host(rout)), hbits(r_ref), err_msg="residual out")
    np.testing.assert_array_equal(hbits(host(normed)), hbits(n_ref), err_msg="normed")
    np.testing.assert_array_equal(host(xq), q_ref, err_msg="codes")
    np.testing.assert_array_equal(hbits(host(xs)), hbits(xs_ref), err_msg="scales")
    np.testing.assert_array_equal(hbits(host(res_d)), hbits(res), err_msg="the residual must not change")


def test_layernorm_quantize_in_place(ops, dev):
    """residual_out may be the residual itself (each thread owns its chunks)."""
    res, inp, bias, gamma, beta = _ln_inputs(4, 4096, 3, True, True, True)
    res_d = to_dev(res, dev)
    xq, xs = ops.layernorm_quantize(res_d, to_dev(gamma, dev), 6, beta=to_dev(beta, dev), input=to_dev(inp, dev),
                                    bias=to_dev(bias, dev), residual_out=res_d)
    r_ref, _, q_ref, _ = oracle.layernorm_quantize(inp, res, gamma, beta, 1e-5, 6, bias=bias)
    np.testing.assert_array_equal(hbits(host(res_d)), hbits(r_ref))
    np.testing.assert_array_equal(host(xq), q_ref)


@pytest.mark.parametrize("M,N,K", [(1, 4096, 4096), (1, 12288, 4096), (1, 16384, 4096), (1, 256, 4096),
                                   (1, 4096, 7168), (4, 4096, 4096), (16, 1024, 9216)])
@pytest.mark.parametrize("form", ["pre", "post"])
def test_layernorm_linear_matches_producer_then_gemm(ops, dev, M, N, K, form):
    """fq_layernorm_linear_w6ax (LayerNorm inside the decode GEMM's prologue at M = 1, K = 4096: the
    OPT-6.7B width) against fq_layernorm_quantize + fq_gemm_w6ax: output and residual output
    bit-identical, the inputs untouched; and the output against the CPU oracle."""
    from common import assert_gemm_close
    post = form == "post"
    res, inp, bias, gamma, beta = _ln_inputs(M, K, M * 13 + N + K, post, post, True)
    eps = 1e-5
    wpk = _image(ops, dev, N, K, 8)
    d = lambda a: None if a is None else to_dev(a, dev)  # noqa: E731
    res_d, g_d, b_d, inp_d, bias_d = d(res), d(gamma), d(beta), d(inp), d(bias)
    fused_expected = M == 1 and K == 4096 and ops.gemm_workspace_bytes(M, N, K) == 0
    assert (int(ops._lib.load().fq_layernorm_linear_scratch_bytes(M, N, K)) == 0) == fused_expected
    rout = torch.empty_like(res_d)
    y, h = ops.layernorm_linear_w6ax(res_d, g_d, wpk, N, 6, beta=b_d, eps=eps, input=inp_d, bias=bias_d,
                                     residual_out=rout)
    rout2 = torch.empty_like(res_d)
    xq, xs = ops.layernorm_quantize(res_d, g_d, 6, beta=b_d, eps=eps, input=inp_d, bias=bias_d, residual_out=rout2)
    y2 = ops.gemm_w6ax(xq, xs, wpk, N, 6)
    np.testing.assert_array_equal(hbits(host(y)), hbits(host(y2)), err_msg="output")
    np.testing.assert_array_equal(hbits(host(h)), hbits(host(rout2)), err_msg="residual out")
    np.testing.assert_array_equal(hbits(host(res_d)), hbits(res), err_msg="the residual must not change")
    _, _, q_ref, xs_ref = oracle.layernorm_quantize(inp, res, gamma, beta, eps, 6, bias=bias)
    wq, ws = ops.unpack_w6(wpk, N, K)
    ref, _, mag = oracle.gemm(q_ref, xs_ref, host(wq), host(ws))
    assert_gemm_close(host(y), ref, mag, "layernorm_linear vs oracle")


def test_producer_linear_alias_rejections(ops, dev):
    """The one-launch forms write residual_out while other workgroups still read their inputs:
    residual_out overlapping the residual, the input or gamma is refused, for RMSNorm
    and LayerNorm alike, through the C ABI and the Python wrappers."""
    from flexq_amd import _lib
    lib = _lib.load()
    K, N = 4096, 256
    buf = torch.zeros(3 * K, dtype=torch.float16, device=dev)
    res, inp = buf[:K].view(1, K), buf[K:2 * K].view(1, K)
    gamma = torch.ones(K, dtype=torch.float16, device=dev)
    wpk = _image(ops, dev, N, K, 9)
    d = torch.empty((1, N), dtype=torch.float16, device=dev)
    s, ptr, z = ops._stream(res), ops._ptr, ctypes_size(0)
    for bad in (inp, buf[K + 8:2 * K + 8].view(1, K), res):  # input, overlapping the input, the residual
        assert lib.fq_rmsnorm_linear_w6ax(ptr(inp), ptr(res), ptr(bad), ptr(gamma), 1e-6, 1, N, K, 6, ptr(wpk),
                                          ptr(d), None, None, None, z, s) == 2
        assert lib.fq_layernorm_linear_w6ax(ptr(inp), ptr(res), None, ptr(bad), ptr(gamma), None, 1e-5, 1, N, K, 6,
                                            ptr(wpk), ptr(d), None, None, None, z, s) == 2
    g16 = torch.zeros(K, dtype=torch.float16, device=dev)
    assert lib.fq_rmsnorm_linear_w6ax(ptr(inp), ptr(res), ptr(g16), ptr(g16), 1e-6, 1, N, K, 6, ptr(wpk), ptr(d),
                                      None, None, None, z, s) == 2
    with pytest.raises(ValueError):
        ops.rmsnorm_linear_w6ax(res, gamma, wpk, N, input=inp, residual_out=inp)
    with pytest.raises(ValueError):
        ops.layernorm_linear_w6ax(res, gamma, wpk, N, input=inp, residual_out=res)
    torch.cuda.synchronize()
