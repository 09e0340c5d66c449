"""CPU checks of the producer oracles (oracle/fq_oracle.c fqo_rmsnorm_quantize, fqo_silu_mul_ref)
against float64 numpy restatements of the reference formulas (layernorm_kernels.cu:1883-1898,
activation_kernels.cu:133,300).  The reference ships no fixtures for these kernels, so this pins
the restatement's formula; the GPU tests pin the kernels to the oracle."""
import numpy as np

from common import oracle, rng


def test_rmsnorm_oracle_matches_float64_formula():
    r = rng(11)
    M, K = 4, 4096
    res = r.standard_normal((M, K)).astype(np.float16)
    inp = r.standard_normal((M, K)).astype(np.float16)
    gamma = (1 + 0.1 * r.standard_normal(K)).astype(np.float16)
    r_out, normed, q, xs = oracle.rmsnorm_quantize(inp, res, gamma, 1e-6, 6)
    added = (inp.astype(np.float32) + res.astype(np.float32)).astype(np.float16)
    np.testing.assert_array_equal(r_out, added)  # one fp32 add, one fp16 rounding: exact
    a = added.astype(np.float64)
    ref = a / np.sqrt((a * a).mean(1, keepdims=True) + 1e-6) * gamma.astype(np.float64)
    ulp = np.spacing(np.abs(ref).astype(np.float16)).astype(np.float64)
    assert (np.abs(normed.astype(np.float64) - ref) <= ulp).all()
    q2, xs2 = oracle.quantize_engine(normed, 6)
    np.testing.assert_array_equal(q, q2)
    np.testing.assert_array_equal(xs.view(np.uint16), xs2.view(np.uint16))


def test_rmsnorm_oracle_clamps_like_the_reference():
    """clamp_inf_for_half (reduce_kernel_utils.cuh:357-361): sums past fp16 range become
    +-64512 (= half(64504)), not inf."""
    K = 128
    res = np.full((1, K), 60000.0, np.float16)
    inp = np.full((1, K), 30000.0, np.float16)
    inp[0, 1] = -30000.0
    r_out, _, _, _ = oracle.rmsnorm_quantize(inp, res, np.ones(K, np.float16), 1e-6, 8)
    assert float(r_out[0, 0]) == 64512.0 and float(r_out[0, 1]) == 30000.0


def test_silu_mul_oracle():
    g = np.array([[0.0, 1.0, -1.0, 10.0, -10.0, 3.5, -0.25, 20.0]], np.float16)
    u = np.array([[1.0, 2.0, 2.0, 0.5, 0.5, -1.0, 4.0, 1.0]], np.float16)
    act = oracle.silu_mul_ref(g, u)
    gd, ud = g.astype(np.float64), u.astype(np.float64)
    np.testing.assert_array_equal(act, (gd / (1 + np.exp(-gd)) * ud).astype(np.float16))


def _ln_numpy(inp, res, gamma, beta, eps, bias=None):
    """generalAddBiasResidualLayerNormOpt2FlexQFusion's element arithmetic in numpy (fp32 sums with
    a different summation order, fp16 elementwise normalisation, layernorm_kernels.cu:357-416)."""
    v = np.zeros(res.shape, np.float32)
    if bias is not None:
        v = v + bias.astype(np.float32)
    v = v + res.astype(np.float32)
    if inp is not None:
        v = v + inp.astype(np.float32)
    h = v.astype(np.float16)
    K = res.shape[1]
    s = v.astype(np.float64).sum(1, keepdims=True)
    q = (v.astype(np.float64) ** 2).sum(1, keepdims=True)
    mean = s / K
    rs = 1.0 / np.sqrt(q / K - mean * mean + eps)
    a = (h - mean.astype(np.float16)).astype(np.float16)
    a = (a * rs.astype(np.float16)).astype(np.float16)
    a = (a * gamma).astype(np.float16)
    if beta is not None:
        a = (a + beta).astype(np.float16)
    return h, a, mean, rs


def test_layernorm_oracle_matches_reference_formula():
    """The oracle's LayerNorm (fqo_layernorm_quantize) against the reference's formula in numpy:
    the residual output exactly; the mean and 1/sigma the oracle rounds to fp16 coincide with the
    float64 ones rounded to fp16 on (almost) every row, and where they do the normalised output is
    bit-identical (every later step is an fp16 operation)."""
    r = rng(12)
    M, K = 16, 4096
    res = (r.standard_normal((M, K)) * 2 + 0.3).astype(np.float16)
    inp = (r.standard_normal((M, K)) * 0.5).astype(np.float16)
    bias = (0.1 * r.standard_normal(K)).astype(np.float16)
    gamma = (1 + 0.1 * r.standard_normal(K)).astype(np.float16)
    beta = (0.05 * r.standard_normal(K)).astype(np.float16)
    r_out, normed, q, xs = oracle.layernorm_quantize(inp, res, gamma, beta, 1e-5, 6, bias=bias)
    h, ref, mean, rs = _ln_numpy(inp, res, gamma, beta, 1e-5, bias=bias)
    np.testing.assert_array_equal(r_out.view(np.uint16), h.view(np.uint16))
    same = 0
    for m in range(M):
        if np.array_equal(normed[m].view(np.uint16), ref[m].view(np.uint16)):
            same += 1
    assert same >= M - 1, f"only {same} of {M} rows bit-identical to the reference formula"
    q2, xs2 = oracle.quantize_engine(normed, 6)
    np.testing.assert_array_equal(q, q2)
    np.testing.assert_array_equal(xs.view(np.uint16), xs2.view(np.uint16))


def test_layernorm_oracle_pre_attention_form():
    """invokeGeneralLayerNorm's FlexQ form (layernorm_kernels.cu:2325-2420): the residual alone, no
    input, no bias; without beta the output is ((h - mean) * rs) * gamma."""
    r = rng(13)
    res = r.standard_normal((3, 1024)).astype(np.float16)
    gamma = (1 + 0.1 * r.standard_normal(1024)).astype(np.float16)
    r_out, normed, _, _ = oracle.layernorm_quantize(None, res, gamma, None, 1e-5, 8)
    np.testing.assert_array_equal(r_out.view(np.uint16), res.view(np.uint16))
    _, ref, _, _ = _ln_numpy(None, res, gamma, None, 1e-5)
    assert (normed.view(np.uint16) == ref.view(np.uint16)).mean() > 0.99
