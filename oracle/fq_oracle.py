"""Python face of the CPU oracle.  TEST INFRASTRUCTURE ONLY.

Two contracts live here:
  * engine semantics -- ctypes bindings of oracle/fq_oracle.c (bit-plane packing, the e2e dynamic
    quantizer, the reference's compute_ref, and the int32-accumulator GEMM contract).
  * Python fake-quant semantics -- `fake_quant_*` / `quant_linear_forward` below restate
    algorithm/flexq_quantize/quantizer.py:93-171 and int_linear.py:56-72 with the same torch CPU
    ops, so they can be pinned bit-for-bit against tests/golden/*.npz and timed as the CPU baseline
    (bench.py `cpu_baseline`, kind "port").

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def build():
    """Compile libfq_oracle.so with gcc (no GPU needed)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "libfq_oracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        P = ctypes.c_void_p
        I = ctypes.c_int
        for name, args in {
            "fqo_pack_bitplanes": [P, I, I, I, P],
            "fqo_unpack_bitplanes": [P, I, I, I, P],
            "fqo_pack_abq": [P, I, I, I, P],
            "fqo_quantize_engine": [P, I, I, I, P, P],
            "fqo_compute_ref": [P, P, P, P, P, I, I, I, I, I],
            "fqo_gemm": [P, P, P, P, I, I, I, P, P, P],
            "fqo_gemm_decode_order": [P, P, P, P, I, I, I, I, P],
            "fqo_xs_to_ref_dup": [P, I, I, P],
            "fqo_pack_fq6": [P, P, I, I, P],
            "fqo_unpack_fq6": [P, I, I, P, P],
            "fqo_rmsnorm_quantize": [P, P, P, ctypes.c_float, I, I, I, P, P, P],
            "fqo_silu_mul_ref": [P, P, I, I, I, P],
            "fqo_layernorm_quantize": [P, P, P, P, P, P, ctypes.c_float, I, I, I, P, P, P],
        }.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = I
        L.fqo_fq6_bytes.argtypes = [I, I]
        L.fqo_fq6_bytes.restype = ctypes.c_size_t
        L.fqo_f32_to_f16.argtypes = [ctypes.c_float]
        L.fqo_f32_to_f16.restype = ctypes.c_uint16
        _LIB = L
    return _LIB


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _check(rc, what):
    if rc != 0:
        raise ValueError(f"oracle {what} rejected its arguments (rc={rc})")


# ------------------------------------------------------------------ engine-side restatements

def pack_bitplanes(vals, bits):
    """int values [R,K] -> reference bit-plane layout int32 (bit_packing.cu:76-133)."""
    vals = np.ascontiguousarray(vals, dtype=np.int32)
    R, K = vals.shape
    out = np.zeros(bits * R * (K // 32), dtype=np.int32)
    _check(lib().fqo_pack_bitplanes(_p(vals), R, K, bits, _p(out)), "pack_bitplanes")
    return out


def unpack_bitplanes(packed, R, K, bits):
    packed = np.ascontiguousarray(packed, dtype=np.int32)
    out = np.zeros((R, K), dtype=np.int32)
    _check(lib().fqo_unpack_bitplanes(_p(packed), R, K, bits, _p(out)), "unpack_bitplanes")
    return out


def pack_abq(vals, bits):
    vals = np.ascontiguousarray(vals, dtype=np.int32)
    R, K = vals.shape
    out = np.zeros(bits * R * (K // 32), dtype=np.uint32)
    _check(lib().fqo_pack_abq(_p(vals), R, K, bits, _p(out)), "pack_abq")
    return out


def quantize_engine(x_f16, bits):
    """e2e dynamic quantizer semantics -> (q int8 [M,K], xs fp16 [K/128, M])."""
    x = np.ascontiguousarray(x_f16, dtype=np.float16)
    M, K = x.shape
    q = np.zeros((M, K), dtype=np.int8)
    xs = np.zeros((K // 128, M), dtype=np.float16)
    _check(lib().fqo_quantize_engine(_p(x), M, K, bits, _p(q), _p(xs)), "quantize_engine")
    return q, xs


def rmsnorm_quantize(inp, residual, gamma, eps, bits):
    """Residual add + RMSNorm + engine quantizer (layernorm_kernels.cu:1851-2051, the HIP kernel's
    summation order) -> (residual_out, normed fp16 [M,K], q int8 [M,K], xs fp16 [K/128, M])."""
    res = np.array(residual, dtype=np.float16, copy=True, order="C")
    M, K = res.shape
    g = np.ascontiguousarray(gamma, dtype=np.float16)
    normed = np.zeros((M, K), dtype=np.float16)
    q = np.zeros((M, K), dtype=np.int8)
    xs = np.zeros((K // 128, M), dtype=np.float16)
    inp = None if inp is None else np.ascontiguousarray(inp, dtype=np.float16)
    _check(lib().fqo_rmsnorm_quantize(None if inp is None else _p(inp), _p(res), _p(g), eps, M, K, bits,
                                      _p(q), _p(xs), _p(normed)), "rmsnorm_quantize")
    return res, normed, q, xs


def layernorm_quantize(inp, residual, gamma, beta, eps, bits, bias=None):
    """OPT-family bias + residual + input LayerNorm + engine quantizer (layernorm_kernels.cu:316-575,
    the HIP kernel's summation order) -> (residual_out = half(v), normed fp16 [M,K], q int8 [M,K],
    xs fp16 [K/128, M]).  inp, beta, bias may be None."""
    res = np.ascontiguousarray(residual, dtype=np.float16)
    M, K = res.shape
    g = np.ascontiguousarray(gamma, dtype=np.float16)
    b = None if beta is None else np.ascontiguousarray(beta, dtype=np.float16)
    bi = None if bias is None else np.ascontiguousarray(bias, dtype=np.float16)
    inp = None if inp is None else np.ascontiguousarray(inp, dtype=np.float16)
    rout = np.zeros((M, K), dtype=np.float16)
    normed = np.zeros((M, K), dtype=np.float16)
    q = np.zeros((M, K), dtype=np.int8)
    xs = np.zeros((K // 128, M), dtype=np.float16)
    opt = lambda a: None if a is None else _p(a)  # noqa: E731
    _check(lib().fqo_layernorm_quantize(opt(inp), _p(res), opt(bi), _p(rout), _p(g), opt(b), ctypes.c_float(eps),
                                        M, K, bits, _p(q), _p(xs), _p(normed)), "layernorm_quantize")
    return rout, normed, q, xs


def silu_mul_ref(gate, up):
    """half(silu(gate) * up) evaluated in double (activation_kernels.cu:133,300)."""
    g = np.ascontiguousarray(gate, dtype=np.float16)
    u = np.ascontiguousarray(up, dtype=np.float16)
    M, N = g.shape
    act = np.zeros((M, N), dtype=np.float16)
    _check(lib().fqo_silu_mul_ref(_p(g), _p(u), N, M, N, _p(act)), "silu_mul_ref")
    return act


def xs_to_ref_dup(xs, M, K):
    xs = np.ascontiguousarray(xs, dtype=np.float16)
    ld = 2 * ((M + 3) // 4 * 4)
    dup = np.zeros((K // 128, ld), dtype=np.float16)
    lib().fqo_xs_to_ref_dup(_p(xs), M, K, _p(dup))
    return dup


def compute_ref(w_packed, w_scale, x_packed, x_scale_dup, M, N, K, wbits, xbits):
    """The reference's own CPU oracle (test_bgemm_kernel.cu:113-146), restated."""
    out = np.zeros((M, N), dtype=np.float16)
    args = [np.ascontiguousarray(a) for a in (w_packed, w_scale, x_packed, x_scale_dup)]
    _check(lib().fqo_compute_ref(_p(args[0]), _p(args[1]), _p(args[2]), _p(args[3]), _p(out),
                                 M, N, K, wbits, xbits), "compute_ref")
    return out


def gemm(xq, xs, wq, ws, want_acc=False):
    """Contract oracle -> (D fp16 [M,N], acc int32 [M,N,K/128] or None, mag float64 [M,N])."""
    xq = np.ascontiguousarray(xq, dtype=np.int8)
    wq = np.ascontiguousarray(wq, dtype=np.int8)
    xs = np.ascontiguousarray(xs, dtype=np.float16)
    ws = np.ascontiguousarray(ws, dtype=np.float16)
    M, K = xq.shape
    N = wq.shape[0]
    out = np.zeros((M, N), dtype=np.float16)
    mag = np.zeros((M, N), dtype=np.float64)
    acc = np.zeros((M, N, K // 128), dtype=np.int32) if want_acc else None
    _check(lib().fqo_gemm(_p(xq), _p(xs), _p(wq), _p(ws), M, N, K, _p(out),
                          _p(acc) if want_acc else None, _p(mag)), "gemm")
    return out, acc, mag


def gemm_decode_order(xq, xs, wq, ws, nw=8):
    """The decode kernel's exact fp32 summation order at S = 1 (NW waves per workgroup: 8 for M <= 16)
    -> D fp16 [M,N], bit-identical to the production decode / chain output (fq_oracle.c)."""
    xq = np.ascontiguousarray(xq, dtype=np.int8)
    wq = np.ascontiguousarray(wq, dtype=np.int8)
    xs = np.ascontiguousarray(xs, dtype=np.float16)
    ws = np.ascontiguousarray(ws, dtype=np.float16)
    M, K = xq.shape
    N = wq.shape[0]
    out = np.zeros((M, N), dtype=np.float16)
    f = lib().fqo_gemm_decode_order
    _check(f(_p(xq), _p(xs), _p(wq), _p(ws), M, N, K, int(nw), _p(out)), "gemm_decode_order")
    return out


def check_div_by_const(hi):
    """Mismatches of the quantizer's Newton-corrected absmax / hi against IEEE division over
    every fp16 absmax (oracle/fq_oracle.c fqo_check_div_by_const); 0 means bit-identical."""
    f = lib().fqo_check_div_by_const
    f.argtypes = [ctypes.c_int]
    f.restype = ctypes.c_long
    return int(f(hi))


def check_quant_fma(bits, rc_ulp=0):
    """Mismatches of the device quantizer's single-FMA element step (biased reciprocal, truncation)
    against roundf(x / s) over every fp16 absmax and element, with the hardware reciprocal moved
    by rc_ulp units in the last place (oracle/fq_oracle.c fqo_check_quant_fma); 0 = identical."""
    f = lib().fqo_check_quant_fma
    f.argtypes = [ctypes.c_int, ctypes.c_int]
    f.restype = ctypes.c_long
    return int(f(bits, rc_ulp))


def fq6_bytes(N, K):
    return int(lib().fqo_fq6_bytes(N, K))


def pack_fq6(wq, ws=None):
    """Weight image: fq6 blocks + blocked fp16 scales (ws [K/128, N]; zeros if None)."""
    wq = np.ascontiguousarray(wq, dtype=np.int8)
    N, K = wq.shape
    if ws is None:
        ws = np.zeros((K // 128, N), np.float16)
    ws = np.ascontiguousarray(ws, dtype=np.float16)
    assert ws.shape == (K // 128, N)
    out = np.zeros(fq6_bytes(N, K), dtype=np.uint8)
    _check(lib().fqo_pack_fq6(_p(wq), _p(ws), N, K, _p(out)), "pack_fq6")
    return out


def unpack_fq6(packed, N, K, want_ws=False):
    wq = np.zeros((N, K), dtype=np.int8)
    ws = np.zeros((K // 128, N), dtype=np.float16)
    _check(lib().fqo_unpack_fq6(_p(np.ascontiguousarray(packed, dtype=np.uint8)), N, K, _p(wq), _p(ws)),
           "unpack_fq6")
    if want_ws:
        return wq, ws
    return wq


def quantize_weight_engine(w_f16, bits=6):
    """Per-output-row, per-128-group symmetric weight quantisation with the engine rounding rule
    (same math as the activation quantizer); returns (wq int8 [N,K], ws fp16 [K/128, N])."""
    return quantize_engine(w_f16, bits)


def gemm_tolerance(ref, mag):
    """Allowed |hip - oracle| per output: 1e-3 relative (north star) plus the fp32 accumulation
    floor the HIP kernel is entitled to (2^-20 of sum_g |s_g acc_g|) plus one fp16 subnormal."""
    return 1e-3 * np.abs(ref.astype(np.float64)) + mag * 2.0 ** -20 + 6e-8


# ------------------------------------------------------------------ Python fake-quant restatement

CLIPMIN = 1e-5


def fake_quant_per_group(x, n_bits, group_size=128):
    """UniformAffineQuantizer(symmetric=True, disable_zero_point=True, dynamic per_group).forward,
    quantizer.py:128-171 (calibration) + 93-125 (fake_quant); returns (x_hat, scale, codes).
    Accepts [M,K] or [1,S,K] (quantizer.py:99-101); larger 3-D inputs are flattened to [-1,K]
    (the reference asserts there)."""
    import torch
    shape = x.shape
    x2 = x.reshape(-1, shape[-1])
    xg = x2.reshape(-1, group_size)
    xmin = xg.amin([-1], keepdim=True)
    xmax = xg.amax([-1], keepdim=True)
    abs_max = torch.max(xmax.abs(), xmin.abs())
    scale = (abs_max / (2 ** (n_bits - 1) - 1)).clamp(min=CLIPMIN, max=1e4)
    qmin, qmax = -(2 ** (n_bits - 1)), 2 ** (n_bits - 1) - 1
    v = xg / scale
    codes = ((v.round() - v) + v).clamp(qmin, qmax)  # round_ste (quantizer.py:28-32): -0.0 -> +0.0
    xhat = codes.mul(scale).reshape(shape)
    return xhat, scale, codes


def quant_linear_forward(x, weight, w_bits=6, a_bits=6, requant_weight=True, w_hat=None):
    """QuantLinear.forward with use_weight_quant and use_act_quant (int_linear.py:56-72).
    requant_weight=True is the reference eval flow (flexqllm.py:106-108 leaves use_weight_quant on,
    so the weight is fake-quantised again on every forward); pass w_hat to time the
    pre-quantised variant."""
    import torch.nn.functional as F
    if w_hat is None or requant_weight:
        w_hat, _, _ = fake_quant_per_group(weight, w_bits)
    xhat, _, _ = fake_quant_per_group(x, a_bits)
    return F.linear(xhat, w_hat)
