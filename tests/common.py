"""Shared test helpers: deterministic inputs and the oracle comparisons."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import fq_oracle as oracle  # noqa: E402,F401  (test infrastructure: the checker)


def rng(seed):
    return np.random.Generator(np.random.PCG64(seed))


def kat_operands(M, N, K, abits, seed):
    """Mirror of the reference kernel test inputs (test_bgemm_kernel.cu:20-63): raw b-bit patterns
    uniform over [0, 2^b) read as two's complement, fp16 scales U[0, 0.1)."""
    r = rng(seed)
    xraw = r.integers(0, 1 << abits, size=(M, K), dtype=np.int32)
    wraw = r.integers(0, 1 << 6, size=(N, K), dtype=np.int32)
    xq = ((xraw ^ (1 << (abits - 1))) - (1 << (abits - 1))).astype(np.int8)
    wq = ((wraw ^ 32) - 32).astype(np.int8)
    xs = (r.random((K // 128, M), dtype=np.float32) * np.float32(0.1)).astype(np.float16)
    ws = (r.random((K // 128, N), dtype=np.float32) * np.float32(0.1)).astype(np.float16)
    return xraw, wraw, xq, wq, xs, ws


def model_operands(M, N, K, abits, seed):
    """Model-like inputs: W ~ N(0, 0.02), X ~ N(0,1) with 1% outlier channels,
    both quantized with the engine rule by the oracle."""
    from inputs import act_input, weight_input
    x = act_input(M, K, seed + 1).astype(np.float16)
    w = weight_input(N, K, seed + 2).astype(np.float16)
    xq, xs = oracle.quantize_engine(x, abits)
    wq, ws = oracle.quantize_engine(w, 6)
    return x, w, xq, wq, xs, ws


def assert_gemm_close(got, ref, mag, what=""):
    got = got.astype(np.float64)
    refd = ref.astype(np.float64)
    tol = oracle.gemm_tolerance(ref, mag)
    err = np.abs(got - refd)
    bad = err > tol
    if bad.any():
        i = np.argwhere(bad)[0]
        raise AssertionError(
            f"{what}: {int(bad.sum())} of {bad.size} outputs outside tolerance; first at {tuple(i)}: "
            f"got {got[tuple(i)]!r} ref {refd[tuple(i)]!r} tol {tol[tuple(i)]!r}")
