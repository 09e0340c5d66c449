"""Deterministic synthetic inputs shared by the golden generator and the tests.

numpy's PCG64 bit generator is stable across numpy versions, so the same seed gives the same
float32 draws here and on the GPU box.  Values are produced in float32 and cast by the caller.
"""
import numpy as np


def act_input(M, K, seed):
    """Activation-like: N(0,1) with 1% of K-channels scaled x16 (outliers), SURVEY.md §8(d)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    x = rng.standard_normal((M, K), dtype=np.float32)
    ch = rng.choice(K, size=max(1, K // 100), replace=False)
    x[:, ch] *= 16.0
    return x


def weight_input(N, K, seed):
    """Weight-like: N(0, 0.02)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return (rng.standard_normal((N, K), dtype=np.float32) * np.float32(0.02)).astype(np.float32)


def edge_inputs():
    """Edge cases for the dynamic quantizer."""
    rng = np.random.Generator(np.random.PCG64(99))
    K = 512
    zero = rng.standard_normal((4, K), dtype=np.float32)
    zero[1, 128:256] = 0.0  # an all-zero group
    zero[3, :] = 0.0  # an all-zero row
    # exact ties: values that are k+0.5 multiples of the group scale (absmax 31 -> scale 1)
    ties = np.tile(np.arange(-15.5, 16.5, 0.5, dtype=np.float32), (2, 8))[:, :K]
    ties[:, ::128] = 31.0
    out = rng.standard_normal((2, K), dtype=np.float32)
    out[0, 5] = 3000.0  # huge outlier inside a group
    out[1, 300] = -1e-3  # tiny group
    out[1, 256:384] *= 1e-4
    tiny = (rng.standard_normal((1, K), dtype=np.float32) * np.float32(1e-6)).astype(np.float32)
    three_d = rng.standard_normal((1, 3, K), dtype=np.float32)
    return {"zero": zero, "ties": ties, "outlier": out, "tiny": tiny, "three_d": three_d}
