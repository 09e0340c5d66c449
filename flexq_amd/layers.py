"""Caller-side blocks built from the engine (the callers either side of the path).

`W6Linear` is one packed W6Ax linear; `FlexQFfn` is FT's LLaMA FFN in its FlexQ mode
(`FfnLayer::forward` with `int8_mode == 5`, e2e .../layers/FfnLayer.cc:371-401, 440-452,
521-561, fed by the fused pre-FFN norm of LlamaContextDecoder.cc:576-592):

    residual += attn_out                                   (residual add, in place)
    xq, xs = rmsnorm_quantize(residual, gamma, 6)          (layernorm_kernels.cu:1851)
    gu     = [gate | up] = W6A6 GEMM(xq, xs)               (ONE launch over the stacked image;
                                                            the reference runs two GEMMs)
    aq, as = silu_mul_quantize(gate, up, 8)                (activation_kernels.cu:245, A8)
    y      = W6A8 GEMM(aq, as)  (down_proj)                (FfnLayer.cc:540-558)

Every step runs the HIP kernels through the C ABI; nothing here computes on the CPU.  Weights come
from `flexq_amd.convert` files or from fp16 tensors.  The block is one whole layer (TP 1); with
the column-parallel shards of `flexq_amd.dist`, rank p's gate_up file holds [gate_p; up_p], so
its SiLU step is rank-local, and down_proj (sharded by output rows, full K) needs the ranks' A8
codes gathered first (one all-gather of M x F bytes + scales) before the per-rank down GEMM.
"""
import json
import os

import torch

from . import convert, ops


class W6Linear:
    """One packed W6Ax linear: `image` (fq_packed_w_bytes(N, K) bytes on the device), N x K,
    activations quantized to `abits` (6, or 8 for down_proj)."""

    def __init__(self, image, N, K, abits=6):
        self.image, self.N, self.K, self.abits = image, N, K, abits

    @classmethod
    def from_fp16(cls, w, abits=6):
        img, _ = ops.quantize_pack_w6(w.half().contiguous())
        return cls(img, w.shape[0], w.shape[1], abits)

    @classmethod
    def from_file(cls, path, device):
        img, meta = convert.load_image(path, device=device)
        return cls(img, meta["N"], meta["K"], meta["abits"])

    def __call__(self, x, out=None):
        """fp16 [M, K] -> fp16 [M, N] (quantize + GEMM; one launch at decode sizes)."""
        return ops.linear_w6ax(x, self.image, self.N, self.abits, out=out)

    def from_codes(self, xq, xs, out=None):
        """Pre-quantized activations (a producer's output) -> fp16 [M, N]."""
        return ops.gemm_w6ax(xq, xs, self.image, self.N, self.abits, out=out)


class FlexQFfn:
    """LLaMA FFN block in FlexQ mode (see the module docstring)."""

    def __init__(self, gate_up, down, gamma, eps=1e-6):
        if gate_up.N % 2 or gate_up.N // 2 != down.K:
            raise ValueError("gate_up must stack [gate; up] rows of the down_proj input width")
        if down.abits != 8 and down.abits != 6:
            raise ValueError("down_proj abits must be 6 or 8")
        self.gate_up, self.down, self.gamma, self.eps = gate_up, down, gamma, eps
        self.F = down.K

    @classmethod
    def from_dir(cls, out_dir, layer, gamma, rank=0, device="cuda:0", eps=1e-6):
        """Load one layer's FFN from flexq_amd.convert output (manifest.json + .fqw6 files)."""
        m = json.load(open(os.path.join(out_dir, "manifest.json")))
        files = {e["name"]: e["file"] for e in m["linears"] if e["layer"] == layer and e["rank"] == rank}
        gu = W6Linear.from_file(os.path.join(out_dir, files["mlp.gate_up_proj"]), device)
        dn = W6Linear.from_file(os.path.join(out_dir, files["mlp.down_proj"]), device)
        return cls(gu, dn, gamma.to(device=device, dtype=torch.float16), eps)

    def __call__(self, residual, attn_out=None, return_intermediates=False):
        """residual fp16 [M, H] (updated in place to residual + attn_out), attn_out fp16 [M, H] or
        None -> FFN output fp16 [M, H] (the caller adds it to the residual)."""
        xq, xs = ops.rmsnorm_quantize(residual, self.gamma, self.gate_up.abits, eps=self.eps, input=attn_out)
        gu = self.gate_up.from_codes(xq, xs)
        aq, as_ = ops.silu_mul_quantize(gu[:, :self.F], gu[:, self.F:], self.down.abits)
        y = self.down.from_codes(aq, as_)
        if return_intermediates:
            return y, dict(xq=xq, xs=xs, gate_up=gu, aq=aq, as_=as_)
        return y
