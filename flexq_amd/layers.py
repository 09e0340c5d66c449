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

`FlexQDecoderLayer` adds the attention half around a caller-supplied attention core (the core
itself is out of scope): pre-attention RMSNorm + A6 codes -> qkv W6A6 -> attention
-> o_proj W6A6 -> the FFN above -> residual (FT LlamaContextDecoder.cc:430-660 order).

Every step runs the HIP kernels through the C ABI; nothing here computes on the CPU.  Weights come
from `flexq_amd.convert` files or from fp16 tensors.  Tensor parallelism is FT's layout
(flexq_amd.dist): qkv and gate_up column-parallel (rank p's files hold [q_p; k_p; v_p] and
[gate_p; up_p], so attention heads and SiLU*up are rank-local), o_proj and down_proj
row-parallel over those rank-local inputs, each finished by ONE all-reduce of the fp16 partial
outputs (RCCL over xGMI; `LlamaContextDecoder.cc:651`).  Two all-reduces per layer, no gathers.
"""
import json
import os

import torch
import torch.distributed as dist

from . import convert, ops
from .dist import all_reduce_sum


class W6Linear:
    """One packed W6Ax linear: `image` (fq_packed_w_bytes(N, K) bytes on the device), N x K,
    activations quantized to `abits` (6, or 8 for down_proj).  row_parallel: this is one rank's
    column shard of a row-parallel linear; its outputs are partial sums, all-reduced over `group`
    when called with reduce=True and the process group has more than one rank."""

    def __init__(self, image, N, K, abits=6, row_parallel=False, group=None):
        self.image, self.N, self.K, self.abits = image, N, K, abits
        self.row_parallel, self.group = row_parallel, group

    @classmethod
    def from_fp16(cls, w, abits=6):
        img, _ = ops.quantize_pack_w6(w.half().contiguous())
        return cls(img, w.shape[0], w.shape[1], abits)

    @classmethod
    def from_file(cls, path, device, group=None):
        img, meta = convert.load_image(path, device=device)
        row = meta["split"] == convert.ROW and meta["tp_size"] > 1
        return cls(img, meta["N"], meta["K"], meta["abits"], row_parallel=row, group=group)

    def _finish(self, y, reduce):
        if self.row_parallel and reduce and dist.is_initialized() and dist.get_world_size(self.group) > 1:
            all_reduce_sum(y, self.group)
        return y

    def __call__(self, x, out=None, reduce=True):
        """fp16 [M, K] -> fp16 [M, N] (quantize + GEMM; one launch at decode sizes)."""
        return self._finish(ops.linear_w6ax(x, self.image, self.N, self.abits, out=out), reduce)

    def from_codes(self, xq, xs, out=None, reduce=True):
        """Pre-quantized activations (a producer's output) -> fp16 [M, N]."""
        return self._finish(ops.gemm_w6ax(xq, xs, self.image, self.N, self.abits, out=out), reduce)


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
    def from_dir(cls, out_dir, layer, gamma, rank=0, device="cuda:0", eps=1e-6, group=None):
        """Load one layer's FFN (rank `rank`'s shards) from flexq_amd.convert output."""
        files = _layer_files(out_dir, layer, rank)
        gu = W6Linear.from_file(os.path.join(out_dir, files["mlp.gate_up_proj"]), device, group)
        dn = W6Linear.from_file(os.path.join(out_dir, files["mlp.down_proj"]), device, group)
        return cls(gu, dn, gamma.to(device=device, dtype=torch.float16), eps)

    def __call__(self, residual, attn_out=None, return_intermediates=False, reduce=True):
        """residual fp16 [M, H] (updated in place to residual + attn_out), attn_out fp16 [M, H] or
        None -> FFN output fp16 [M, H] (the caller adds it to the residual).  Tensor-parallel:
        this rank's gate_up / down shards; reduce=False returns the rank's partial sum."""
        xq, xs = ops.rmsnorm_quantize(residual, self.gamma, self.gate_up.abits, eps=self.eps, input=attn_out)
        gu = self.gate_up.from_codes(xq, xs)
        aq, as_ = ops.silu_mul_quantize(gu[:, :self.F], gu[:, self.F:], self.down.abits)
        y = self.down.from_codes(aq, as_, reduce=reduce)
        if return_intermediates:
            return y, dict(xq=xq, xs=xs, gate_up=gu, aq=aq, as_=as_)
        return y

    def fused(self, residual, attn_out, residual_out, reduce=True):
        """run_layers' form of __call__, the same bits: residual + attn_out goes to residual_out
        (not in place), the norm runs inside gate_up's GEMM and SiLU * up inside down_proj's (one
        launch each at decode sizes; ops.rmsnorm_linear_w6ax / silu_linear_w6ax).  Returns (y, the
        updated residual)."""
        gu, h = ops.rmsnorm_linear_w6ax(residual, self.gamma, self.gate_up.image, self.gate_up.N,
                                        self.gate_up.abits, eps=self.eps, input=attn_out,
                                        residual_out=residual_out if attn_out is not None else None)
        y = ops.silu_linear_w6ax(gu[:, :self.F], gu[:, self.F:], self.down.image, self.down.N, self.down.abits)
        return self.down._finish(y, reduce), h


def _layer_files(out_dir, layer, rank):
    m = json.load(open(os.path.join(out_dir, "manifest.json")))
    return {e["name"]: e["file"] for e in m["linears"] if e["layer"] == layer and e["rank"] == rank}


class FlexQDecoderLayer:
    """One LLaMA decoder layer in FlexQ mode around a caller-supplied attention core
    (FT `LlamaContextDecoder::forward`, int8_mode 5, LlamaContextDecoder.cc:430-660):

        xq, xs = rmsnorm_quantize(h, gamma_attn, 6)               (pre-attention norm + A6 codes)
        ctx    = attn_fn(qkv.from_codes(xq, xs))                  (rank-local heads: [M, 3H/P] -> [M, H/P])
        a      = o_proj(ctx)           + all-reduce                (row-parallel, W6A6)
        y      = FlexQFfn(h, a)        + all-reduce in down_proj   (h += a inside the fused norm)
        h     += y

    `attn_fn` is the out-of-scope attention (RoPE, KV cache, softmax): any callable mapping this
    rank's qkv output [M, q + k + v columns] to its context [M, o_proj.K]."""

    def __init__(self, qkv, o, ffn, gamma_attn, attn_fn, eps=1e-6):
        if o.K % 128:
            raise ValueError("o_proj input width must be whole 128-groups (head_dim 128 = one group)")
        self.qkv, self.o, self.ffn, self.gamma_attn, self.attn_fn, self.eps = qkv, o, ffn, gamma_attn, attn_fn, eps

    @classmethod
    def from_dir(cls, out_dir, layer, gamma_attn, gamma_ffn, attn_fn, rank=0, device="cuda:0", eps=1e-6,
                 group=None):
        files = _layer_files(out_dir, layer, rank)
        qkv = W6Linear.from_file(os.path.join(out_dir, files["attention.query_key_value"]), device, group)
        o = W6Linear.from_file(os.path.join(out_dir, files["attention.dense"]), device, group)
        ffn = FlexQFfn.from_dir(out_dir, layer, gamma_ffn, rank, device, eps, group)
        return cls(qkv, o, ffn, gamma_attn.to(device=device, dtype=torch.float16), attn_fn, eps)

    def attention(self, h, reduce=True, pending=None):
        """h fp16 [M, H] -> attention output [M, H] (this rank's partial sum when reduce=False).
        h is not modified, unless `pending` (the previous layer's FFN output) is given: then
        h += pending is fused into the pre-attention norm (FT's add-residual + norm kernel)."""
        xq, xs = ops.rmsnorm_quantize(h, self.gamma_attn, self.qkv.abits, eps=self.eps, input=pending)
        ctx = self.attn_fn(self.qkv.from_codes(xq, xs))
        return self.o(ctx.contiguous(), reduce=reduce)

    def step(self, h, pending, spare, reduce=True):
        """run_layers' form of one layer (defer=True, the same bits): the two fused residual adds
        write the other of two residual buffers (h, spare) instead of updating h in place -- a
        decode GEMM's other workgroups are still reading h -- and both norms and SiLU * up run
        inside their GEMMs (layer = qkv, o_proj, gate_up, down_proj: four launches at M = 1 plus
        the attention core).  Returns (y to pass as the next `pending`, the residual, the free
        buffer)."""
        qkv, h1 = ops.rmsnorm_linear_w6ax(h, self.gamma_attn, self.qkv.image, self.qkv.N, self.qkv.abits,
                                         eps=self.eps, input=pending,
                                         residual_out=spare if pending is not None else None)
        free = h if pending is not None else spare
        a = self.o(self.attn_fn(qkv).contiguous(), reduce=reduce)
        y, h2 = self.ffn.fused(h1, a, free, reduce=reduce)
        return y, h2, h1

    def __call__(self, h, pending=None, defer=False, reduce=True):
        """h fp16 [M, H], updated in place to the layer output and returned.  With defer=True the
        final residual add is left to the caller: the FFN output y is returned instead (h holds
        the layer input + attention), to be passed as the next layer's `pending` -- one launch
        less per layer, the same bits (the fused add is the same fp16 addition)."""
        a = self.attention(h, reduce=reduce, pending=pending)
        y = self.ffn(h, a, reduce=reduce)  # h += a (fused into the pre-FFN norm)
        if defer:
            return y
        h += y
        return h


def run_layers_chained(layers, h, check=False):
    """run_layers on one rank as decode chains (ops.linear_chain_w6ax), the same bits: the first
    layer's RMSNorm + qkv alone, then per layer one chain o_i -> RMSNorm + gate_up_i -> SiLU * up +
    down_i -> RMSNorm + qkv_i+1 (the last layer's without the qkv): the linears between two attention
    cores in one persistent launch where the chain allows it (M = 1 for the norms), their entry points
    otherwise.  The attention core (attn_fn) must return a view of its input or a tensor computed
    before the chain (as the bench's stand-in ctx = v does): a chain cannot run a kernel between its
    links.  The residual rotates through three buffers (h and two scratch), since a chain reads one and
    writes two.  Returns h.
    Speed: measured SLOWER than run_layers' one-launch-per-linear form (1.353 vs 1.320 ms per 32-layer
    LLaMA-2-7B step at M = 1, round 5: each producer hand-off -- the RMSNorm's cross-wave sum, SiLU * up
    polling two sources -- costs more than the kernel boundary it removes), so bench.py no longer times it
    and run_layers stays the decoder path; kept as a tested, bit-identical API.
    Failure: a chain wait that timed out (e.g. other kernels holding CUs the chain needs, include/flexq_hip.h)
    leaves the stream's chain workspace in the timed-out state, and the next call raises
    _lib.ChainTimeoutError before launching anything (ops.chain_reset clears it).  check=True also
    synchronises after the step and raises if THIS step timed out (its h is then undefined)."""
    if dist.is_initialized() and any(L.o.row_parallel and dist.get_world_size(L.o.group) > 1 for L in layers):
        raise ValueError("run_layers_chained is single-rank (tensor parallelism needs the all-reduces between links)")
    if not layers:
        return h
    if check:
        out = run_layers_chained(layers, h)
        torch.cuda.current_stream(h.device).synchronize()
        if ops.chain_status(h.device):
            from ._lib import ChainTimeoutError
            raise ChainTimeoutError("run_layers_chained", 6)
        return out
    M, H = h.shape
    dev = h.device
    res = [h, torch.empty_like(h), torch.empty_like(h)]
    r = 0  # res[r] holds the current residual value
    L0 = layers[0]
    qkv = torch.empty((M, L0.qkv.N), dtype=torch.float16, device=dev)
    ops.rmsnorm_linear_w6ax(res[r], L0.gamma_attn, L0.qkv.image, L0.qkv.N, L0.qkv.abits, eps=L0.eps, out=qkv)
    pending = None
    for i, L in enumerate(layers):
        F = L.ffn.F
        ctx = L.attn_fn(qkv)
        if not ctx.is_contiguous():
            ctx = ctx.contiguous()
        a = torch.empty((M, L.o.N), dtype=torch.float16, device=dev)
        gu = torch.empty((M, L.ffn.gate_up.N), dtype=torch.float16, device=dev)
        y = torch.empty((M, L.ffn.down.N), dtype=torch.float16, device=dev)
        r1, r2 = (r + 1) % 3, (r + 2) % 3
        links = [(ctx, L.o.image, L.o.N, L.o.abits, a),
                 ops.chain_rmsnorm(res[r], L.ffn.gamma, L.ffn.gate_up.image, L.ffn.gate_up.N, L.ffn.gate_up.abits, gu,
                                   input=a, residual_out=res[r1], eps=L.ffn.eps),
                 ops.chain_silu(gu[:, :F], gu[:, F:], L.ffn.down.image, L.ffn.down.N, L.ffn.down.abits, y)]
        if i + 1 < len(layers):
            Ln = layers[i + 1]
            qkv = torch.empty((M, Ln.qkv.N), dtype=torch.float16, device=dev)
            links.append(ops.chain_rmsnorm(res[r1], Ln.gamma_attn, Ln.qkv.image, Ln.qkv.N, Ln.qkv.abits, qkv,
                                           input=y, residual_out=res[r2], eps=Ln.eps))
            r = r2
        else:
            r, pending = r1, y
        ops.linear_chain_w6ax(links)
    torch.add(res[r], pending, out=h)  # (res[r] may be h itself: an elementwise in-place add)
    return h


def run_layers(layers, h, reduce=True):
    """Run decoder layers in order on h (in place), each layer's final residual add fused into the
    next layer's pre-attention norm, the norms and SiLU * up fused into their GEMMs
    (FlexQDecoderLayer.step; the residual alternates between h and one scratch buffer); returns h.  reduce=False (no all-reduces) is a single-rank /
    timing mode: with more than one rank the unreduced partial sums would feed the next layer's
    norm, so it is rejected there."""
    if not reduce and dist.is_initialized() and any(
            L.o.row_parallel and dist.get_world_size(L.o.group) > 1 for L in layers):
        raise ValueError("run_layers(reduce=False) is single-rank only: with more than one rank every "
                         "layer's input must be the all-reduced sum")
    pending, cur, spare = None, h, torch.empty_like(h)
    for L in layers:
        pending, cur, spare = L.step(cur, pending, spare, reduce=reduce)
    if pending is not None:
        torch.add(cur, pending, out=h)  # (cur may be h itself: an elementwise in-place add)
    return h
