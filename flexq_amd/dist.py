"""Tensor-parallel W6Ax linears across GPUs.

Column-parallel (the north-star N-shard): rank p of P holds output rows [p*N/P, (p+1)*N/P) of
the weight (packed per shard into its own weight image), the activations are replicated, every
rank runs the fused linear on its shard, and ONE all-gather over RCCL/xGMI (torch.distributed,
backend "nccl") assembles the fp16 output.  Shards are 16-column aligned (the image's tile width).

Row-parallel (FT's decoder layout, `LlamaDecoderLayerWeight.cc:386-409`: attention.dense and
mlp.down_proj are split along their input dimension, `hidden / tp` and `inter / tp`, and the
partial outputs are summed by `ftNcclAllReduceSum`, `LlamaContextDecoder.cc:651`): rank p holds
the weight columns [k_lo, k_hi), split on 128-group boundaries, so its activation quantization
groups are exactly the single-GPU groups of that slice (codes, scales and the per-group int32
accumulators are unchanged), and ONE all-reduce (sum) of the fp16 partial outputs finishes the
linear.  Its input is rank-local: the attention heads of the rank (head_dim 128 = one group) or
its SiLU*up slice [gate_p; up_p], which the column-parallel qkv / gate_up feed without any
exchange.  The gather / reduce logic is backend-agnostic and tested with gloo on CPU
(tests/test_dist.py).
"""
import torch
import torch.distributed as dist

TILE = 16
GROUP = 128


def shard_range(N, world, rank):
    """Output rows [lo, hi) of rank `rank`: equal 16-aligned shards."""
    if N % (TILE * world):
        raise ValueError(f"N={N} does not split into {world} shards of whole {TILE}-column tiles")
    n = N // world
    return rank * n, (rank + 1) * n


def shard_weight(w, world, rank):
    """Rows of a [N, K] weight (codes, or fp16 for fq_quantize_pack_w6) owned by `rank`."""
    lo, hi = shard_range(w.shape[0], world, rank)
    return w[lo:hi].contiguous()


def shard_scales(ws, world, rank):
    """Columns of a [K/128, N] scale matrix owned by `rank`."""
    lo, hi = shard_range(ws.shape[1], world, rank)
    return ws[:, lo:hi].contiguous()


def gather_columns(local, group=None, out=None):
    """[M, N/P] per rank -> [M, N] on every rank with one all_gather_into_tensor.  The collective
    returns [P][M][N/P] (rank-major); for M = 1 that already is [N], otherwise one transpose."""
    world = dist.get_world_size(group)
    M, n = local.shape
    if out is None:
        out = torch.empty((M, world * n), dtype=local.dtype, device=local.device)
    if M == 1 and out.is_contiguous() and not (local.is_cuda and dist.get_backend(group) == "gloo"):
        # rank-major IS the column order: gather straight into the output (no copy launch)
        dist.all_gather_into_tensor(out.view(-1), local.contiguous().view(-1), group=group)
        return out
    flat = torch.empty((world * M * n,), dtype=local.dtype, device=local.device)
    if local.is_cuda and dist.get_backend(group) == "gloo":  # gloo: device tensors through the host
        host = torch.empty((world * M * n,), dtype=local.dtype)
        dist.all_gather_into_tensor(host, local.contiguous().view(-1).cpu(), group=group)
        flat.copy_(host)
    else:
        dist.all_gather_into_tensor(flat, local.contiguous().view(-1), group=group)
    full = flat.view(world, M, n)
    if M == 1:
        out.view(-1).copy_(flat)
    else:
        out.view(M, world, n).copy_(full.permute(1, 0, 2))
    return out


class ColumnParallelW6Linear:
    """One rank's part of a column-parallel W6Ax linear: `image` is this rank's shard
    (ops.pack_w6 / quantize_pack_w6 of shard_weight(...)), N the full output width."""

    def __init__(self, image, N, K, abits=6, group=None):
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.N, self.K, self.abits, self.group = N, K, abits, group
        self.lo, self.hi = shard_range(N, self.world, self.rank)
        self.image = image

    def __call__(self, x):
        from . import ops
        local = ops.linear_w6ax(x, self.image, self.hi - self.lo, self.abits)
        if self.world == 1:
            return local
        return gather_columns(local, self.group)


def group_shard_range(D, world, rank):
    """[lo, hi) of rank `rank` when a dimension of D (a multiple of 128) is split on 128-group
    boundaries, as evenly as whole groups allow (the first D/128 mod P ranks hold one more group:
    LLaMA-2-7B's 11008 = 86 groups at P = 4 -> 22, 22, 21, 21).  Used for the K of row-parallel
    linears and the matching rows of the column-parallel gate/up that feed them."""
    if D % GROUP:
        raise ValueError(f"{D} is not a multiple of the {GROUP}-wide group")
    G = D // GROUP
    if G < world:
        raise ValueError(f"{G} groups cannot be split over {world} ranks")
    q, r = divmod(G, world)
    lo = rank * q + min(rank, r)
    return lo * GROUP, (lo + q + (1 if rank < r else 0)) * GROUP


def shard_weight_k(w, world, rank):
    """Columns of a [N, K] weight owned by `rank` in a row-parallel linear."""
    lo, hi = group_shard_range(w.shape[1], world, rank)
    return w[:, lo:hi].contiguous()


def all_reduce_sum(t, group=None):
    """In-place sum of the ranks' partial outputs (RCCL all-reduce over xGMI on GPUs)."""
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


class RowParallelW6Linear:
    """One rank's part of a row-parallel W6Ax linear: `image` packs this rank's weight columns
    [k_lo, k_hi) (ops.quantize_pack_w6 of shard_weight_k(...)); the input is the rank-local
    activation slice [M, k_hi - k_lo]; the output is the full [M, N] after one all-reduce."""

    def __init__(self, image, N, K, abits=6, group=None):
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.N, self.K, self.abits, self.group = N, K, abits, group
        self.k_lo, self.k_hi = group_shard_range(K, self.world, self.rank)
        self.image = image

    def __call__(self, x_local, reduce=True):
        from . import ops
        if x_local.shape[-1] != self.k_hi - self.k_lo:
            raise ValueError(f"rank-local input must have {self.k_hi - self.k_lo} columns")
        part = ops.linear_w6ax(x_local, self.image, self.N, self.abits)
        if self.world > 1 and reduce:
            all_reduce_sum(part, self.group)
        return part
