"""Column-parallel W6Ax linears across GPUs.

Rank p of P holds output rows [p*N/P, (p+1)*N/P) of the weight (packed per shard into its own
weight image), the activations are replicated, every rank runs the fused linear on its shard,
and ONE all-gather over RCCL/xGMI (torch.distributed, backend "nccl") assembles the fp16 output.
Shards are 16-column aligned (the image's tile width).  The gather/reorder logic is
backend-agnostic and tested with gloo on CPU (tests/test_dist.py).
"""
import torch
import torch.distributed as dist

TILE = 16


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
    flat = torch.empty((world * M * n,), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(flat, local.contiguous().view(-1), group=group)
    full = flat.view(world, M, n)
    if out is None:
        out = torch.empty((M, world * n), dtype=local.dtype, device=local.device)
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
