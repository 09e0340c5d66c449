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
import numpy as np
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


# ------------------------------------------------------------------------- peer-store all-gather

def _hip():
    """The HIP runtime torch already loaded (IPC calls only; kernels go through libflexq_hip.so)."""
    import ctypes
    import ctypes.util
    for name in ("libamdhip64.so", "libamdhip64.so.7", "libamdhip64.so.6"):
        try:
            return ctypes.CDLL(name)
        except OSError:
            continue
    raise RuntimeError("libamdhip64 not found")


_IPC_HANDLE = []


def _handle_type():
    """hipIpcMemHandle_t (64 bytes), a Structure so that ctypes passes it BY VALUE to
    hipIpcOpenMemHandle (a char array would decay to a pointer)."""
    if not _IPC_HANDLE:
        import ctypes

        class IpcMemHandle(ctypes.Structure):
            _fields_ = [("reserved", ctypes.c_char * 64)]  # HIP_IPC_HANDLE_SIZE
        _IPC_HANDLE.append(IpcMemHandle)
    return _IPC_HANDLE[0]


def _ipc_export(t):
    """(handle bytes, offset) of a device tensor: the IPC handle names the whole allocation that
    holds it (torch's caching allocator sub-allocates), the offset locates the tensor in it."""
    import ctypes
    hip = _hip()
    base, size = ctypes.c_void_p(), ctypes.c_size_t()
    if hip.hipMemGetAddressRange(ctypes.byref(base), ctypes.byref(size), ctypes.c_void_p(t.data_ptr())) != 0:
        raise RuntimeError("hipMemGetAddressRange failed")
    h = _handle_type()()
    if hip.hipIpcGetMemHandle(ctypes.byref(h), base) != 0:
        raise RuntimeError("hipIpcGetMemHandle failed (HSA_ENABLE_IPC_MODE_LEGACY=0 is required)")
    return bytes(h), t.data_ptr() - base.value


def _ipc_open(handle, offset):
    import ctypes
    hip = _hip()
    h = _handle_type().from_buffer_copy(handle)
    p = ctypes.c_void_p()
    hip.hipIpcOpenMemHandle.argtypes = [ctypes.POINTER(ctypes.c_void_p), _handle_type(), ctypes.c_uint]
    st = hip.hipIpcOpenMemHandle(ctypes.byref(p), h, ctypes.c_uint(1))  # hipIpcMemLazyEnablePeerAccess
    if st != 0:
        raise RuntimeError(f"hipIpcOpenMemHandle failed (hipError {st})")
    return p.value, p.value + offset


class _DevArray:
    """__cuda_array_interface__ of a raw device allocation (torch.as_tensor wraps it without a copy)."""

    def __init__(self, ptr, shape, typestr):
        self.__cuda_array_interface__ = {"shape": tuple(shape), "typestr": typestr, "data": (ptr, False),
                                         "version": 2, "strides": None}


def _uncached_zeros(shape, dtype, dev):
    """A zeroed device tensor in UNCACHED device memory (hipExtMallocWithFlags(hipDeviceMallocUncached)):
    the gather buffers and flags that peers store into over xGMI are then never served from a stale
    line of this GPU's L2.  Returns (tensor, raw pointer to hipFree) or (plain torch.zeros, None)
    when the allocation or the wrapping is not available."""
    import ctypes
    import torch
    nbytes = int(np.prod(shape)) * torch.tensor([], dtype=dtype).element_size()
    try:
        hip = _hip()
        p = ctypes.c_void_p()
        hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
        if hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(nbytes), ctypes.c_uint(0x3)) != 0 or not p.value:
            raise RuntimeError("hipExtMallocWithFlags(hipDeviceMallocUncached) failed")
        if hip.hipMemset(p, 0, ctypes.c_size_t(nbytes)) != 0:
            hip.hipFree(p)
            raise RuntimeError("hipMemset failed")
        typestr = {torch.float16: "<f2", torch.int32: "<i4"}[dtype]
        t = torch.as_tensor(_DevArray(p.value, shape, typestr), device=dev)
        if t.data_ptr() != p.value:
            hip.hipFree(p)
            raise RuntimeError("the tensor does not alias the allocation")
        return t, p.value
    except Exception:  # noqa: BLE001
        return torch.zeros(shape, dtype=dtype, device=dev), None


def _exportable_zeros(shape, dtype, dev):
    """(tensor, raw uncached pointer or None, IPC export): uncached memory when it can be allocated,
    wrapped and IPC-exported, else torch memory (every rank then reports `uncached` False)."""
    import ctypes
    import torch
    t, raw = _uncached_zeros(shape, dtype, dev)
    if raw is not None:
        try:
            torch.cuda.synchronize(dev)
            return t, raw, _ipc_export(t)
        except RuntimeError:
            del t
            _hip().hipFree(ctypes.c_void_p(raw))
    t = torch.zeros(shape, dtype=dtype, device=dev)
    torch.cuda.synchronize(dev)
    return t, None, _ipc_export(t)


class PeerGather:
    """Buffers of the fused peer-store all-gather (include/flexq_hip.h fq_linear_w6ax_gather): two
    gather buffers fp16 [M_max, N_total] per rank, used alternately, plus the rank's flag words, all
    IPC-exported and opened by every other rank (xGMI peer mappings on a node; the same device in
    the one-GPU multi-process tests), and one device fq_gather descriptor per buffer parity.

    `linear(x, image, abits)` runs this rank's column shard of a linear, stores it into every rank's
    gather buffer, waits until all ranks' shards have arrived and returns the full [M, N_total]
    output, a view of this rank's gather buffer.  Lifetime: the output of call c must be consumed
    (or copied) by work enqueued on the stream BEFORE this object's next linear() call.  After call
    c + 1 a peer may already be at call c + 2, which stores into the same buffer parity as call c
    (it only waits for every rank's call c + 1 flag), so reading output c after enqueuing call
    c + 1 races with those stores.  Replaces ColumnParallelW6Linear's RCCL all_gather
    at decode sizes (M <= 32).  The buffers and flags are uncached device memory (`uncached`)."""

    def __init__(self, M_max, N_total, group=None, device=None):
        import ctypes
        import torch
        from . import ops  # noqa: F401  (loads the library)
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if self.world > 8:
            raise ValueError("at most 8 ranks (FQ_GATHER_MAX_RANKS)")
        self.M_max, self.N_total, self.group = M_max, N_total, group
        self.lo, self.hi = shard_range(N_total, self.world, self.rank)
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.dev = dev
        # the buffers peers store into, and the flags they raise, live in uncached device memory (no
        # stale L2 line of this GPU can serve a read of a peer's xGMI store)
        allocs = [_exportable_zeros((M_max, N_total), torch.float16, dev) for _ in range(2)]
        allocs.append(_exportable_zeros((8,), torch.int32, dev))
        self._raw = [a[1] for a in allocs if a[1] is not None]
        self.uncached = len(self._raw) == 3
        self.bufs = [allocs[0][0], allocs[1][0]]
        self.flags = allocs[2][0]
        self.state = torch.zeros(2, dtype=torch.int32, device=dev)  # done, gen
        self.err = torch.zeros(1, dtype=torch.int32, device=dev)
        torch.cuda.synchronize(dev)
        mine = [a[2] for a in allocs]
        allh = [None] * self.world
        dist.all_gather_object(allh, mine, group=group)
        self._opened = []
        ptrs = []  # per rank q: (buf0, buf1, flags)
        failure = None
        try:
            for q in range(self.world):
                if q == self.rank:
                    ptrs.append((self.bufs[0].data_ptr(), self.bufs[1].data_ptr(), self.flags.data_ptr()))
                    continue
                row = []
                for (h, off) in allh[q]:
                    base, p = _ipc_open(h, off)
                    self._opened.append(base)
                    row.append(p)
                ptrs.append(tuple(row))
        except Exception as e:  # noqa: BLE001
            failure = f"rank {self.rank}: {e}"
        # every rank learns whether every mapping succeeded, so a failure raises on all ranks alike
        # (no rank may go on to store into, or wait on, a peer that could not map it)
        fails = [None] * self.world
        dist.all_gather_object(fails, failure, group=group)
        if any(fails):
            self.close()
            raise RuntimeError("PeerGather: IPC mapping failed: " + "; ".join(f for f in fails if f))
        # two descriptors (fq_gather, include/flexq_hip.h): buffer parity 0 and 1
        P8 = ctypes.c_uint64 * 8
        I4 = ctypes.c_int32 * 4

        class Desc(ctypes.Structure):
            _fields_ = [("out", P8), ("flags", P8), ("done", ctypes.c_uint64), ("gen", ctypes.c_uint64), ("ints", I4)]
        self.desc = []
        for parity in range(2):
            d = Desc()
            for q in range(self.world):
                d.out[q] = ptrs[q][parity]
                d.flags[q] = ptrs[q][2]
            d.done = self.state.data_ptr()
            d.gen = self.state.data_ptr() + 4
            d.ints = I4(self.world, self.rank, self.lo, N_total)
            raw = torch.frombuffer(bytearray(bytes(d)), dtype=torch.uint8)
            self.desc.append(raw.to(dev))
        torch.cuda.synchronize(dev)
        dist.barrier(group=group)  # every rank's buffers are mapped before anyone stores into them
        self.calls = 0

    def linear(self, x, image, abits=6, parity=None, after=None, wait=True):
        """x fp16 [M, K] (replicated) -> full output [M, N_total] (this rank's gather buffer).
        parity: which of the two gather buffers (default: alternate per call); a caller capturing
        a fixed sequence of calls (a HIP graph) passes it explicitly, alternating per object.
        after=(pg, parity): x is the output of that PeerGather call, issued with wait=False: its
        wait runs inside this launch (fq_linear_w6ax_gather_after: after the weight DMAs, no wait
        launch) when both objects' buffers are uncached, else as fq_gather_wait first.
        wait=False: skip this call's own wait -- the caller must pass after=(self, parity) to the
        next linear that reads this output (or call wait(parity) before reading it otherwise)."""
        import ctypes
        import torch
        from . import _lib, ops
        M, K = x.shape
        if M > self.M_max:
            raise ValueError(f"M={M} > M_max={self.M_max}")
        n = self.hi - self.lo
        if parity is None:
            parity = self.calls & 1
            self.calls += 1
        s = ops._stream(x)
        nb = ops.gemm_workspace_bytes(M, n, K)
        wbuf = ops.workspace(x.device, nb, s.value)
        xq = xs = None
        if ops.act_scratch_bytes(M, n, K):
            xq = torch.empty((M, K), dtype=torch.int8, device=x.device)
            xs = torch.empty((K // GROUP, M), dtype=torch.float16, device=x.device)
        wsz = ctypes.c_size_t(wbuf.numel() if wbuf is not None else 0)
        if after is not None:
            src, sp = after
            if self.uncached and src.uncached:
                _lib.call("fq_linear_w6ax_gather_after", ops._ptr(x), ops._ptr(src.desc[sp]), ops._ptr(src.err), M, n,
                          K, abits, ops._ptr(image), ops._ptr(self.desc[parity]), ops._ptr(xq), ops._ptr(xs),
                          ops._ptr(wbuf), wsz, s)
            else:
                src.wait(sp, x)
                after = None
        if after is None:
            _lib.call("fq_linear_w6ax_gather", ops._ptr(x), M, n, K, abits, ops._ptr(image),
                      ops._ptr(self.desc[parity]), ops._ptr(xq), ops._ptr(xs), ops._ptr(wbuf), wsz, s)
        if wait:
            self.wait(parity, x)
        return self.bufs[parity][:M]

    def wait(self, parity, like):
        """fq_gather_wait for this object's latest call (the stream of tensor `like`)."""
        from . import _lib, ops
        _lib.call("fq_gather_wait", ops._ptr(self.desc[parity]), ops._ptr(self.err), ops._stream(like))

    def error(self):
        """Nonzero when a wait timed out (a rank stopped publishing)."""
        return int(self.err.item())

    def close(self):
        """Unmap the peers' buffers.  This rank's own uncached buffers stay allocated for the life of
        the process: a captured graph may still name them, and peers may still hold mappings."""
        hip = _hip()
        import ctypes
        for p in self._opened:
            hip.hipIpcCloseMemHandle(ctypes.c_void_p(p))
        self._opened = []
