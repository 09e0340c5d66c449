"""Torch-facing wrappers of the C ABI (include/flexq_hip.h).

Every function validates shapes/dtypes/devices on the host before anything is enqueued, passes
raw device pointers and torch's current HIP stream to libflexq_hip.so, and returns new tensors.
There is no fallback: CPU tensors are rejected and a missing library raises.
"""
import ctypes

import torch

from . import _lib

GROUP = 128


def _stream(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _need(cond, msg):
    if not cond:
        raise ValueError(msg)


def _dev(t, dtype, name, dim=None):
    _need(isinstance(t, torch.Tensor), f"{name} must be a tensor")
    _need(t.is_cuda, f"{name} must be a HIP device tensor (no CPU path by design)")
    _need(t.dtype == dtype, f"{name} must be {dtype}, got {t.dtype}")
    _need(t.is_contiguous(), f"{name} must be contiguous")
    if dim is not None:
        _need(t.dim() == dim, f"{name} must be {dim}-D, got shape {tuple(t.shape)}")


def _k_ok(K):
    _need(K > 0 and K % GROUP == 0, f"K={K} must be a positive multiple of {GROUP}")


# ------------------------------------------------------------------------- sizes / workspace

def packed_w_bytes(N, K):
    return int(_lib.load().fq_packed_w_bytes(N, K))


def gemm_workspace_bytes(M, N, K):
    return int(_lib.load().fq_gemm_workspace_bytes(M, N, K))


_WS = {}
_WS_CAPTURED = set()  # ids of workspaces a HIP graph capture has seen
_WS_RETIRED = []  # superseded workspaces a captured graph may still address


def workspace(device, nbytes, stream_handle):
    """Per-(device, stream) scratch for the split-K fix-up and the prefill weight unpack (zeroed
    once, the ticket region kept zero by the kernels).  It grows geometrically (x1.5, 1 MiB
    granules), so a rising sequence of shapes reallocates O(log) times.  A superseded buffer that a
    graph capture has seen is kept for the process (the graph bakes its address into its launches:
    split-K tickets and slabs, the unpack image); one no capture has seen is released."""
    if nbytes == 0:
        return None
    key = (device, stream_handle)
    buf = _WS.get(key)
    if buf is None or buf.numel() < nbytes:
        old = buf.numel() if buf is not None else 0
        nbytes = max(nbytes, old + old // 2, 1 << 20)
        nbytes = (nbytes + (1 << 20) - 1) >> 20 << 20
        if buf is not None and id(buf) in _WS_CAPTURED:
            _WS_RETIRED.append(buf)
        buf = torch.empty(nbytes, dtype=torch.uint8, device=device)
        _lib.call("fq_workspace_init", _ptr(buf), ctypes.c_size_t(nbytes), ctypes.c_void_p(stream_handle))
        _WS[key] = buf
    if torch.cuda.is_current_stream_capturing():
        _WS_CAPTURED.add(id(buf))
    return buf


_CWS = {}  # (device, stream) -> chain workspace (fq_chain_workspace_init; written by chain launches only)
_CWS_STATUS = {}  # chain workspace data_ptr -> its pinned host status word (fq_chain_bind_status)
_CWS_HOSTS = []  # every host status word ever bound, kept for the process: a superseded workspace may still
                 # have a chain in flight whose timed-out wait stores into its word


def chain_workspace(device, nbytes, stream_handle):
    """Per-(device, stream) chain workspace of fq_linear_chain_w6ax: zeroed once, then written by chain
    launches only; grown like workspace() (a superseded one a capture has seen is kept).  Each one has a
    pinned host status word bound to it (a timed-out in-kernel wait sets it; chain_status reads it)."""
    key = (device, stream_handle)
    buf = _CWS.get(key)
    if buf is None or buf.numel() < nbytes:
        old = buf.numel() if buf is not None else 0
        nbytes = max(nbytes, old + old // 2, 1 << 20)
        nbytes = (nbytes + (1 << 20) - 1) >> 20 << 20
        if buf is not None and id(buf) in _WS_CAPTURED:
            _WS_RETIRED.append(buf)
        buf = torch.empty(nbytes, dtype=torch.uint8, device=device)
        _lib.call("fq_chain_workspace_init", _ptr(buf), ctypes.c_size_t(nbytes), ctypes.c_void_p(stream_handle))
        if hasattr(_lib.load(), "fq_chain_bind_status"):  # (an older A/B build may lack it)
            host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
            _lib.call("fq_chain_bind_status", _ptr(buf), ctypes.c_size_t(nbytes), ctypes.c_void_p(host.data_ptr()),
                      ctypes.c_void_p(stream_handle))
            _CWS_STATUS[buf.data_ptr()] = host
            _CWS_HOSTS.append(host)
        _CWS[key] = buf
    if torch.cuda.is_current_stream_capturing():
        _WS_CAPTURED.add(id(buf))
    return buf


def workspace_device_bytes():
    """Bytes held by the workspaces (current and retired), for tests and diagnostics."""
    return (sum(b.numel() for b in _WS.values()) + sum(b.numel() for b in _CWS.values()) +
            sum(b.numel() for b in _WS_RETIRED))


def reserve_workspace(device, shapes, stream=None):
    """Size the stream's workspace once for the largest of `shapes` [(M, N, K)] before any graph
    capture (the way a serving loop would at start-up), so no later call grows it."""
    s = stream if stream is not None else torch.cuda.current_stream(device)
    nb = max((gemm_workspace_bytes(M, N, K) for (M, N, K) in shapes), default=0)
    return workspace(torch.device(device), nb, s.cuda_stream)


# ------------------------------------------------------------------------- weights

def _ws_ok(ws, N, K, dev):
    _dev(ws, torch.float16, "ws", 2)
    _need(tuple(ws.shape) == (K // GROUP, N), f"ws must be [K/128, N] = {(K // GROUP, N)}")
    _need(ws.device == dev, "ws must be on the weights' device")


def pack_w6(wq, ws):
    """int8 codes [N,K] in [-32,31] + fp16 group scales [K/128, N] -> weight image (uint8)."""
    _dev(wq, torch.int8, "wq", 2)
    N, K = wq.shape
    _k_ok(K)
    _ws_ok(ws, N, K, wq.device)
    out = torch.empty(packed_w_bytes(N, K), dtype=torch.uint8, device=wq.device)
    _lib.call("fq_pack_w6", _ptr(wq), _ptr(ws), N, K, _ptr(out), _stream(wq))
    return out


def unpack_w6(wpk, N, K):
    """Weight image -> (int8 codes [N,K], fp16 scales [K/128, N])."""
    _img_ok(wpk, N, K)
    out = torch.empty((N, K), dtype=torch.int8, device=wpk.device)
    ws = torch.empty((K // GROUP, N), dtype=torch.float16, device=wpk.device)
    _lib.call("fq_unpack_w6", _ptr(wpk), N, K, _ptr(out), _ptr(ws), _stream(wpk))
    return out, ws


def _img_ok(wpk, N, K):
    _dev(wpk, torch.uint8, "w_packed", 1)
    _k_ok(K)
    _need(N > 0 and wpk.numel() == packed_w_bytes(N, K), "w_packed size does not match (N, K)")


def quantize_pack_w6(w, return_codes=False):
    """fp16 weight [N,K] -> (weight image, ws fp16 [K/128, N]) (+ int8 codes if requested)."""
    _dev(w, torch.float16, "w", 2)
    N, K = w.shape
    _k_ok(K)
    wpk = torch.empty(packed_w_bytes(N, K), dtype=torch.uint8, device=w.device)
    ws = torch.empty((K // GROUP, N), dtype=torch.float16, device=w.device)
    wq = torch.empty((N, K), dtype=torch.int8, device=w.device) if return_codes else None
    _lib.call("fq_quantize_pack_w6", _ptr(w), N, K, _ptr(wpk), _ptr(ws), _ptr(wq), _stream(w))
    return (wpk, ws, wq) if return_codes else (wpk, ws)


# ------------------------------------------------------------------------- activations

def quantize_act(x, abits):
    """fp16 [M,K] -> (xq int8 [M,K], xs fp16 [K/128, M]) -- engine rounding semantics."""
    _dev(x, torch.float16, "x", 2)
    _need(abits in (6, 8), "abits must be 6 or 8")
    M, K = x.shape
    _k_ok(K)
    xq = torch.empty((M, K), dtype=torch.int8, device=x.device)
    xs = torch.empty((K // GROUP, M), dtype=torch.float16, device=x.device)
    _lib.call("fq_quantize_act", _ptr(x), M, K, abits, _ptr(xq), _ptr(xs), _stream(x))
    return xq, xs


# ------------------------------------------------------------------------- GEMM

PREFILL_U8_MIN_M = 2048  # fq_gemm_w6ax unpacks the weights (once per call) at and above this M


def prepare_prefill_weights(wpk, N, K):
    """The weight image's int8 MFMA operands, unpacked once (fq_prefill_unpack_weights; 1 byte per
    weight): pass them as gemm_w6ax / linear_w6ax(..., w_u8=) so that prefill-sized calls skip the
    per-call unpack pass.  A uint8 tensor owned by the caller (the model), on the image's device."""
    _img_ok(wpk, N, K)
    nb = int(_lib.load().fq_prefill_weight_bytes(N, K))
    w_u8 = torch.empty(nb, dtype=torch.uint8, device=wpk.device)
    _lib.call("fq_prefill_unpack_weights", _ptr(wpk), N, K, _ptr(w_u8), _stream(wpk))
    return w_u8


def gemm_w6ax(xq, xs, wpk, N, abits=6, return_acc=False, out=None, w_u8=None):
    """d fp16 [M,N] from quantized operands; with return_acc also the int32 group accumulators
    [M, N, K/128] (bit-exact debug output).  w_u8: the prepared operands of prepare_prefill_weights
    (fq_gemm_w6ax_u8; bit-identical, no per-call unpack at M >= 2048)."""
    _dev(xq, torch.int8, "xq", 2)
    M, K = xq.shape
    _k_ok(K)
    _dev(xs, torch.float16, "xs", 2)
    _need(tuple(xs.shape) == (K // GROUP, M), f"xs must be [K/128, M] = {(K // GROUP, M)}")
    _img_ok(wpk, N, K)
    _need(abits in (6, 8), "abits must be 6 or 8")
    dev = xq.device
    for t in (xs, wpk):
        _need(t.device == dev, "all operands must be on one device")
    if out is None:
        out = torch.empty((M, N), dtype=torch.float16, device=dev)
    else:
        _dev(out, torch.float16, "out", 2)
        _need(tuple(out.shape) == (M, N), "out shape mismatch")
    acc = torch.empty((M, N, K // GROUP), dtype=torch.int32, device=dev) if return_acc else None
    s = _stream(xq)
    if w_u8 is not None and M >= PREFILL_U8_MIN_M:
        _dev(w_u8, torch.uint8, "w_u8", 1)
        _need(w_u8.numel() >= int(_lib.load().fq_prefill_weight_bytes(N, K)) and w_u8.device == dev,
              "w_u8 must be prepare_prefill_weights(wpk, N, K) on the operands' device")
        _lib.call("fq_gemm_w6ax_u8", _ptr(xq), _ptr(xs), _ptr(wpk), _ptr(w_u8), M, N, K, abits, _ptr(out),
                  _ptr(acc), None, ctypes.c_size_t(0), s)
        return (out, acc) if return_acc else out
    nb = gemm_workspace_bytes(M, N, K)
    wbuf = workspace(dev, nb, s.value)
    _lib.call("fq_gemm_w6ax", _ptr(xq), _ptr(xs), _ptr(wpk), M, N, K, abits, _ptr(out),
              _ptr(acc), _ptr(wbuf), ctypes.c_size_t(wbuf.numel() if wbuf is not None else 0), s)
    return (out, acc) if return_acc else out


def gemm_q_workspace_bytes(M, N, K):
    """Workspace of gemm_w6ax_q's one-launch form (fq_gemm_q_workspace_bytes): the GEMM's own plus the
    epilogue quantizer's group tickets."""
    return int(_lib.load().fq_gemm_q_workspace_bytes(M, N, K))


def gemm_w6ax_q(xq, xs, wpk, N, abits, w_u8, q_shape, qbits, out=None):
    """gemm_w6ax that also returns the NEXT linear's quantized input: the fp16 output's leading qM * qK
    values read row-major as [qM, qK] and quantized to qbits -- bit-identical to
    quantize_act(out.view(-1)[:qM*qK].view(qM, qK), qbits).  Prefill sizes over prepared operands
    (w_u8, fq_gemm_w6ax_u8_q): in the 256 x 256 prefill kernel's epilogue; M <= 16 (w_u8 None,
    fq_gemm_w6ax_q): in the decode GEMM's epilogue, one launch.  Returns (out, qxq, qxs)."""
    _dev(xq, torch.int8, "xq", 2)
    M, K = xq.shape
    _k_ok(K)
    _dev(xs, torch.float16, "xs", 2)
    _need(tuple(xs.shape) == (K // GROUP, M), f"xs must be [K/128, M] = {(K // GROUP, M)}")
    _img_ok(wpk, N, K)
    _need(abits in (6, 8) and qbits in (6, 8), "abits and qbits must be 6 or 8")
    qM, qK = q_shape
    _k_ok(qK)
    _need(0 < qM * qK <= M * N, "the next input must be a prefix of the output")
    dev = xq.device
    if w_u8 is not None:
        _dev(w_u8, torch.uint8, "w_u8", 1)
        _need(w_u8.numel() >= int(_lib.load().fq_prefill_weight_bytes(N, K)) and w_u8.device == dev,
              "w_u8 must be prepare_prefill_weights(wpk, N, K) on the operands' device")
    if out is None:
        out = torch.empty((M, N), dtype=torch.float16, device=dev)
    else:
        _dev(out, torch.float16, "out", 2)
        _need(tuple(out.shape) == (M, N), "out shape mismatch")
    qxq = torch.empty((qM, qK), dtype=torch.int8, device=dev)
    qxs = torch.empty((qK // GROUP, qM), dtype=torch.float16, device=dev)
    s = _stream(xq)
    if w_u8 is not None:
        wbuf = workspace(dev, gemm_workspace_bytes(M, N, K), s.value)
        _lib.call("fq_gemm_w6ax_u8_q", _ptr(xq), _ptr(xs), _ptr(wpk), _ptr(w_u8), M, N, K, abits, _ptr(out),
                  _ptr(qxq), _ptr(qxs), qM, qK, qbits, _ptr(wbuf),
                  ctypes.c_size_t(wbuf.numel() if wbuf is not None else 0), s)
    else:
        wbuf = workspace(dev, gemm_q_workspace_bytes(M, N, K), s.value)
        _lib.call("fq_gemm_w6ax_q", _ptr(xq), _ptr(xs), _ptr(wpk), M, N, K, abits, _ptr(out), _ptr(qxq), _ptr(qxs),
                  qM, qK, qbits, _ptr(wbuf), ctypes.c_size_t(wbuf.numel() if wbuf is not None else 0), s)
    return out, qxq, qxs


def linear_w6ax(x, wpk, N, abits=6, out=None, w_u8=None):
    """Quantize + GEMM (FLEXQGEMMWrapper::gemm(const half* A ...)) for fp16 x [M,K].  w_u8: the
    prepared operands of prepare_prefill_weights (prefill sizes: quantize + fq_gemm_w6ax_u8)."""
    _dev(x, torch.float16, "x", 2)
    M, K = x.shape
    _k_ok(K)
    _img_ok(wpk, N, K)
    _need(wpk.device == x.device, "x and the weight image must be on one device")
    _need(abits in (6, 8), "abits must be 6 or 8")
    dev = x.device
    if out is None:
        out = torch.empty((M, N), dtype=torch.float16, device=dev)
    else:
        _dev(out, torch.float16, "out", 2)
        _need(tuple(out.shape) == (M, N), f"out must be [M, N] = {(M, N)}")
    if w_u8 is not None and M >= PREFILL_U8_MIN_M:
        xq, xs = quantize_act(x, abits)
        return gemm_w6ax(xq, xs, wpk, N, abits, out=out, w_u8=w_u8)
    xq = xs = None
    if act_scratch_bytes(M, N, K):  # prefill sizes quantize in a separate launch
        xq = torch.empty((M, K), dtype=torch.int8, device=dev)
        xs = torch.empty((K // GROUP, M), dtype=torch.float16, device=dev)
    s = _stream(x)
    nb = gemm_workspace_bytes(M, N, K)
    wbuf = workspace(dev, nb, s.value)
    _lib.call("fq_linear_w6ax", _ptr(x), M, N, K, abits, _ptr(wpk), _ptr(out), _ptr(xq),
              _ptr(xs), _ptr(wbuf), ctypes.c_size_t(wbuf.numel() if wbuf is not None else 0), s)
    return out


class _ChainLink(ctypes.Structure):  # fq_chain_link (include/flexq_hip.h)
    _fields_ = [("x", ctypes.c_void_p), ("w_packed", ctypes.c_void_p), ("d", ctypes.c_void_p),
                ("N", ctypes.c_int), ("K", ctypes.c_int), ("abits", ctypes.c_int), ("pro", ctypes.c_int),
                ("in_", ctypes.c_void_p), ("gamma", ctypes.c_void_p), ("res_out", ctypes.c_void_p),
                ("eps", ctypes.c_float), ("ldh", ctypes.c_int)]


def chain_rmsnorm(residual, gamma, wpk, N, abits, out, input=None, residual_out=None, eps=1e-6):
    """A chain link computed as rmsnorm_linear_w6ax(residual, gamma, wpk, N, abits, eps, input,
    residual_out, out) (residual_out required with input)."""
    return dict(kind="rmsnorm", x=residual, gamma=gamma, w=wpk, N=N, abits=abits, out=out, input=input,
                residual_out=residual_out, eps=eps)


def chain_silu(gate, up, wpk, N, abits, out):
    """A chain link computed as silu_linear_w6ax(gate, up, wpk, N, abits, out)."""
    return dict(kind="silu", x=gate, up=up, w=wpk, N=N, abits=abits, out=out)


def linear_chain_w6ax(links):
    """Consecutive decode linears (fq_linear_chain_w6ax), each computed exactly as its own call would be,
    in order: a tuple (x, wpk, N, abits, out) is linear_w6ax(x, wpk, N, abits, out=out); chain_rmsnorm(...)
    and chain_silu(...) are rmsnorm_linear_w6ax / silu_linear_w6ax.  An input may be a view of the previous
    link's out, and an RMSNorm link's residual an earlier RMSNorm link's residual_out (the chain's
    hand-offs).  Runs that can chain (M <= 4; RMSNorm at M = 1, K = 4096) are one
    persistent launch each.  Returns the list of outputs.  Raises _lib.ChainTimeoutError once an in-kernel
    wait on this stream's chain workspace has timed out (that launch's results are undefined), until
    chain_reset()."""
    _need(len(links) > 0, "empty chain")
    M, dev, scratch, Kmax = None, None, 0, 0
    arr = (_ChainLink * len(links))()
    outs = []
    for i, lk in enumerate(links):
        if isinstance(lk, dict):
            kind = lk["kind"]
            x, wpk, N, abits, out = lk["x"], lk["w"], lk["N"], lk["abits"], lk["out"]
        else:
            kind = "linear"
            x, wpk, N, abits, out = lk
        _need(isinstance(x, torch.Tensor) and x.is_cuda and x.dtype == torch.float16 and x.dim() == 2,
              "x must be a 2-D fp16 HIP tensor")
        m, K = x.shape
        _need(x.stride(1) == 1, "x rows must be contiguous")
        M = m if M is None else M
        dev = x.device if dev is None else dev
        _need(m == M, "every link has the same M")
        _k_ok(K)
        _img_ok(wpk, N, K)
        _need(abits in (6, 8), "abits must be 6 or 8")
        _dev(out, torch.float16, "out", 2)
        _need(tuple(out.shape) == (M, N), f"out must be [M, N] = {(M, N)}")
        _need(wpk.device == x.device == out.device == dev, "one device")
        c = _ChainLink(x=_ptr(x), w_packed=_ptr(wpk), d=_ptr(out), N=N, K=K, abits=abits, pro=0, eps=0.0, ldh=0)
        if kind == "linear":
            _need(M == 1 or x.stride(0) == K, "x must be a contiguous [M, K] row block")
            _need(not _overlap(out, x), "a link's output must not overlap its input")
            sb = act_scratch_bytes(M, N, K)
        elif kind == "rmsnorm":
            gamma, inp, ro = lk["gamma"], lk["input"], lk["residual_out"]
            _need(M == 1 or x.stride(0) == K, "the residual must be a contiguous [M, K] row block")
            _dev(gamma, torch.float16, "gamma", 1)
            _need(gamma.numel() == K and gamma.device == dev, "gamma must be [K] on the residual's device")
            if inp is not None:
                _dev(inp, torch.float16, "input", 2)
                _need(tuple(inp.shape) == (M, K) and (M == 1 or inp.stride(0) == K), "input must match residual")
                _dev(ro, torch.float16, "residual_out", 2)
                _need(tuple(ro.shape) == (M, K), "residual_out must match residual")
                for name, t in (("residual", x), ("input", inp), ("gamma", gamma)):
                    _need(not _overlap(ro, t), f"residual_out must not overlap {name}")
            c.pro, c.gamma, c.eps = 1, _ptr(gamma), float(lk["eps"])
            c.in_, c.res_out = _ptr(inp), _ptr(ro if inp is not None else None)
            sb = int(_lib.load().fq_rmsnorm_linear_scratch_bytes(M, N, K))
        elif kind == "silu":
            up = lk["up"]
            _need(isinstance(up, torch.Tensor) and up.is_cuda and up.dtype == torch.float16 and up.device == dev,
                  "up must be an fp16 HIP tensor on x's device")
            _need(up.shape == x.shape and up.stride(0) == x.stride(0) and up.stride(1) == 1,
                  "gate and up must have one shape and row stride")
            c.pro, c.in_, c.ldh = 2, _ptr(up), (x.stride(0) if M > 1 else K)
            sb = int(_lib.load().fq_silu_linear_scratch_bytes(M, N, K))
        else:
            raise ValueError(f"unknown chain link kind {kind!r}")
        arr[i] = c
        scratch, Kmax = max(scratch, sb), max(Kmax, K)
        outs.append(out)
    xq = xs = None
    if scratch:
        xq = torch.empty((M, Kmax), dtype=torch.int8, device=dev)
        xs = torch.empty((Kmax // GROUP, M), dtype=torch.float16, device=dev)
    x0 = links[0]["x"] if isinstance(links[0], dict) else links[0][0]
    s = _stream(x0)
    cb = int(_lib.load().fq_chain_workspace_bytes(ctypes.cast(arr, ctypes.c_void_p), len(links), M))
    cbuf = chain_workspace(dev, cb, s.value)
    nb = max(gemm_workspace_bytes(M, c.N, c.K) for c in arr)
    wbuf = workspace(dev, nb, s.value)
    _lib.call("fq_linear_chain_w6ax", ctypes.cast(arr, ctypes.c_void_p), len(links), M, _ptr(cbuf),
              ctypes.c_size_t(cbuf.numel()), _ptr(xq), _ptr(xs), _ptr(wbuf),
              ctypes.c_size_t(wbuf.numel() if wbuf is not None else 0), s)
    return outs


def chain_workspace_buffer(device=None, stream=None):
    """The stream's chain workspace (None before its first chain call)."""
    dev = torch.device(device if device is not None else "cuda")
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    return _CWS.get((dev, ctypes.c_void_p(s.cuda_stream).value))  # (the key _stream() makes)


def chain_error(device=None, stream=None):
    """The decode chain's sticky error word in the stream's chain workspace (0: every in-kernel wait
    ended in time; 1: one timed out and the results since are undefined).  Reads device memory (a
    synchronising copy); chain_status() reads the host-visible copy instead."""
    buf = chain_workspace_buffer(device, stream)
    if buf is None:
        return 0
    off = int(_lib.load().fq_chain_error_offset())
    return int(buf[off:off + 4].view(torch.int32).item())


def chain_status(device=None, stream=None):
    """True while the stream's chain workspace is in the timed-out state (fq_chain_status: the pinned host
    word the kernel sets; no synchronisation, so it shows once the launch that timed out has finished).
    linear_chain_w6ax then raises ChainTimeoutError until chain_reset()."""
    buf = chain_workspace_buffer(device, stream)
    return buf is not None and int(_lib.load().fq_chain_status(_ptr(buf))) != _lib.FQ_OK


def chain_reset(device=None, stream=None):
    """Clear a timed-out chain workspace (fq_chain_reset): re-zeroed on the stream, its host word cleared.
    Synchronises the stream first (no chain launch may be in flight)."""
    dev = torch.device(device if device is not None else "cuda")
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    buf = chain_workspace_buffer(dev, s)
    if buf is None:
        return
    s.synchronize()
    _lib.call("fq_chain_reset", _ptr(buf), ctypes.c_size_t(buf.numel()), ctypes.c_void_p(s.cuda_stream))


def act_scratch_bytes(M, N, K):
    """Activation scratch fq_linear_w6ax needs (0: decode sizes run as one fused launch)."""
    return int(_lib.load().fq_linear_act_scratch_bytes(M, N, K))


# ------------------------------------------------------------------------- fused producers

def rmsnorm_quantize(residual, gamma, abits, eps=1e-6, input=None, return_normed=False):
    """Residual add + RMSNorm + dynamic group quantization (fq_rmsnorm_quantize; the reference's
    generalAddResidualT5LayerNormFlexQFusion, layernorm_kernels.cu:1851-2051).  residual fp16
    [M,K] is updated IN PLACE to residual + input when input is given.  Returns (xq int8 [M,K],
    xs fp16 [K/128, M]) (+ the fp16 normalised activations)."""
    _dev(residual, torch.float16, "residual", 2)
    M, K = residual.shape
    _k_ok(K)
    _need(K <= 32768, "K must be <= 32768")
    _dev(gamma, torch.float16, "gamma", 1)
    _need(gamma.numel() == K and gamma.device == residual.device, "gamma must be [K] on the residual's device")
    if input is not None:
        _dev(input, torch.float16, "input", 2)
        _need(tuple(input.shape) == (M, K) and input.device == residual.device, "input must match residual")
    _need(abits in (6, 8), "abits must be 6 or 8")
    dev = residual.device
    xq = torch.empty((M, K), dtype=torch.int8, device=dev)
    xs = torch.empty((K // GROUP, M), dtype=torch.float16, device=dev)
    normed = torch.empty((M, K), dtype=torch.float16, device=dev) if return_normed else None
    _lib.call("fq_rmsnorm_quantize", _ptr(input), _ptr(residual), _ptr(gamma), ctypes.c_float(eps), M, K, abits,
              _ptr(xq), _ptr(xs), _ptr(normed), _stream(residual))
    return (xq, xs, normed) if return_normed else (xq, xs)


def silu_mul_quantize(gate, up, abits, return_act=False):
    """SiLU(gate) * up + dynamic group quantization (fq_silu_mul_quantize; the reference's
    flexq_generic_activation, activation_kernels.cu:245-450).  gate and up are fp16 [M,N] views
    with a contiguous last dimension and one common row stride (e.g. the two column halves of a
    merged gate_up output).  Returns (xq int8 [M,N], xs fp16 [N/128, M]) (+ the fp16 product)."""
    for name, t in (("gate", gate), ("up", up)):
        _need(isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float16 and t.dim() == 2,
              f"{name} must be a 2-D fp16 HIP tensor")
        _need(t.stride(1) == 1, f"{name} rows must be contiguous")
    _need(gate.shape == up.shape and gate.stride(0) == up.stride(0) and gate.device == up.device,
          "gate and up must have one shape, row stride and device")
    M, N = gate.shape
    _k_ok(N)
    _need(abits in (6, 8), "abits must be 6 or 8")
    ld = gate.stride(0) if M > 1 else N
    dev = gate.device
    xq = torch.empty((M, N), dtype=torch.int8, device=dev)
    xs = torch.empty((N // GROUP, M), dtype=torch.float16, device=dev)
    act = torch.empty((M, N), dtype=torch.float16, device=dev) if return_act else None
    _lib.call("fq_silu_mul_quantize", _ptr(gate), _ptr(up), ld, M, N, abits, _ptr(xq), _ptr(xs), _ptr(act),
              _stream(gate))
    return (xq, xs, act) if return_act else (xq, xs)


def _vec_ok(t, name, K, dev):
    if t is not None:
        _dev(t, torch.float16, name, 1)
        _need(t.numel() == K and t.device == dev, f"{name} must be [K] on the residual's device")


def _span(t):
    return (t.data_ptr(), t.data_ptr() + t.numel() * t.element_size()) if t is not None else None


def _overlap(a, b):
    a, b = _span(a), _span(b)
    return a is not None and b is not None and a[0] < b[1] and b[0] < a[1]


def layernorm_quantize(residual, gamma, abits, beta=None, eps=1e-5, input=None, bias=None, residual_out=None,
                       return_normed=False):
    """Residual [+ input] [+ bias] + LayerNorm (gamma, beta) + dynamic group quantization
    (fq_layernorm_quantize; the reference's OPT-family generalAddBiasResidualLayerNormOpt2FlexQFusion,
    layernorm_kernels.cu:316-575, and its pre-attention form, :2325-2420).  residual_out (fp16 [M,K],
    may be the residual itself) receives half(residual + input + bias) when given.  Returns (xq int8
    [M,K], xs fp16 [K/128, M]) (+ the fp16 normalised activations)."""
    _dev(residual, torch.float16, "residual", 2)
    M, K = residual.shape
    _k_ok(K)
    _need(K <= 32768, "K must be <= 32768")
    dev = residual.device
    _vec_ok(gamma, "gamma", K, dev)
    _need(gamma is not None, "gamma is required")
    _vec_ok(beta, "beta", K, dev)
    _vec_ok(bias, "bias", K, dev)
    if input is not None:
        _dev(input, torch.float16, "input", 2)
        _need(tuple(input.shape) == (M, K) and input.device == dev, "input must match residual")
    if residual_out is not None:
        _dev(residual_out, torch.float16, "residual_out", 2)
        _need(tuple(residual_out.shape) == (M, K) and residual_out.device == dev, "residual_out must match residual")
        for name, t in (("input", input), ("bias", bias), ("gamma", gamma), ("beta", beta)):
            _need(not _overlap(residual_out, t), f"residual_out must not overlap {name}")
        _need(residual_out.data_ptr() == residual.data_ptr() or not _overlap(residual_out, residual),
              "residual_out must be the residual or not overlap it")
    _need(abits in (6, 8), "abits must be 6 or 8")
    xq = torch.empty((M, K), dtype=torch.int8, device=dev)
    xs = torch.empty((K // GROUP, M), dtype=torch.float16, device=dev)
    normed = torch.empty((M, K), dtype=torch.float16, device=dev) if return_normed else None
    _lib.call("fq_layernorm_quantize", _ptr(input), _ptr(residual), _ptr(bias), _ptr(residual_out), _ptr(gamma),
              _ptr(beta), ctypes.c_float(eps), M, K, abits, _ptr(xq), _ptr(xs), _ptr(normed), _stream(residual))
    return (xq, xs, normed) if return_normed else (xq, xs)


def _act_scratch(fn, M, N, K, dev):
    if not int(getattr(_lib.load(), fn)(M, N, K)):
        return None, None  # the producer runs inside the decode GEMM: no activation scratch
    return (torch.empty((M, K), dtype=torch.int8, device=dev),
            torch.empty((K // GROUP, M), dtype=torch.float16, device=dev))


def _out_ok(out, M, N, dev):
    if out is None:
        return torch.empty((M, N), dtype=torch.float16, device=dev)
    _dev(out, torch.float16, "out", 2)
    _need(tuple(out.shape) == (M, N) and out.device == dev, f"out must be [M, N] = {(M, N)} on {dev}")
    return out


def rmsnorm_linear_w6ax(residual, gamma, wpk, N, abits=6, eps=1e-6, input=None, residual_out=None, out=None):
    """Residual add + RMSNorm + quantize + W6Ax GEMM (fq_rmsnorm_linear_w6ax): one launch at
    decode sizes (M = 1, K = 4096), else fq_rmsnorm_quantize + GEMM -- the same bits either way.
    With input, residual + input is written to residual_out (allocated when None; never the
    residual itself).  Returns (d fp16 [M, N], the updated residual: residual_out, or residual
    when input is None)."""
    _dev(residual, torch.float16, "residual", 2)
    M, K = residual.shape
    _k_ok(K)
    dev = residual.device
    _dev(gamma, torch.float16, "gamma", 1)
    _need(gamma.numel() == K and gamma.device == dev, "gamma must be [K] on the residual's device")
    _img_ok(wpk, N, K)
    _need(wpk.device == dev, "the weight image must be on the residual's device")
    _need(abits in (6, 8), "abits must be 6 or 8")
    if input is not None:
        _dev(input, torch.float16, "input", 2)
        _need(tuple(input.shape) == (M, K) and input.device == dev, "input must match residual")
        if residual_out is None:
            residual_out = torch.empty_like(residual)
        _dev(residual_out, torch.float16, "residual_out", 2)
        _need(tuple(residual_out.shape) == (M, K) and residual_out.device == dev, "residual_out must match residual")
        for name, t in (("residual", residual), ("input", input), ("gamma", gamma)):
            _need(not _overlap(residual_out, t), f"residual_out must not overlap {name}")
    else:
        residual_out = None
    out = _out_ok(out, M, N, dev)
    xq, xs = _act_scratch("fq_rmsnorm_linear_scratch_bytes", M, N, K, dev)
    s = _stream(residual)
    wbuf = workspace(dev, gemm_workspace_bytes(M, N, K), s.value)
    _lib.call("fq_rmsnorm_linear_w6ax", _ptr(input), _ptr(residual), _ptr(residual_out), _ptr(gamma),
              ctypes.c_float(eps), M, N, K, abits, _ptr(wpk), _ptr(out), _ptr(xq), _ptr(xs), _ptr(wbuf),
              ctypes.c_size_t(wbuf.numel() if wbuf is not None else 0), s)
    return out, (residual_out if input is not None else residual)


def layernorm_linear_w6ax(residual, gamma, wpk, N, abits=6, beta=None, eps=1e-5, input=None, bias=None,
                          residual_out=None, out=None):
    """Residual [+ input] [+ bias] + LayerNorm + quantize + W6Ax GEMM (fq_layernorm_linear_w6ax; the OPT
    decoder's LayerNorm -> qkv / fc1 pair): one launch at decode sizes (M = 1, K = 4096), else
    fq_layernorm_quantize + GEMM -- the same bits either way.  residual_out (optional; allocated when
    input or bias is given and it is None) receives half(residual + input + bias); it must not
    overlap the residual or any other input.  Returns (d fp16 [M, N], residual_out or None)."""
    _dev(residual, torch.float16, "residual", 2)
    M, K = residual.shape
    _k_ok(K)
    dev = residual.device
    _vec_ok(gamma, "gamma", K, dev)
    _need(gamma is not None, "gamma is required")
    _vec_ok(beta, "beta", K, dev)
    _vec_ok(bias, "bias", K, dev)
    _img_ok(wpk, N, K)
    _need(wpk.device == dev, "the weight image must be on the residual's device")
    _need(abits in (6, 8), "abits must be 6 or 8")
    if input is not None:
        _dev(input, torch.float16, "input", 2)
        _need(tuple(input.shape) == (M, K) and input.device == dev, "input must match residual")
    if residual_out is None and (input is not None or bias is not None):
        residual_out = torch.empty_like(residual)
    if residual_out is not None:
        _dev(residual_out, torch.float16, "residual_out", 2)
        _need(tuple(residual_out.shape) == (M, K) and residual_out.device == dev, "residual_out must match residual")
        for name, t in (("residual", residual), ("input", input), ("bias", bias), ("gamma", gamma), ("beta", beta)):
            _need(not _overlap(residual_out, t), f"residual_out must not overlap {name}")
    out = _out_ok(out, M, N, dev)
    xq, xs = _act_scratch("fq_layernorm_linear_scratch_bytes", M, N, K, dev)
    s = _stream(residual)
    wbuf = workspace(dev, gemm_workspace_bytes(M, N, K), s.value)
    _lib.call("fq_layernorm_linear_w6ax", _ptr(input), _ptr(residual), _ptr(bias), _ptr(residual_out), _ptr(gamma),
              _ptr(beta), ctypes.c_float(eps), M, N, K, abits, _ptr(wpk), _ptr(out), _ptr(xq), _ptr(xs), _ptr(wbuf),
              ctypes.c_size_t(wbuf.numel() if wbuf is not None else 0), s)
    return out, residual_out


def silu_linear_w6ax(gate, up, wpk, N, abits=8, out=None):
    """SiLU(gate) * up + quantize + W6Ax GEMM (fq_silu_linear_w6ax; down_proj after gate_up): one
    launch at decode sizes, else fq_silu_mul_quantize + GEMM -- the same bits either way.  gate
    and up as for silu_mul_quantize (e.g. the halves of a merged gate_up output)."""
    for name, t in (("gate", gate), ("up", up)):
        _need(isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float16 and t.dim() == 2,
              f"{name} must be a 2-D fp16 HIP tensor")
        _need(t.stride(1) == 1, f"{name} rows must be contiguous")
    _need(gate.shape == up.shape and gate.stride(0) == up.stride(0) and gate.device == up.device,
          "gate and up must have one shape, row stride and device")
    M, K = gate.shape
    _k_ok(K)
    dev = gate.device
    _img_ok(wpk, N, K)
    _need(wpk.device == dev, "the weight image must be on the activations' device")
    _need(abits in (6, 8), "abits must be 6 or 8")
    ld = gate.stride(0) if M > 1 else K
    out = _out_ok(out, M, N, dev)
    xq, xs = _act_scratch("fq_silu_linear_scratch_bytes", M, N, K, dev)
    s = _stream(gate)
    wbuf = workspace(dev, gemm_workspace_bytes(M, N, K), s.value)
    _lib.call("fq_silu_linear_w6ax", _ptr(gate), _ptr(up), ld, M, N, K, abits, _ptr(wpk), _ptr(out), _ptr(xq),
              _ptr(xs), _ptr(wbuf), ctypes.c_size_t(wbuf.numel() if wbuf is not None else 0), s)
    return out


# ------------------------------------------------------------------------- reference layouts

def _rows_ok(R):
    _need(R > 0 and (R <= 8 or R % 8 == 0), f"rows={R}: the reference bit-plane layout needs <= 8 or a multiple of 8")


def ref_bit_packing(vals, bits):
    """flexq_bit_packing(const int*...): int32 raw b-bit patterns [R,K] -> bit planes."""
    _dev(vals, torch.int32, "vals", 2)
    R, K = vals.shape
    _k_ok(K)
    _rows_ok(R)
    out = torch.empty(bits * R * (K // 32), dtype=torch.int32, device=vals.device)
    _lib.call("fq_ref_bit_packing", _ptr(vals), _ptr(out), R, K, bits, _stream(vals))
    return out


def ref_quantize_bit_packing(x, bits):
    """e2e flexq_bit_packing(const half*...): fp16 [M,K] -> (bit planes, x_scale_dup)."""
    _dev(x, torch.float16, "x", 2)
    M, K = x.shape
    _k_ok(K)
    _rows_ok(M)
    _need(bits in (6, 8), "bits must be 6 or 8")
    planes = torch.empty(bits * M * (K // 32), dtype=torch.int32, device=x.device)
    ld = 2 * ((M + 3) // 4 * 4)
    dup = torch.zeros((K // GROUP, ld), dtype=torch.float16, device=x.device)
    _lib.call("fq_ref_quantize_bit_packing", _ptr(x), _ptr(planes), _ptr(dup), M, K, bits, _stream(x))
    return planes, dup


def import_ref_w(planes, ws, N, K):
    """Reference bit-plane weights + W_SCALE [K/128, N] -> weight image."""
    _dev(planes, torch.int32, "planes", 1)
    _k_ok(K)
    _rows_ok(N)
    _need(planes.numel() == 6 * N * (K // 32), "planes size does not match 6-bit [N,K]")
    _ws_ok(ws, N, K, planes.device)
    out = torch.empty(packed_w_bytes(N, K), dtype=torch.uint8, device=planes.device)
    _lib.call("fq_import_ref_w", _ptr(planes), _ptr(ws), N, K, _ptr(out), _stream(planes))
    return out


def gemm_w6ax_planes(planes, dup, wpk, M, N, K, bits, out=None):
    """GEMM straight from the reference's bit-plane activations + duplicated x-scales (the X /
    X_SCALE of FQBMMAExecFn_t, FLEXQGEMMWrapper::gemm(const int* A ...)): one launch at decode
    sizes (the planes unpacked in the GEMM prologue), import + GEMM otherwise."""
    _dev(planes, torch.int32, "planes", 1)
    _dev(dup, torch.float16, "x_scale_dup", 2)
    _k_ok(K)
    _rows_ok(M)
    _need(bits in (6, 8), "bits must be 6 or 8")
    _need(planes.numel() == bits * M * (K // 32), "planes size does not match [M,K]")
    _need(tuple(dup.shape) == (K // GROUP, 2 * ((M + 3) // 4 * 4)), "x_scale_dup must be [K/128, 2*ceil4(M)]")
    _img_ok(wpk, N, K)
    dev = planes.device
    for t in (dup, wpk):
        _need(t.device == dev, "all operands must be on one device")
    if out is None:
        out = torch.empty((M, N), dtype=torch.float16, device=dev)
    else:
        _dev(out, torch.float16, "out", 2)
        _need(tuple(out.shape) == (M, N), "out shape mismatch")
    xq = xs = None
    if int(_lib.load().fq_planes_act_scratch_bytes(M, N, K)):
        xq = torch.empty((M, K), dtype=torch.int8, device=dev)
        xs = torch.empty((K // GROUP, M), dtype=torch.float16, device=dev)
    s = _stream(planes)
    wbuf = workspace(dev, gemm_workspace_bytes(M, N, K), s.value)
    _lib.call("fq_gemm_w6ax_planes", _ptr(planes), _ptr(dup), _ptr(wpk), M, N, K, bits, _ptr(out), _ptr(xq),
              _ptr(xs), _ptr(wbuf), ctypes.c_size_t(wbuf.numel() if wbuf is not None else 0), s)
    return out


def import_ref_x(planes, dup, M, K, bits):
    _dev(planes, torch.int32, "planes", 1)
    _dev(dup, torch.float16, "x_scale_dup", 2)
    _k_ok(K)
    _rows_ok(M)
    _need(planes.numel() == bits * M * (K // 32), "planes size does not match [M,K]")
    xq = torch.empty((M, K), dtype=torch.int8, device=planes.device)
    xs = torch.empty((K // GROUP, M), dtype=torch.float16, device=planes.device)
    _lib.call("fq_import_ref_x", _ptr(planes), _ptr(dup), M, K, bits, _ptr(xq), _ptr(xs), _stream(planes))
    return xq, xs
