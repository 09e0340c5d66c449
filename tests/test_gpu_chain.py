"""The decode chain (fq_linear_chain_w6ax): consecutive dependent linears in one persistent launch,
each waiting in the kernel for the previous linear's output.  Every output must be bit-identical to
running the same linears one fq_linear_w6ax launch at a time, over chains of a LLaMA-2-7B layer
(o -> gate_up -> down (A8) -> next qkv, each input the leading M*K values of the previous output, as
bench.py's step), uneven per-link load (LLaMA-2-70B shapes beside 7B ones), runs split at 8 links,
links that cannot chain (k-split shapes, M > 4) interleaved, repeated launches and graph replays (the
hand-off tags advance with the epoch, the start counter returns to zero, the wrap of the tag clears
the hand-off region), and the error word stays 0 throughout."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops(dev):
    from flexq_amd import ops as _ops
    return _ops


def image(ops, N, K, g, dev):
    wq = torch.randint(-32, 32, (N, K), dtype=torch.int8, device=dev, generator=g)
    ws = ((torch.rand((K // 128, N), device=dev, generator=g) + 0.5) / (18.5 * 1.04 * K ** 0.5)).half()
    return ops.pack_w6(wq, ws)


LAYER_7B = [(4096, 4096, 6), (22016, 4096, 6), (4096, 11008, 8), (12288, 4096, 6)]


def build(ops, dev, M, shapes, seed=5):
    """links [(x, wpk, N, abits, out)] where x of link l is the leading M*K of link l-1's output."""
    g = torch.Generator(device=dev).manual_seed(seed)
    x0 = torch.randn((M, shapes[0][1]), dtype=torch.float16, device=dev, generator=g)
    links, prev = [], x0
    for (N, K, abits) in shapes:
        x = prev.view(-1)[:M * K].view(M, K) if prev is not x0 else x0
        out = torch.full((M, N), float("nan"), dtype=torch.float16, device=dev)
        links.append((x, image(ops, N, K, g, dev), N, abits, out))
        prev = out
    return links


def sequential(ops, links, dev):
    """The same linears one launch at a time, into fresh buffers (inputs re-pointed at them)."""
    outs, prev_src, prev_dst = [], None, None
    for (x, wpk, N, abits, out) in links:
        M, K = x.shape
        if prev_src is not None and x.data_ptr() >= prev_src.data_ptr() and \
                x.data_ptr() < prev_src.data_ptr() + prev_src.numel() * 2:
            off = (x.data_ptr() - prev_src.data_ptr()) // 2
            xs = prev_dst.view(-1)[off:off + M * K].view(M, K)
        else:
            xs = x
        y = ops.linear_w6ax(xs, wpk, N, abits)
        outs.append(y)
        prev_src, prev_dst = out, y
    torch.cuda.synchronize()
    return outs


def check(ops, links, dev, what):
    ref = sequential(ops, links, dev)
    for i, ((*_, out), r) in enumerate(zip(links, ref)):
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint16), r.cpu().numpy().view(np.uint16),
                                      err_msg=f"{what}: link {i}")
    assert ops.chain_error(dev) == 0, f"{what}: a chain wait timed out"


@pytest.mark.parametrize("M", [1, 2, 4])
def test_chain_layer_bit_identical(ops, dev, M):
    links = build(ops, dev, M, LAYER_7B + LAYER_7B[:3])  # two layers' worth: 7 links, one launch
    for rep in range(3):  # repeated launches: the counters are zero again after each
        for (*_, out) in links:
            out.fill_(float("nan"))
        ops.linear_chain_w6ax(links)
        torch.cuda.synchronize()
        check(ops, links, dev, f"M={M} rep {rep}")


def test_chain_uneven_links_and_run_split(ops, dev):
    """70B gate_up (7 tiles per CU) beside 1-tile links, 11 links: runs of 8 and 3."""
    shapes = [(28672, 8192, 6), (8192, 28672, 8), (4096, 8192, 6), (8192, 4096, 6), (57344, 8192, 6),
              (8192, 28672, 8), (4096, 8192, 6), (12288, 4096, 6), (4096, 4096, 6), (22016, 4096, 6),
              (4096, 11008, 8)]
    links = build(ops, dev, 1, shapes, seed=9)
    ops.linear_chain_w6ax(links)
    torch.cuda.synchronize()
    check(ops, links, dev, "uneven")


def test_chain_with_unchainable_links(ops, dev):
    """Links whose plan is not one S = 1 tile set over the chip (N = 1024: k-split; N = 2000 not a
    multiple of 16) run as plain linears between chained runs; same bits."""
    shapes = [(4096, 4096, 6), (1024, 4096, 6), (4096, 1024, 8), (12288, 4096, 6), (2000, 4096, 6),
              (4096, 1024, 6), (11008, 4096, 6), (4096, 11008, 8)]
    links = build(ops, dev, 1, shapes, seed=3)
    ops.linear_chain_w6ax(links)
    torch.cuda.synchronize()
    check(ops, links, dev, "mixed")


def test_chain_m16_falls_back(ops, dev):
    """M > 4: every link runs as fq_linear_w6ax (quantize launches included); same bits."""
    links = build(ops, dev, 16, LAYER_7B, seed=4)
    ops.linear_chain_w6ax(links)
    torch.cuda.synchronize()
    check(ops, links, dev, "M=16")


def test_chain_graph_replay(ops, dev):
    links = build(ops, dev, 1, LAYER_7B * 2, seed=6)
    s = torch.cuda.Stream(dev)
    ops.reserve_workspace(dev, [(1, 22016, 4096)], stream=s)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        ops.linear_chain_w6ax(links)  # warm-up on the capture stream
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        ops.linear_chain_w6ax(links)
    for rep in range(5):
        for (*_, out) in links:
            out.fill_(float("nan"))
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            g.replay()
        s.synchronize()
        ref = sequential(ops, links, dev)
        for i, ((*_, out), r) in enumerate(zip(links, ref)):
            np.testing.assert_array_equal(out.cpu().numpy().view(np.uint16), r.cpu().numpy().view(np.uint16),
                                          err_msg=f"replay {rep} link {i}")
    assert ops.chain_error(dev, stream=s) == 0


def test_chain_rejections(ops, dev):
    links = build(ops, dev, 1, LAYER_7B[:2], seed=2)
    x, wpk, N, abits, out = links[0]
    with pytest.raises(ValueError):
        ops.linear_chain_w6ax([(x, wpk, N, abits, x.view(-1)[:N].view(1, N))])  # output over its input
    with pytest.raises(ValueError):
        ops.linear_chain_w6ax([links[0], (torch.zeros((2, 4096), dtype=torch.float16, device=dev),) + links[1][1:]])


def test_chain_sync_words_and_epoch_wrap(ops, dev):
    """After every chain launch the start counter is zero and the epoch has advanced by one; the
    launch whose tag is 2^31 - 1 clears the hand-off granules and the epoch (tags never repeat, never
    carry the poison bit 31)."""
    links = build(ops, dev, 1, LAYER_7B, seed=8)
    ops.linear_chain_w6ax(links)
    torch.cuda.synchronize()
    buf = ops.chain_workspace_buffer(dev)
    words = buf[:4096].view(torch.int32)  # sync words 128 B apart: 0..7 start counter, 8 epoch, 9 error
    e0 = int(words[8 * 32].item())
    assert e0 >= 1 and all(int(words[32 * s].item()) == 0 for s in range(8))
    ops.linear_chain_w6ax(links)
    torch.cuda.synchronize()
    assert int(words[8 * 32].item()) == e0 + 1
    words[8 * 32] = 0x7ffffffe  # the next launch's tag is 2^31 - 1 (bit 31 marks poisoned granules)
    for rep, want in ((0, 0), (1, 1), (2, 2)):
        for (*_, out) in links:
            out.fill_(float("nan"))
        ops.linear_chain_w6ax(links)
        torch.cuda.synchronize()
        check(ops, links, dev, f"wrap rep {rep}")
        assert int(words[8 * 32].item()) == want
        assert all(int(words[32 * s].item()) == 0 for s in range(8)) and int(words[10 * 32].item()) == 0
    tags = buf[4096:].view(torch.int32)[1::2]  # every granule's tag word
    assert bool(((tags >= 0) & (tags <= 2)).all().item())  # no tag older than the wrap survives


def test_chain_error_word_fails_fast_and_recovers(ops, dev):
    """With the chain workspace's error word set (a wait timed out earlier) every in-kernel wait
    returns at once -- the chain finishes fast, results undefined, never a hang; cleared, the chain
    computes the right bits again."""
    import time
    links = build(ops, dev, 1, LAYER_7B * 2, seed=12)
    ops.linear_chain_w6ax(links)
    torch.cuda.synchronize()
    buf = ops.chain_workspace_buffer(dev)
    words = buf[:4096].view(torch.int32)
    words[9 * 32] = 1
    t0 = time.time()
    for _ in range(3):
        for (*_, out) in links:
            out.zero_()
        ops.linear_chain_w6ax(links)
    torch.cuda.synchronize()
    assert time.time() - t0 < 5.0
    assert ops.chain_error(dev) == 1
    assert_failed_outputs_nan(ops, links, dev, "error word set")
    words[9 * 32] = 0
    for (*_, out) in links:
        out.fill_(float("nan"))
    ops.linear_chain_w6ax(links)
    torch.cuda.synchronize()
    check(ops, links, dev, "after clearing the error word")


def assert_failed_outputs_nan(ops, links, dev, what):
    """After a failed chain launch: every link that waited for a previous link's
    output wrote fp16 NaN over its whole output; a run's first link (its input ready before the launch)
    waited for nothing and holds its right bits."""
    ref = sequential(ops, links, dev)
    for i, ((x, _, _, _, out), r) in enumerate(zip(links, ref)):
        prev = links[i - 1][4] if i else None
        waited = prev is not None and prev.data_ptr() <= x.data_ptr() < prev.data_ptr() + prev.numel() * 2
        o = out.cpu()
        if waited:
            assert bool(torch.isnan(o).all()), f"{what}: link {i} has {int((~torch.isnan(o)).sum())} non-NaN outputs"
        else:
            np.testing.assert_array_equal(o.numpy().view(np.uint16), r.cpu().numpy().view(np.uint16),
                                          err_msg=f"{what}: link {i} (ready input)")


def test_headline_step_pinned_to_the_oracle(ops, dev):
    """The headline step itself (bench.py's LLaMA-2-7B M = 1 stack as bench.chain_runs builds it, two layers:
    qkv_0 | o_0, gate_up_0, down_0, qkv_1 | o_1, gate_up_1, down_1) against the CPU oracle directly, link by
    link: each link's actual input (the chain's own previous output) quantized by the
    oracle is bit-identical to the engine's codes and scales; the oracle's int32 group accumulators over the
    link's weight image (unpacked by the oracle) equal the debug kernel's bit for bit
    (engine/test_bgemm_kernel.cu:113-146's check); the chain's fp16 output equals that debug launch's bit for
    bit, lies within oracle.gemm_tolerance of the oracle's, and equals bit for bit the oracle's restatement
    of the decode kernel's own fp32 summation order (oracle.gemm_decode_order)."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from common import assert_gemm_close, oracle
    cfg = (2, 1, bench.CONFIGS["llama2-7b-m1"][2], "two LLaMA-2-7B layers")
    stack = bench.build_stack(cfg, 0, 1, dev, merge=True, seed=77)
    runs = bench.chain_runs(stack)
    assert [len(r) for r in runs] == [1, 4, 3]
    bench.run_chains(runs)
    torch.cuda.synchronize()
    assert ops.chain_error(dev) == 0
    for i, (x, pk, N, abits, out) in enumerate(link for r in runs for link in r):
        K = x.shape[1]
        q, s = oracle.quantize_engine(x.cpu().numpy(), abits)
        xq, xs = ops.quantize_act(x.contiguous(), abits)
        np.testing.assert_array_equal(xq.cpu().numpy(), q, err_msg=f"link {i}: activation codes")
        np.testing.assert_array_equal(xs.cpu().numpy().view(np.uint16), s.view(np.uint16), err_msg=f"link {i}: scales")
        wq, ws = oracle.unpack_fq6(pk.cpu().numpy(), N, K, want_ws=True)
        ref, acc_ref, mag = oracle.gemm(q, s, wq, ws, want_acc=True)
        d_dbg, acc = ops.gemm_w6ax(xq, xs, pk, N, abits, return_acc=True)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(acc.cpu().numpy(), acc_ref, err_msg=f"link {i}: int32 group accumulators")
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint16), d_dbg.cpu().numpy().view(np.uint16),
                                      err_msg=f"link {i}: chain output vs the debug launch")
        assert_gemm_close(out.cpu().numpy(), ref, mag, f"headline link {i} ({N}x{K})")
        # and directly: the chain's own fp16 output bit for bit against the oracle's restatement of the
        # decode kernel's fp32 summation order (8 waves, S = 1)
        exact = oracle.gemm_decode_order(q, s, wq, ws, nw=8)
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint16), exact.view(np.uint16),
                                      err_msg=f"link {i}: chain output vs the oracle's decode-order sum")


def test_chain_host_status_raises_until_reset(ops, dev):
    """A set host status word (what a timed-out wait leaves) makes the next linear_chain_w6ax raise
    ChainTimeoutError without launching; chain_reset clears the workspace and the word, and the chain
    computes the right bits again."""
    from flexq_amd import _lib
    links = build(ops, dev, 1, LAYER_7B * 2, seed=13)
    ops.linear_chain_w6ax(links)
    torch.cuda.synchronize()
    assert not ops.chain_status(dev)
    buf = ops.chain_workspace_buffer(dev)
    ops._CWS_STATUS[buf.data_ptr()][0] = 1  # as chain_fail's system-scope store would
    with pytest.raises(_lib.ChainTimeoutError):
        ops.linear_chain_w6ax(links)
    ops.chain_reset(dev)
    assert not ops.chain_status(dev) and ops.chain_error(dev) == 0
    for (*_, out) in links:
        out.fill_(float("nan"))
    ops.linear_chain_w6ax(links)
    torch.cuda.synchronize()
    check(ops, links, dev, "after chain_reset")


def test_chain_not_coresident_times_out_and_recovers(ops, dev):
    """The co-residency failure: a kernel on another stream holds half of the CUs for 6 s
    while a chain launches, so half of the chain's workgroups cannot start.  (The blocker must outlast
    every resident wave's bounded wait, 2^20 polls = 1-2.5 s: a wave still polling when the blocker ends
    sees the late workgroups' outputs arrive and computes the right values instead of NaN.)  The resident ones' waits end
    after ~1 s with the error word set (never a hang); the kernel itself writes the bound host word and NaN
    over every output that depended on the failed waits, the next call raises ChainTimeoutError, and after
    chain_reset the chain is bit-exact again."""
    import ctypes
    import os
    import time
    from flexq_amd import _lib
    so = os.path.join(os.path.dirname(__file__), "cpp", "libcu_blocker.so")
    if not os.path.exists(so):
        pytest.skip("tests/cpp/libcu_blocker.so not built (__graft_entry__.build())")
    blk = ctypes.CDLL(so)
    blk.fq_test_cu_blocker.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    links = build(ops, dev, 1, LAYER_7B * 2, seed=14)
    ops.linear_chain_w6ax(links)  # the workspace exists and is bound
    torch.cuda.synchronize()
    for (*_, out) in links:
        out.zero_()
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    sink = torch.zeros(cus, dtype=torch.int32, device=dev)
    side = torch.cuda.Stream(dev)
    assert blk.fq_test_cu_blocker(cus // 2, 6000, ctypes.c_void_p(sink.data_ptr()),
                                  ctypes.c_void_p(side.cuda_stream)) == 0
    time.sleep(0.2)  # the blocker is resident
    t0 = time.time()
    ops.linear_chain_w6ax(links)
    torch.cuda.synchronize()
    assert time.time() - t0 < 30.0
    assert ops.chain_error(dev) == 1, "the chain could not have been co-resident"
    assert ops.chain_status(dev), "the kernel did not write the bound host status word"
    assert_failed_outputs_nan(ops, links, dev, "co-residency timeout")
    with pytest.raises(_lib.ChainTimeoutError):
        ops.linear_chain_w6ax(links)
    ops.chain_reset(dev)
    for (*_, out) in links:
        out.fill_(float("nan"))
    ops.linear_chain_w6ax(links)
    torch.cuda.synchronize()
    check(ops, links, dev, "after the co-residency timeout and chain_reset")


def _layer_links(ops, dev, g, x_attn, h, n_layers=1):
    """A LLaMA-2-7B decoder layer's linears after the attention core as chain links (M = 1):
    o -> RMSNorm(h + o) + gate_up -> SiLU(gate) * up + down -> RMSNorm(h' + down) + next qkv.
    Returns (links, the same as one callable per link for the sequential reference)."""
    H, F = 4096, 11008
    links, x = [], x_attn
    res = h
    for _ in range(n_layers):
        o_out = torch.empty((1, H), dtype=torch.float16, device=dev)
        gu_out = torch.empty((1, 2 * F), dtype=torch.float16, device=dev)
        dn_out = torch.empty((1, H), dtype=torch.float16, device=dev)
        qkv_out = torch.empty((1, 3 * H), dtype=torch.float16, device=dev)
        r1 = torch.empty((1, H), dtype=torch.float16, device=dev)
        r2 = torch.empty((1, H), dtype=torch.float16, device=dev)
        g1 = (1.0 + 0.2 * torch.randn(H, device=dev, generator=g)).half()
        g2 = (1.0 + 0.2 * torch.randn(H, device=dev, generator=g)).half()
        links += [(x, image(ops, H, H, g, dev), H, 6, o_out),
                  ops.chain_rmsnorm(res, g1, image(ops, 2 * F, H, g, dev), 2 * F, 6, gu_out, input=o_out,
                                    residual_out=r1),
                  ops.chain_silu(gu_out[:, :F], gu_out[:, F:], image(ops, H, F, g, dev), H, 8, dn_out),
                  ops.chain_rmsnorm(r1, g2, image(ops, 3 * H, H, g, dev), 3 * H, 6, qkv_out, input=dn_out,
                                    residual_out=r2)]
        x, res = qkv_out[:, 2 * H:], r2  # the attention stand-in: ctx = v
    return links


def _sequential_any(ops, links):
    """Each link through its own entry point, in order, on the same buffers (fresh outputs compared)."""
    res = []
    for lk in links:
        if isinstance(lk, dict) and lk["kind"] == "rmsnorm":
            out = torch.empty_like(lk["out"])
            ro = torch.empty_like(lk["residual_out"]) if lk["input"] is not None else None
            ops.rmsnorm_linear_w6ax(lk["x"], lk["gamma"], lk["w"], lk["N"], lk["abits"], eps=lk["eps"],
                                    input=lk["input"], residual_out=ro, out=out)
            res.append((out, ro))
        elif isinstance(lk, dict):
            out = torch.empty_like(lk["out"])
            ops.silu_linear_w6ax(lk["x"], lk["up"], lk["w"], lk["N"], lk["abits"], out=out)
            res.append((out, None))
        else:
            x, wpk, N, abits, o = lk
            res.append((ops.linear_w6ax(x, wpk, N, abits), None))
    torch.cuda.synchronize()
    return res


def _outs(lk):
    if isinstance(lk, dict):
        return lk["out"], lk.get("residual_out") if lk.get("input") is not None else None
    return lk[4], None


@pytest.mark.parametrize("n_layers", [1, 2])
def test_chain_decoder_layer_with_producers(ops, dev, n_layers):
    """o -> RMSNorm + gate_up -> SiLU * up + down -> RMSNorm + qkv as one launch (two layers: 8 links),
    every output and residual output bit-identical to the four entry points called one by one.  The
    sequential reference runs AFTER the chain on the chain's own inputs (each link's inputs are the
    chain's buffers, which the chain filled with the same bits the entry points produce)."""
    g = torch.Generator(device=dev).manual_seed(41 + n_layers)
    x_attn = torch.randn((1, 4096), dtype=torch.float16, device=dev, generator=g)
    h = torch.randn((1, 4096), dtype=torch.float16, device=dev, generator=g)
    links = _layer_links(ops, dev, g, x_attn, h, n_layers)
    for rep in range(2):
        for lk in links:
            o, ro = _outs(lk)
            o.fill_(float("nan"))
            if ro is not None:
                ro.fill_(float("nan"))
        ops.linear_chain_w6ax(links)
        torch.cuda.synchronize()
        ref = _sequential_any(ops, links)
        for i, (lk, (ro_ref_out, ro_ref_res)) in enumerate(zip(links, ref)):
            o, ro = _outs(lk)
            np.testing.assert_array_equal(o.cpu().numpy().view(np.uint16), ro_ref_out.cpu().numpy().view(np.uint16),
                                          err_msg=f"rep {rep} link {i} output")
            if ro is not None:
                np.testing.assert_array_equal(ro.cpu().numpy().view(np.uint16), ro_ref_res.cpu().numpy().view(np.uint16),
                                              err_msg=f"rep {rep} link {i} residual output")
        assert ops.chain_error(dev) == 0


def test_chain_silu_link_at_m2(ops, dev):
    """gate_up -> SiLU * up + down -> qkv at M = 2 (gate / up rows of stride 2F inside the previous
    output): one launch, bit-identical to the entry points."""
    g = torch.Generator(device=dev).manual_seed(53)
    H, F = 4096, 11008
    x = torch.randn((2, H), dtype=torch.float16, device=dev, generator=g)
    gu = torch.empty((2, 2 * F), dtype=torch.float16, device=dev)
    dn = torch.empty((2, H), dtype=torch.float16, device=dev)
    qkv = torch.empty((2, 3 * H), dtype=torch.float16, device=dev)
    links = [(x, image(ops, 2 * F, H, g, dev), 2 * F, 6, gu),
             ops.chain_silu(gu[:, :F], gu[:, F:], image(ops, H, F, g, dev), H, 8, dn),
             (dn, image(ops, 3 * H, H, g, dev), 3 * H, 6, qkv)]
    ops.linear_chain_w6ax(links)
    torch.cuda.synchronize()
    ref = _sequential_any(ops, links)
    for i, (lk, (r, _)) in enumerate(zip(links, ref)):
        np.testing.assert_array_equal(_outs(lk)[0].cpu().numpy().view(np.uint16), r.cpu().numpy().view(np.uint16),
                                      err_msg=f"link {i}")
    assert ops.chain_error(dev) == 0
