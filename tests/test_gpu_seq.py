"""GPU parity tests of the one-launch linear chain (fq_linear_seq_*, flexq_amd.ops.LinearSeq).

A chain must compute exactly what calling fq_linear_w6ax on each linear in order computes:
  * bit-identical to the one-by-one launches on LLaMA-shaped linears (their plans have no
    k-split, so the summation order is the same), with real data dependencies between the
    linears (the input of one is a column slice of an earlier output) -- this is the cross-XCD
    hand-off inside the launch;
  * every linear within the oracle tolerance of the CPU restatement, fed the chain's own input;
  * WAR / WAW hazards (a later linear overwriting an earlier one's input or output) ordered;
  * repeated runs with changed inputs read fresh data (stale-line hazard), graph replay works,
    the counters are left zero and the error word stays zero.
"""
import numpy as np
import pytest
import torch

from common import assert_gemm_close, oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops(dev):
    from flexq_amd import ops as _ops
    return _ops


def weight(ops, dev, N, K, seed):
    """Weight image of a random [N, K] fp16 matrix with unit gain (std 1/sqrt(K)), so values stay
    O(1) through a chain of dependent linears; also returns its codes and scales."""
    g = torch.Generator(device=dev).manual_seed(seed)
    w = (torch.randn((N, K), generator=g, device=dev) / K ** 0.5).half()
    wpk, ws, wq = ops.quantize_pack_w6(w, return_codes=True)
    return wpk, wq, ws


def oracle_linear(x, wq, ws, abits):
    """The CPU restatement of one decode linear on the GPU's own input x (fp16 [M, K])."""
    xq, xs = oracle.quantize_engine(x, abits)
    d, _, mag = oracle.gemm(xq, xs, wq, ws)
    return d, mag


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def llama_chain(ops, dev, M, layers, down_bits=6, seed=0):
    """`layers` LLaMA-2-7B-shaped layers as a dependent chain: qkv(x) -> o(qkv[:, :4096]) ->
    gate_up(o) -> down(gate_up[:, :11008]) -> next layer's qkv(down).  Returns the list of
    linears (x producer, N, K, abits, weight) and the chain input."""
    shapes = [("qkv", 12288, 4096, 6), ("o", 4096, 4096, 6), ("gate_up", 22016, 4096, 6),
              ("down", 4096, 11008, down_bits)]
    lins = []
    for l in range(layers):
        for i, (name, N, K, ab) in enumerate(shapes):
            wpk, wq, ws = weight(ops, dev, N, K, seed + 17 * l + i)
            lins.append(dict(name=f"{name}{l}", N=N, K=K, abits=ab, wpk=wpk, wq=wq, ws=ws))
    g = torch.Generator(device=dev).manual_seed(seed + 999)
    x0 = torch.randn((M, 4096), generator=g, device=dev).half()
    return lins, x0


def wire(lins, x0, M, dev):
    """Output buffers and inputs of the chain: input j = first K columns of output j - 1."""
    outs = [torch.empty((M, l["N"]), dtype=torch.float16, device=dev) for l in lins]
    xs = [x0] + [outs[j - 1][:, :lins[j]["K"]] for j in range(1, len(lins))]
    return outs, xs


def run_sequential(ops, lins, x0, M, dev):
    outs, xs = wire(lins, x0, M, dev)
    for l, x, o in zip(lins, xs, outs):
        ops.linear_w6ax(x.contiguous(), l["wpk"], l["N"], l["abits"], out=o)
    torch.cuda.synchronize()
    return outs, xs


def make_seq(ops, lins, x0, M, dev):
    outs, xs = wire(lins, x0, M, dev)
    seq = ops.LinearSeq([(x, l["wpk"], l["N"], l["abits"], o) for l, x, o in zip(lins, xs, outs)])
    return seq, outs, xs


@pytest.mark.parametrize("M,down_bits", [(1, 6), (2, 8), (4, 6)])
def test_chain_matches_one_by_one_llama(ops, dev, M, down_bits):
    lins, x0 = llama_chain(ops, dev, M, layers=2, down_bits=down_bits, seed=M)
    ref, _ = run_sequential(ops, lins, x0, M, dev)
    seq, outs, xs = make_seq(ops, lins, x0, M, dev)
    seq.run()
    torch.cuda.synchronize()
    assert seq.error_word() == 0
    assert not seq.counters().any(), "counters must be left zero"
    for l, a, b in zip(lins, outs, ref):
        an, bn = host(a), host(b)
        assert np.isfinite(an.astype(np.float32)).all(), l["name"]
        np.testing.assert_array_equal(an.view(np.uint16), bn.view(np.uint16), err_msg=l["name"])
    # each linear against the oracle on the chain's own input (sampled columns of the big ones)
    for j in (0, 1, 3, 4, 7):
        l = lins[j]
        x = host(xs[j].contiguous())
        cols = np.arange(0, l["N"], 7)
        wq = host(l["wq"])[cols]
        ws = host(l["ws"])[:, cols]
        got = host(outs[j])[:, cols]
        ref_o, mag = oracle_linear(x, wq, ws, l["abits"])
        assert_gemm_close(got, ref_o, mag, l["name"])


@pytest.mark.parametrize("M", [1, 3])
def test_chain_independent_ragged_shapes(ops, dev, M):
    """Independent linears (no overlaps: no waits) over ragged shapes: N % 16 != 0 and more
    tiles than CUs (N = 4100 -> 257 tiles), K = 128 (one group: waves with no groups), K = 11008,
    A8; each against the oracle."""
    shapes = [(4100, 1024, 6), (64, 128, 8), (2052, 11008, 6), (512, 256, 8), (4096, 384, 6)]
    ents, chk = [], []
    for i, (N, K, ab) in enumerate(shapes):
        wpk, wq, ws = weight(ops, dev, N, K, 100 + i)
        g = torch.Generator(device=dev).manual_seed(200 + i)
        x = torch.randn((M, K), generator=g, device=dev).half()
        o = torch.full((M, N), float("nan"), dtype=torch.float16, device=dev)
        ents.append((x, wpk, N, ab, o))
        chk.append((x, wq, ws, ab, o))
    seq = ops.LinearSeq(ents)
    for rep in range(2):
        seq.run()
        torch.cuda.synchronize()
        assert seq.error_word() == 0
        for (x, wq, ws, ab, o) in chk:
            ref, mag = oracle_linear(host(x), host(wq), host(ws), ab)
            assert_gemm_close(host(o), ref, mag, f"N={o.shape[1]} rep={rep}")


def test_chain_war_and_waw_hazards(ops, dev):
    """Linear 1 overwrites linear 0's input (WAR); linear 2 reads linear 1's output and writes
    linear 0's output buffer (RAW + WAW); linear 3 reads that.  The chain must equal the
    launches in order."""
    M, K = 1, 4096
    N = 4096
    w = [weight(ops, dev, N, K, 300 + i)[0] for i in range(4)]
    g = torch.Generator(device=dev).manual_seed(5)
    a0 = torch.randn((M, K), generator=g, device=dev).half()
    c0 = torch.randn((M, K), generator=g, device=dev).half()

    def program(run_seq):
        A, C = a0.clone(), c0.clone()
        B = torch.empty((M, N), dtype=torch.float16, device=dev)
        D = torch.empty((M, N), dtype=torch.float16, device=dev)
        steps = [(A, w[0], B), (C, w[1], A), (A, w[2], B), (B, w[3], D)]
        if run_seq:
            seq = ops.LinearSeq([(x, wp, N, 6, o) for (x, wp, o) in steps])
            seq.run()
            torch.cuda.synchronize()
            assert seq.error_word() == 0
        else:
            for (x, wp, o) in steps:
                ops.linear_w6ax(x, wp, N, 6, out=o)
        torch.cuda.synchronize()
        return [host(t).view(np.uint16) for t in (A, B, D)]

    for got, ref in zip(program(True), program(False)):
        np.testing.assert_array_equal(got, ref)


def test_chain_fresh_inputs_graph_replay(ops, dev):
    """Re-running the chain after its input changed must read the new data (every consumer CU
    has the old lines cached), eagerly and under graph replay."""
    M = 1
    lins, x0 = llama_chain(ops, dev, M, layers=1, seed=11)
    seq, outs, xs = make_seq(ops, lins, x0, M, dev)
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        seq.run()
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        seq.run()
    g = torch.Generator(device=dev).manual_seed(77)
    for rep in range(3):
        x0.copy_(torch.randn(x0.shape, generator=g, device=dev).half())
        torch.cuda.synchronize()
        if rep == 1:
            with torch.cuda.stream(s):
                seq.run()
        else:
            graph.replay()
        torch.cuda.synchronize()
        ref, _ = run_sequential(ops, lins, x0, M, dev)
        for l, a, b in zip(lins, outs, ref):
            np.testing.assert_array_equal(host(a).view(np.uint16), host(b).view(np.uint16),
                                          err_msg=f"{l['name']} rep={rep}")
    assert seq.error_word() == 0
    assert not seq.counters().any()


def test_chain_rejects_unsupported(ops, dev):
    from flexq_amd._lib import FlexQError
    wpk, _, _ = weight(ops, dev, 64, 128, 1)
    x5 = torch.zeros((5, 128), dtype=torch.float16, device=dev)
    o5 = torch.empty((5, 64), dtype=torch.float16, device=dev)
    with pytest.raises(FlexQError):  # M > 4
        ops.LinearSeq([(x5, wpk, 64, 6, o5)])
    wpk2, _, _ = weight(ops, dev, 66, 128, 2)
    x1 = torch.zeros((1, 128), dtype=torch.float16, device=dev)
    o1 = torch.empty((1, 66), dtype=torch.float16, device=dev)
    with pytest.raises(FlexQError):  # N % 4 != 0
        ops.LinearSeq([(x1, wpk2, 66, 6, o1)])
