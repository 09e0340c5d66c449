"""GPU test of the FlexQ FFN block (flexq_amd.layers.FlexQFfn: RMSNorm+quantize -> gate_up W6A6
-> SiLU*up -> A8 -> down W6A8, FT FfnLayer int8_mode 5).  Each stage is checked against the
oracle on the block's own intermediate inputs (bit-exact where the stage is integer/bit-exact,
oracle tolerance for the GEMMs), and the whole block against a float64 unquantized FFN
(loose: W6A6/W6A8 quantization error), loaded from converter files at TP 1 and 2 (FT's layout: column-parallel gate_up, row-parallel
down_proj + all-reduce); the decoder layer (attention half around a stand-in attention core)
likewise, and once through a real two-process all-reduce."""
import numpy as np
import pytest
import torch

from common import assert_gemm_close, oracle

pytestmark = pytest.mark.gpu

H, F = 512, 768


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


@pytest.fixture(scope="module")
def weights():
    g = torch.Generator().manual_seed(5)
    return dict(gate=(torch.randn((F, H), generator=g) / H ** 0.5).half(),
                up=(torch.randn((F, H), generator=g) / H ** 0.5).half(),
                down=(torch.randn((H, F), generator=g) / F ** 0.5).half(),
                gamma=(1 + 0.1 * torch.randn(H, generator=g)).half())


@pytest.mark.parametrize("M", [1, 16])
def test_ffn_stages_against_oracle(dev, weights, M):
    from flexq_amd.layers import FlexQFfn, W6Linear
    w = weights
    ffn = FlexQFfn(W6Linear.from_fp16(torch.cat([w["gate"], w["up"]]).to(dev), 6),
                   W6Linear.from_fp16(w["down"].to(dev), 8), w["gamma"].to(dev))
    g = torch.Generator().manual_seed(M)
    res0 = torch.randn((M, H), generator=g).half()
    attn = torch.randn((M, H), generator=g).half()
    res = res0.to(dev)
    y, im = ffn(res, attn.to(dev), return_intermediates=True)
    # stage 1: residual add + RMSNorm + A6 codes, bit-exact
    r_ref, _, q_ref, xs_ref = oracle.rmsnorm_quantize(attn.numpy(), res0.numpy(), w["gamma"].numpy(), 1e-6, 6)
    np.testing.assert_array_equal(host(res).view(np.uint16), r_ref.view(np.uint16))
    np.testing.assert_array_equal(host(im["xq"]), q_ref)
    # stage 2: gate_up GEMM within the oracle tolerance
    wq_gu, ws_gu = oracle.quantize_engine(torch.cat([w["gate"], w["up"]]).numpy(), 6)
    ref, _, mag = oracle.gemm(q_ref, xs_ref, wq_gu, ws_gu)
    assert_gemm_close(host(im["gate_up"]), ref, mag, "gate_up")
    # stage 3: SiLU*up A8 codes == engine quantizer of the kernel's product (tested in detail elsewhere)
    gu = host(im["gate_up"])
    act = oracle.silu_mul_ref(gu[:, :F], gu[:, F:])
    aq_ref, as_ref = oracle.quantize_engine(act, 8)
    mism = (host(im["aq"]).astype(int) - aq_ref.astype(int))
    assert np.abs(mism).max() <= 1 and (mism != 0).mean() < 1e-2  # one-ulp fp16 products only
    # stage 4: down GEMM on the block's own codes
    wq_d, ws_d = oracle.quantize_engine(w["down"].numpy(), 6)
    ref_y, _, mag_y = oracle.gemm(host(im["aq"]), host(im["as_"]), wq_d, ws_d)
    assert_gemm_close(host(y), ref_y, mag_y, "down")
    # the block against an unquantized float64 FFN: W6A6/W6A8 error only
    a = r_ref.astype(np.float64)
    n = a / np.sqrt((a * a).mean(1, keepdims=True) + 1e-6) * w["gamma"].numpy().astype(np.float64)
    gt = n @ w["gate"].numpy().astype(np.float64).T
    ut = n @ w["up"].numpy().astype(np.float64).T
    yt = (gt / (1 + np.exp(-gt)) * ut) @ w["down"].numpy().astype(np.float64).T
    rel = np.linalg.norm(host(y).astype(np.float64) - yt) / np.linalg.norm(yt)
    # 6-bit per-group activations of Gaussian data carry ~2-3 % RMS error per operand (step
    # absmax/31), compounded through gate/up, SiLU and down: a sanity bound, not a parity one
    assert rel < 0.1, rel


def _ckpt(tmp_path, w, attn=None):
    from safetensors.torch import save_file
    t = {"model.layers.0.mlp.gate_proj.weight": w["gate"], "model.layers.0.mlp.up_proj.weight": w["up"],
         "model.layers.0.mlp.down_proj.weight": w["down"]}
    for n in ("q", "k", "v", "o"):  # (separate storage: safetensors refuses shared tensors)
        t[f"model.layers.0.self_attn.{n}_proj.weight"] = (attn[n] if attn else w["down"][:, :H]).clone()
    save_file(t, str(tmp_path / "m.safetensors"))
    return str(tmp_path / "m.safetensors")


def ulp16(a):
    return np.spacing(np.abs(a).astype(np.float16)).astype(np.float64)


@pytest.mark.parametrize("tp", [1, 2])
def test_ffn_from_converter_files(dev, weights, tmp_path, tp):
    """Converter files (FT's TP layout): at TP 1 the FFN block loads and matches the block built
    from fp16 weights bit for bit.  At TP 2 each rank runs its [gate_p; up_p] image, its SiLU*up
    (rank-local A8 codes: concatenated, exactly the TP-1 codes, since the split is on 128-group
    boundaries) and its row-parallel down_proj column slice (partial sum within the oracle
    tolerance on its own codes); the partials' sum (what the all-reduce returns) is the TP-1
    output within the full-K oracle tolerance plus one fp16 rounding per partial."""
    from flexq_amd import convert
    from flexq_amd.layers import FlexQFfn, W6Linear
    w = weights
    out = str(tmp_path / "out")
    convert.convert_llama_safetensors(_ckpt(tmp_path, w), out, tp_size=tp, device=str(dev))
    x = torch.randn((4, H), generator=torch.Generator().manual_seed(9)).half().to(dev)
    ref = FlexQFfn(W6Linear.from_fp16(torch.cat([w["gate"], w["up"]]).to(dev), 6),
                   W6Linear.from_fp16(w["down"].to(dev), 8), w["gamma"].to(dev))
    y_ref, im_ref = ref(x.clone(), None, return_intermediates=True)
    if tp == 1:
        ffn = FlexQFfn.from_dir(out, 0, w["gamma"], device=dev)
        y = ffn(x.clone())
        np.testing.assert_array_equal(host(y).view(np.uint16), host(y_ref).view(np.uint16))
        return
    aqs, parts = [], []
    for r in range(tp):
        ffn_r = FlexQFfn.from_dir(out, 0, w["gamma"], rank=r, device=dev)
        assert ffn_r.down.row_parallel and not ffn_r.gate_up.row_parallel
        y_r, im_r = ffn_r(x.clone(), None, return_intermediates=True, reduce=False)
        cols, _ = convert.shard_columns(w["down"], tp, r)
        wq, ws = oracle.quantize_engine(cols.numpy(), 6)
        ref_r, _, mag_r = oracle.gemm(host(im_r["aq"]), host(im_r["as_"]), wq, ws)
        assert_gemm_close(host(y_r), ref_r, mag_r, f"down_proj partial, rank {r}")
        aqs.append(host(im_r["aq"]))
        parts.append(host(y_r).astype(np.float64))
    np.testing.assert_array_equal(np.concatenate(aqs, 1), host(im_ref["aq"]))
    wq, ws = oracle.quantize_engine(w["down"].numpy(), 6)
    ref_full, _, mag = oracle.gemm(host(im_ref["aq"]), host(im_ref["as_"]), wq, ws)
    tol = oracle.gemm_tolerance(ref_full, mag) + sum(ulp16(p) for p in parts)
    assert (np.abs(sum(parts) - ref_full.astype(np.float64)) <= tol).all()


HD = 128  # head_dim = one quantization group


def _attn_stand_in(qkv):
    """Stand-in for the out-of-scope attention core: each head's context = its v slice (rank-local
    per head, like the real core)."""
    return qkv[:, 2 * qkv.shape[1] // 3:]


def _decoder_weights():
    g = torch.Generator().manual_seed(11)
    return {n: (torch.randn((H, H), generator=g) / H ** 0.5).half() for n in ("q", "k", "v", "o")}


def test_run_layers_defers_residual_bit_identical(dev, weights, tmp_path):
    """run_layers fuses each layer's final residual add into the next layer's pre-attention norm
    (FT's add-residual + norm): the same bits as calling the layers one by one."""
    from flexq_amd import convert
    from flexq_amd.layers import FlexQDecoderLayer, run_layers
    w, aw = weights, _decoder_weights()
    ga = (1 + 0.1 * torch.randn(H, generator=torch.Generator().manual_seed(21))).half()
    out = str(tmp_path / "tp1")
    convert.convert_llama_safetensors(_ckpt(tmp_path, w, aw), out, tp_size=1, device=str(dev))
    L = FlexQDecoderLayer.from_dir(out, 0, ga, w["gamma"], _attn_stand_in, device=dev)
    for M in (1, 5):
        x = torch.randn((M, H), generator=torch.Generator().manual_seed(22 + M)).half().to(dev)
        h_ref = x.clone()
        for _ in range(3):
            L(h_ref)
        h = run_layers([L, L, L], x.clone())
        assert torch.equal(h.view(torch.int16), h_ref.view(torch.int16))


@pytest.mark.parametrize("tp", [1, 2])
def test_decoder_layer_tp(dev, weights, tmp_path, tp):
    """FlexQDecoderLayer (FT LlamaContextDecoder order) from converter files.  TP 1: the attention
    half against the oracle stage by stage, the layer against a float64 unquantized layer
    (sanity bound).  TP 2, both ranks simulated on one GPU: each rank's o_proj partial on its own
    heads and each rank's FFN partial, summed as the all-reduces would (fp16 sums), against TP 1."""
    from flexq_amd import convert, ops
    from flexq_amd.layers import FlexQDecoderLayer
    w, aw = weights, _decoder_weights()
    ga = (1 + 0.1 * torch.randn(H, generator=torch.Generator().manual_seed(12))).half()
    out1, outp = str(tmp_path / "tp1"), str(tmp_path / "tpn")
    ck = _ckpt(tmp_path, w, aw)
    convert.convert_llama_safetensors(ck, out1, tp_size=1, device=str(dev))
    x = torch.randn((5, H), generator=torch.Generator().manual_seed(13)).half()
    L1 = FlexQDecoderLayer.from_dir(out1, 0, ga, w["gamma"], _attn_stand_in, device=dev)
    a1 = L1.attention(x.to(dev))
    h1 = L1(x.to(dev).clone())
    # attention half against the oracle: A6 codes of the pre-attention norm, qkv, o_proj
    _, _, q_ref, xs_ref = oracle.rmsnorm_quantize(None, x.numpy(), ga.numpy(), 1e-6, 6)
    wq, ws = oracle.quantize_engine(torch.cat([aw["q"], aw["k"], aw["v"]]).numpy(), 6)
    qkv_ref, _, mag = oracle.gemm(q_ref, xs_ref, wq, ws)
    xq, xs = ops.rmsnorm_quantize(x.to(dev), ga.to(dev), 6)
    qkv = L1.qkv.from_codes(xq, xs)
    assert_gemm_close(host(qkv), qkv_ref, mag, "qkv")
    cq, cs = oracle.quantize_engine(host(_attn_stand_in(qkv)), 6)
    wq, ws = oracle.quantize_engine(aw["o"].numpy(), 6)
    a_ref, _, mag_a = oracle.gemm(cq, cs, wq, ws)
    assert_gemm_close(host(a1), a_ref, mag_a, "o_proj")
    if tp == 1:
        # the whole layer against float64 unquantized math (W6A6/W6A8 error only)
        def rms(v, gm):
            return v / np.sqrt((v * v).mean(1, keepdims=True) + 1e-6) * gm.numpy().astype(np.float64)
        f = lambda t: t.numpy().astype(np.float64)  # noqa: E731
        h = f(x)
        n = rms(h, ga)
        a = (n @ f(aw["v"]).T) @ f(aw["o"]).T
        h = h + a
        n = rms(h, w["gamma"])
        gt, ut = n @ f(w["gate"]).T, n @ f(w["up"]).T
        h = h + (gt / (1 + np.exp(-gt)) * ut) @ f(w["down"]).T
        rel = np.linalg.norm(host(h1).astype(np.float64) - h) / np.linalg.norm(h)
        assert rel < 0.05, rel
        return
    convert.convert_llama_safetensors(ck, outp, tp_size=tp, device=str(dev))
    Ls = [FlexQDecoderLayer.from_dir(outp, 0, ga, w["gamma"], _attn_stand_in, rank=r, device=dev) for r in range(tp)]
    assert all(L.o.row_parallel and L.o.K == H // tp for L in Ls)
    a_parts = [L.attention(x.to(dev), reduce=False) for L in Ls]
    a_sum = a_parts[0] + a_parts[1]  # the fp16 all-reduce of 2 ranks
    tol = oracle.gemm_tolerance(a_ref, mag_a) + sum(ulp16(host(p)) for p in a_parts) + ulp16(a_ref)
    assert (np.abs(host(a_sum).astype(np.float64) - a_ref.astype(np.float64)) <= tol).all()
    # FFN half on the same input (h + the all-reduced attention output): a one-ulp difference in
    # a_sum can flip a 6-bit code at a rounding boundary, so the TP-1 reference takes a_sum too
    h = x.to(dev).clone()
    y_parts = [L.ffn(h.clone(), a_sum, reduce=False) for L in Ls]
    y1 = L1.ffn(h.clone(), a_sum)
    y = host(y_parts[0] + y_parts[1]).astype(np.float64)
    tol = 2e-3 * np.abs(host(y1).astype(np.float64)) + sum(ulp16(host(p)) for p in y_parts) + ulp16(host(y1))
    assert (np.abs(y - host(y1).astype(np.float64)) <= tol).all()


def _mp_worker(rank, world, port, out_dir, x, ga, gf, q):
    import torch.distributed as dist
    from flexq_amd.layers import FlexQDecoderLayer
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        from flexq_amd.layers import run_layers
        L = FlexQDecoderLayer.from_dir(out_dir, 0, ga, gf, _attn_stand_in, rank=rank, device="cuda:0")
        h = L(x.to("cuda:0").clone())
        h2 = L(h.clone())  # two layers one by one ...
        hr = run_layers([L, L], x.to("cuda:0").clone())  # ... and through run_layers' fused forms
        torch.cuda.synchronize()
        q.put((rank, h.cpu(), h2.cpu(), hr.cpu()))
    finally:
        dist.destroy_process_group()


def test_decoder_layer_two_processes(dev, weights, tmp_path):
    """The real collective path: two ranks (processes) sharing the box's one GPU, the layer's two
    all-reduces through torch.distributed (gloo here, RCCL on an 8-GPU node); both ranks end with
    the same hidden state, equal to the one-GPU simulation of the same shards."""
    import socket
    import torch.multiprocessing as mp
    from flexq_amd import convert
    from flexq_amd.layers import FlexQDecoderLayer
    w, aw = weights, _decoder_weights()
    ga = (1 + 0.1 * torch.randn(H, generator=torch.Generator().manual_seed(12))).half()
    out = str(tmp_path / "tp2")
    convert.convert_llama_safetensors(_ckpt(tmp_path, w, aw), out, tp_size=2, device=str(dev))
    x = torch.randn((3, H), generator=torch.Generator().manual_seed(14)).half()
    Ls = [FlexQDecoderLayer.from_dir(out, 0, ga, w["gamma"], _attn_stand_in, rank=r, device=dev) for r in range(2)]
    a = Ls[0].attention(x.to(dev), reduce=False) + Ls[1].attention(x.to(dev), reduce=False)
    h = x.to(dev).clone()
    y = Ls[0].ffn(h.clone(), a, reduce=False) + Ls[1].ffn(h.clone(), a, reduce=False)
    h += a
    h += y
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_mp_worker, args=(r, 2, port, out, x, ga, w["gamma"], q)) for r in range(2)]
    for p_ in procs:
        p_.start()
    res = {}
    for _ in range(2):
        r, *outs = q.get(timeout=100)
        res[r] = [o.numpy().view(np.uint16) for o in outs]
    for p_ in procs:
        p_.join(timeout=60)
        assert p_.exitcode == 0
    for k in range(3):
        np.testing.assert_array_equal(res[0][k], res[1][k])
    np.testing.assert_array_equal(res[0][0], host(h).view(np.uint16))
    np.testing.assert_array_equal(res[0][2], res[0][1])  # run_layers == layer by layer, with all-reduces


def test_run_layers_fused_producers_llama_width(dev):
    """At the LLaMA-2-7B widths (H = 4096, F = 11008) run_layers takes the one-launch forms -- the
    RMSNorm (+ residual add) inside qkv's and gate_up's decode GEMMs at M = 1, SiLU * up inside
    down_proj's -- and must give the bits of the unfused layer calls (producer kernel, then GEMM)."""
    from flexq_amd import ops
    from flexq_amd.layers import FlexQDecoderLayer, FlexQFfn, W6Linear, run_layers
    Hs, Fs = 4096, 11008
    g = torch.Generator().manual_seed(31)
    rnd = lambda n, k: (torch.randn((n, k), generator=g) / k ** 0.5).half().to(dev)  # noqa: E731
    lin = lambda n, k, ab=6: W6Linear.from_fp16(rnd(n, k), ab)  # noqa: E731
    ga = (1 + 0.1 * torch.randn(Hs, generator=g)).half().to(dev)
    gf = (1 + 0.1 * torch.randn(Hs, generator=g)).half().to(dev)
    ffn = FlexQFfn(lin(2 * Fs, Hs), lin(Hs, Fs, 8), gf)
    L = FlexQDecoderLayer(lin(3 * Hs, Hs), lin(Hs, Hs), ffn, ga, lambda qkv: qkv[:, 2 * Hs:])
    assert int(ops._lib.load().fq_rmsnorm_linear_scratch_bytes(1, 3 * Hs, Hs)) == 0  # fused at M = 1
    assert int(ops._lib.load().fq_silu_linear_scratch_bytes(1, Hs, Fs)) == 0
    for M in (1, 3):
        x = torch.randn((M, Hs), generator=torch.Generator().manual_seed(40 + M)).half().to(dev)
        h_ref = x.clone()
        for _ in range(3):
            L(h_ref)
        h = run_layers([L, L, L], x.clone())
        assert torch.equal(h.view(torch.int16), h_ref.view(torch.int16)), f"M = {M}"


def test_run_layers_chained_bit_identical(dev):
    """run_layers_chained (decode chains: o -> RMSNorm + gate_up -> SiLU * up + down -> RMSNorm + next
    qkv as one launch per layer at M = 1; the entry points elsewhere) gives run_layers' bits, at M = 1
    (chained) and M = 3 (every link alone), over three layers."""
    from flexq_amd import ops
    from flexq_amd.layers import FlexQDecoderLayer, FlexQFfn, W6Linear, run_layers, run_layers_chained
    Hs, Fs = 4096, 11008
    g = torch.Generator().manual_seed(33)
    rnd = lambda n, k: (torch.randn((n, k), generator=g) / k ** 0.5).half().to(dev)  # noqa: E731
    lin = lambda n, k, ab=6: W6Linear.from_fp16(rnd(n, k), ab)  # noqa: E731
    layers = []
    for _ in range(3):
        ga = (1 + 0.1 * torch.randn(Hs, generator=g)).half().to(dev)
        gf = (1 + 0.1 * torch.randn(Hs, generator=g)).half().to(dev)
        ffn = FlexQFfn(lin(2 * Fs, Hs), lin(Hs, Fs, 8), gf)
        layers.append(FlexQDecoderLayer(lin(3 * Hs, Hs), lin(Hs, Hs), ffn, ga, lambda qkv: qkv[:, 2 * Hs:]))
    for M in (1, 3):
        x = torch.randn((M, Hs), generator=torch.Generator().manual_seed(50 + M)).half().to(dev)
        h_ref = run_layers(layers, x.clone())
        h = run_layers_chained(layers, x.clone())
        torch.cuda.synchronize()
        assert torch.equal(h.view(torch.int16), h_ref.view(torch.int16)), f"M = {M}"
        assert ops.chain_error(dev) == 0
