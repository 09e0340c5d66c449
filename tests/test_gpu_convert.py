"""GPU test of the offline converter (flexq_amd.convert): a tiny synthetic
LLaMA checkpoint (safetensors, random fp16 weights -- no real checkpoint exists offline) is
converted at TP 1 and 2; every file must hold exactly the image fq_quantize_pack_w6 makes of the
rank's shard (stacked rows of qkv / gate_up, the 128-group column slice of o_proj / down_proj),
and a linear run from a loaded file must match the oracle."""
import json
import os

import numpy as np
import pytest
import torch

from common import assert_gemm_close, oracle

pytestmark = pytest.mark.gpu

H, F, LAYERS = 256, 384, 2


@pytest.fixture(scope="module")
def ckpt(tmp_path_factory):
    from safetensors.torch import save_file
    g = torch.Generator().manual_seed(0)
    t = {}
    for li in range(LAYERS):
        p = f"model.layers.{li}."
        for n, shape in [("self_attn.q_proj", (H, H)), ("self_attn.k_proj", (H // 2, H)),
                         ("self_attn.v_proj", (H // 2, H)), ("self_attn.o_proj", (H, H)),
                         ("mlp.gate_proj", (F, H)), ("mlp.up_proj", (F, H)), ("mlp.down_proj", (H, F))]:
            t[p + n + ".weight"] = (torch.randn(shape, generator=g) * 0.05).half()
        t[p + "input_layernorm.weight"] = torch.ones(H).half()
    d = tmp_path_factory.mktemp("ckpt")
    save_file(t, str(d / "model.safetensors"))
    return str(d / "model.safetensors"), t


@pytest.mark.parametrize("tp", [1, 2])
def test_convert_llama(dev, ckpt, tmp_path, tp):
    from flexq_amd import convert, ops
    path, t = ckpt
    m = convert.convert_llama_safetensors(path, str(tmp_path), tp_size=tp, device=str(dev))
    assert len(m["linears"]) == LAYERS * 4 * tp
    assert json.load(open(tmp_path / "manifest.json"))["tp_size"] == tp
    for e in m["linears"]:
        parts = [t[f"model.layers.{e['layer']}.{p}.weight"] for p in e["parts"]]
        img, meta = convert.load_image(os.path.join(str(tmp_path), e["file"]), device=dev)
        if e["split"] == "row":  # attention.dense, down_proj: the rank's 128-group column slice
            w_r, k_off = convert.shard_columns(parts[0], tp, e["rank"])
            assert meta["split"] == convert.ROW and meta["k_offset"] == k_off == e["k_offset"]
        else:  # qkv, gate_up: the rank's rows of each part, stacked
            w_r = convert.shard_parts(parts, tp, e["rank"], by_group=e["name"] == "mlp.gate_up_proj")
            assert meta["split"] == convert.COLUMN
        assert (meta["N"], meta["K"], meta["tp_rank"], meta["abits"]) == (w_r.shape[0], w_r.shape[1], e["rank"],
                                                                          8 if "down" in e["name"] else 6)
        ref_img, ws = ops.quantize_pack_w6(w_r.to(dev))
        assert torch.equal(img, ref_img), e["file"]
        if e["layer"] == 0:  # the loaded image runs: linear vs the oracle
            N, K = w_r.shape
            x = torch.randn((3, K), generator=torch.Generator().manual_seed(1)).half()
            d = ops.linear_w6ax(x.to(dev), img, N, meta["abits"])
            xq, xs = oracle.quantize_engine(x.numpy(), meta["abits"])
            wq, wsr = oracle.quantize_engine(w_r.numpy(), 6)
            ref, _, mag = oracle.gemm(xq, xs, wq, wsr)
            torch.cuda.synchronize()
            assert_gemm_close(d.cpu().numpy(), ref, mag, e["file"])
