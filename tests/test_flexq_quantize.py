"""CPU tests of the flexq_quantize operator surface (flexq_amd/flexq_quantize) against golden
vectors generated from the reference package (tests/golden/gen_golden.py), plus the main.py flag
mapping and the model-level helpers.  The engine mode is covered in test_gpu_flexq_quantize.py."""
import argparse
import hashlib
import os

import numpy as np
import pytest
import torch
import torch.nn as nn

from common import ROOT
from inputs import act_input, edge_inputs, weight_input

from flexq_amd.flexq_quantize import (QuantLinear, QuantMatMul, UniformAffineQuantizer, build_quant_params,
                                      flexqllm, make_arg_parser, register_scales_and_zeros, set_quant_state,
                                      weight_quant_inplace)

GOLD = os.path.join(ROOT, "tests", "golden")
DT = {"fp16": torch.float16, "fp32": torch.float32}


def load(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


def sym(bits, group=128):  # main.py --symmetric --a_group_size 128
    return dict(n_bits=bits, per_channel_axes=[], symmetric=True, dynamic_method="per_group",
                group_size=group, disable_zero_point=True)


def wsym():  # main.py --wbits 6 --w_group_size 128 --symmetric
    return dict(n_bits=6, per_channel_axes=[0], symmetric=True, dynamic_method="per_group",
                group_size=128, disable_zero_point=True)


@pytest.mark.parametrize("dname", ["fp16", "fp32"])
@pytest.mark.parametrize("bits", [6, 8])
def test_quantizer_activation_golden(dname, bits):
    g = load(f"act_{dname}_a{bits}.npz")
    x = torch.from_numpy(act_input(16, 1024, seed=11 + bits)).to(DT[dname])
    q = UniformAffineQuantizer(**sym(bits))
    xhat = q(x.clone())
    np.testing.assert_array_equal(q.scale.numpy(), g["scale"])
    np.testing.assert_array_equal(xhat.numpy(), g["xhat"])


@pytest.mark.parametrize("dname", ["fp16", "fp32"])
def test_quantizer_weight_golden_and_codes(dname):
    g = load(f"wq_{dname}.npz")
    w = torch.from_numpy(weight_input(64, 512, seed=7)).to(DT[dname])
    q = UniformAffineQuantizer(**wsym(), shape=w.shape)
    what = q(w.clone())
    np.testing.assert_array_equal(what.numpy(), g["what"])
    codes, ws = q.codes_and_scales(w)
    np.testing.assert_array_equal(codes.numpy().reshape(-1, 128), g["codes"])
    assert tuple(ws.shape) == (512 // 128, 64)
    np.testing.assert_array_equal(ws.t().reshape(-1, 1).numpy(), g["scale"])


@pytest.mark.parametrize("dname", ["fp16", "fp32"])
def test_quantizer_edge_golden(dname):
    g = load(f"edge_{dname}.npz")
    for name, arr in edge_inputs().items():
        x = torch.from_numpy(arr).to(DT[dname])
        for bits in (6, 8):
            q = UniformAffineQuantizer(**sym(bits))
            xhat = q(x.clone())
            np.testing.assert_array_equal(q.scale.numpy(), g[f"{name}_a{bits}_scale"], err_msg=name)
            np.testing.assert_array_equal(xhat.numpy(), g[f"{name}_a{bits}_xhat"], err_msg=name)


@pytest.mark.parametrize("dname", ["fp16", "fp32"])
def test_quantizer_other_configurations_golden(dname):
    """Asymmetric (zero point), per-token, 2-bit, symmetric-with-zero-point, 16-bit passthrough
    and fix0to1: the rest of UniformAffineQuantizer's surface, pinned by the reference."""
    g = load(f"variants_{dname}.npz")
    x = torch.from_numpy(act_input(8, 512, seed=31)).to(DT[dname])
    cases = {
        "asym_g128_a6": dict(n_bits=6, symmetric=False, dynamic_method="per_group", group_size=128),
        "asym_g128_a8": dict(n_bits=8, symmetric=False, dynamic_method="per_group", group_size=128),
        "asym_tok_a8": dict(n_bits=8, symmetric=False, dynamic_method="per_token"),
        "asym_g128_a2": dict(n_bits=2, symmetric=False, dynamic_method="per_group", group_size=128),
        "symzp_g128_a6": dict(n_bits=6, symmetric=True, dynamic_method="per_group", group_size=128),
        "sym_tok_a6": dict(n_bits=6, symmetric=True, dynamic_method="per_token", disable_zero_point=True),
        "a16": dict(n_bits=16, symmetric=False, dynamic_method="per_group", group_size=128),
    }
    for tag, params in cases.items():
        q = UniformAffineQuantizer(**params)
        np.testing.assert_array_equal(q(x.clone()).numpy(), g[f"{tag}_xhat"], err_msg=tag)
        if f"{tag}_scale" in g.files:
            np.testing.assert_array_equal(q.scale.numpy(), g[f"{tag}_scale"], err_msg=tag)
        if f"{tag}_zero" in g.files:
            np.testing.assert_array_equal(q.round_zero_point.numpy(), g[f"{tag}_zero"], err_msg=tag)
    p01 = torch.from_numpy(np.abs(act_input(4, 256, seed=5)) / 8).to(DT[dname]).clamp(0, 1)
    q = UniformAffineQuantizer(n_bits=8, metric="fix0to1")
    np.testing.assert_array_equal(q(p01.clone()).numpy(), g["fix0to1_a8_xhat"])


def test_quantizer_change_bits_and_register():
    q = UniformAffineQuantizer(**sym(6))
    assert (q.qmin, q.qmax) == (-32, 31)
    q.change_n_bits(8)
    assert (q.qmin, q.qmax) == (-128, 127)
    q2 = UniformAffineQuantizer(n_bits=4)
    assert (q2.qmin, q2.qmax) == (0, 15)
    x = torch.randn(2, 256)
    q(x)
    scale = q.scale
    q.register_scales_and_zeros()
    assert torch.equal(q.scales, scale) and q.zeros is None
    assert "scales" in dict(q.named_buffers()) and not hasattr(q, "scale")
    with pytest.raises(NotImplementedError):
        UniformAffineQuantizer(n_bits=6, dynamic_method="static")(x)


@pytest.mark.parametrize("dname", ["fp16", "fp32"])
@pytest.mark.parametrize("M,K,N,abits,tag", [(1, 4096, 4096, 6, "m1"), (16, 1024, 256, 8, "m16a8")])
def test_quantlinear_fakequant_golden(dname, M, K, N, abits, tag):
    g = load(f"linear_{dname}_{tag}.npz")
    lin = nn.Linear(K, N, bias=False)
    lin.weight.data = torch.from_numpy(weight_input(N, K, seed=1)).to(DT[dname])
    ql = QuantLinear(lin, wsym(), sym(abits))
    ql.set_quant_state(True, True)
    x = torch.from_numpy(act_input(M, K, seed=2)).to(DT[dname])
    with torch.no_grad():
        y = ql(x)
        what = ql.weight_quantizer(ql.weight.clone())
    assert hashlib.sha256(what.contiguous().view(torch.uint8).numpy().tobytes()).hexdigest() == str(g["w_hat_sha256"])
    np.testing.assert_array_equal(ql.weight_quantizer.scale.numpy(), g["w_scale"])
    np.testing.assert_array_equal(ql.act_quantizer.scale.numpy(), g["x_scale"])
    # F.linear itself runs on this host's BLAS: equal within the dtype's accumulation noise
    tol = 2e-2 if dname == "fp16" else 1e-4
    np.testing.assert_allclose(y.float().numpy(), g["y"].astype(np.float32), rtol=tol, atol=tol)


def test_quantlinear_states_and_bias():
    lin = nn.Linear(256, 32, bias=True)
    ql = QuantLinear(lin, wsym(), sym(6))
    x = torch.randn(3, 256)
    assert torch.allclose(ql(x), lin(x))  # quantization off by default (reference behaviour)
    ql.set_quant_state(True, False)
    assert not torch.allclose(ql(x), lin(x))
    ql2 = QuantLinear(lin, wsym(), disable_input_quant=True)
    assert ql2.act_quantizer is None
    ql2.set_quant_state(True, True)
    ql2(x)
    assert ql.engine_ready() and not QuantLinear(lin, wsym(), dict(n_bits=6, symmetric=False, group_size=128)).engine_ready()


def test_quantmatmul_16bit_is_identity():
    mm = QuantMatMul(dict(n_bits=16), dict(n_bits=16), matmul_func=torch.matmul)
    set_quant_state(mm, True, True)
    a, b = torch.randn(2, 4, 8), torch.randn(2, 8, 5)
    assert torch.equal(mm(a, b), torch.matmul(a, b))


def parse(argv):
    return build_quant_params(make_arg_parser().parse_args(argv))


def test_flag_mapping_matches_main_py():
    """main.py:222-296: --symmetric implies disable_zero_point; group sizes imply per_group;
    --flex_linear_quant gives A6 everywhere and A8 for down_proj."""
    a = parse("--wbits 6 --abits 6 --w_group_size 128 --a_group_size 128 --symmetric --flex_linear_quant".split())
    assert a.disable_zero_point and a.w_dynamic_method == "per_group" and a.a_dynamic_method == "per_group"
    assert a.weight_quant_params == dict(n_bits=6, per_channel_axes=[0], symmetric=True, dynamic_method="per_group",
                                         group_size=128, disable_zero_point=True)
    grouped = dict(per_channel_axes=[], symmetric=True, dynamic_method="per_group", group_size=128,
                   disable_zero_point=True)
    assert a.act_quant_params == dict(n_bits=6, **grouped)
    assert a.act_down_proj_quant_params == dict(n_bits=8, **grouped)
    assert a.p_quant_params == dict(n_bits=16, metric="fix0to1")
    assert a.q_quant_params["n_bits"] == 16
    b = parse("--wbits 4 --abits 8".split())
    assert not b.disable_zero_point and b.w_dynamic_method == "per_channel"
    assert b.act_quant_params == dict(n_bits=8, per_channel_axes=[], symmetric=False, dynamic_method="per_token")
    assert b.act_down_proj_quant_params["n_bits"] == 8
    assert b.weight_quant_params["group_size"] is None


class _MLP(nn.Module):
    def __init__(self, h, f):
        super().__init__()
        self.gate_proj, self.up_proj, self.down_proj = nn.Linear(h, f, False), nn.Linear(h, f, False), nn.Linear(f, h, False)


class _Attn(nn.Module):
    def __init__(self, h):
        super().__init__()
        self.q_proj, self.k_proj, self.v_proj, self.o_proj = (nn.Linear(h, h, False) for _ in range(4))


class _Layer(nn.Module):
    def __init__(self, h, f):
        super().__init__()
        self.self_attn, self.mlp = _Attn(h), _MLP(h, f)


class _Tiny(nn.Module):  # LLaMA naming: model.model.layers[i].{self_attn,mlp}.*_proj
    def __init__(self, h=256, f=384, n=2):
        super().__init__()
        self.model = nn.Module()
        self.model.layers = nn.ModuleList([_Layer(h, f) for _ in range(n)])


def test_flexqllm_quantizes_every_projection_with_the_bit_map():
    model = _Tiny()
    ref_w = model.model.layers[0].mlp.down_proj.weight.clone()
    args = parse("--wbits 6 --abits 6 --w_group_size 128 --a_group_size 128 --symmetric --flex_linear_quant".split())
    flexqllm(model, args)
    layer = model.model.layers[0]
    for m in (layer.self_attn.q_proj, layer.self_attn.o_proj, layer.mlp.gate_proj, layer.mlp.up_proj):
        assert isinstance(m, QuantLinear) and m.act_quantizer.n_bits == 6 and m.use_act_quant
    down = layer.mlp.down_proj
    assert isinstance(down, QuantLinear) and down.act_quantizer.n_bits == 8
    assert down.weight.dtype == torch.float16 and hasattr(down.weight_quantizer, "scales")
    # weights were fake-quantized in place: exactly codes * scale per group
    q = UniformAffineQuantizer(**wsym())
    expect = q(ref_w.clone()).half()
    assert torch.equal(down.weight, expect)
