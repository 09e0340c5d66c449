"""GPU tests of the operator surface's engine mode: QuantLinear.to_engine() runs the HIP W6Ax
linear and agrees with the oracle on the codes the fake-quant path defines."""
import numpy as np
import pytest
import torch
import torch.nn as nn

from common import assert_gemm_close, oracle
from inputs import act_input, weight_input

from flexq_amd.flexq_quantize import (QuantLinear, build_quant_params, flexqllm, make_arg_parser,
                                      register_scales_and_zeros, set_quant_state, weight_quant_inplace)

pytestmark = pytest.mark.gpu


def wsym():
    return dict(n_bits=6, per_channel_axes=[0], symmetric=True, dynamic_method="per_group", group_size=128,
                disable_zero_point=True)


def asym(bits):
    return dict(n_bits=bits, per_channel_axes=[], symmetric=True, dynamic_method="per_group", group_size=128,
                disable_zero_point=True)


@pytest.mark.parametrize("M,K,N,abits", [(1, 4096, 4096, 6), (16, 1024, 256, 8), (3, 512, 200, 6), (64, 256, 128, 8)])
def test_quantlinear_engine_matches_oracle(dev, M, K, N, abits):
    lin = nn.Linear(K, N, bias=False)
    lin.weight.data = torch.from_numpy(weight_input(N, K, seed=1)).half()
    ql = QuantLinear(lin, wsym(), asym(abits)).to(dev)
    set_quant_state(ql, True, True)
    weight_quant_inplace(ql)            # the reference flow: weights become codes * scale
    register_scales_and_zeros(ql)
    x = torch.from_numpy(act_input(M, K, seed=2)).half().to(dev)
    with torch.no_grad():
        y_fake = ql(x).float()
        ql.to_engine()
        y = ql(x)
    torch.cuda.synchronize()
    scales = ql.weight_quantizer.scales.float()  # [N*K/128, 1], row-major groups
    wq = (ql.weight.float().reshape(-1, 128) / scales).round().reshape(N, K).to(torch.int8).cpu().numpy()
    ws = scales.reshape(N, K // 128).t().contiguous().half().cpu().numpy()
    xq, xs = oracle.quantize_engine(x.cpu().numpy(), abits)
    ref, _, mag = oracle.gemm(xq, xs, wq, ws)
    assert_gemm_close(y.cpu().numpy(), ref, mag, f"QuantLinear engine M={M} N={N} K={K}")
    # and the serving arithmetic stays close to the fake-quant accuracy path
    rel = (y.float() - y_fake).norm() / y_fake.norm()
    assert rel < 0.03, float(rel)


def test_quantlinear_engine_rejects_what_it_cannot_run(dev):
    lin = nn.Linear(256, 64, bias=True).half().to(dev)
    ql = QuantLinear(lin, wsym(), asym(6))
    ql.to_engine()
    x = torch.randn(2, 256, device=dev, dtype=torch.float16)
    y = ql(x)
    assert y.shape == (2, 64)
    with pytest.raises(ValueError):
        ql(x.float())
    bad = QuantLinear(lin, wsym(), dict(n_bits=6, symmetric=False, dynamic_method="per_group", group_size=128))
    with pytest.raises(ValueError):
        bad.to_engine()


def test_flexqllm_engine_mode(dev):
    from test_flexq_quantize import _Tiny
    model = _Tiny(256, 384, 2).half().to(dev)
    args = build_quant_params(make_arg_parser().parse_args(
        "--wbits 6 --abits 6 --w_group_size 128 --a_group_size 128 --symmetric --flex_linear_quant --engine".split()))
    flexqllm(model, args)
    layer = model.model.layers[1]
    assert layer.mlp.down_proj.engine and layer.self_attn.q_proj.engine
    x = torch.randn(1, 256, device=dev, dtype=torch.float16)
    h = layer.mlp.down_proj(layer.mlp.gate_proj(x))
    torch.cuda.synchronize()
    assert h.shape == (1, 256) and torch.isfinite(h).all()
