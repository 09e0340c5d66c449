"""flexqllm -- quantize a LLaMA / OPT style model layer by layer (algorithm/flexq_quantize/flexqllm.py:48-122).

The reference swaps each decoder layer for its own QuantLlamaDecoderLayer / QuantOPTDecoderLayer
wrappers (algorithm/models/, out of scope here).  This version swaps the linears inside the
existing layers for QuantLinear with the same bit assignment (int_llama_layer.py:31-94: every
projection takes act_quant_params, down_proj / fc2 take act_down_proj_quant_params under
--flex_linear_quant), then runs the reference's sequence: set_quant_state(True, True),
weight_quant_inplace, half(), register_scales_and_zeros.  With args.engine the quantized linears
are moved onto the HIP W6Ax engine.
"""
import torch
import torch.nn as nn

from .int_linear import QuantLinear
from .utils import pack_for_engine, register_scales_and_zeros, set_quant_state, weight_quant_inplace

DOWN_NAMES = ("down_proj", "fc2")   # the W6A8 projections (main.py:202, int_llama_layer.py:35-37)


def decoder_layers(model):
    """(layers, family) of a HF causal LM: LLaMA-style model.model.layers, OPT model.model.decoder.layers."""
    inner = getattr(model, "model", model)
    if hasattr(inner, "layers"):
        return inner.layers, "llama"
    if hasattr(inner, "decoder") and hasattr(inner.decoder, "layers"):
        return inner.decoder.layers, "opt"
    raise ValueError("Only support for llama/Llama-2 and OPT style models now")


def quantize_layer_linears(layer, args):
    """Replace every nn.Linear below `layer` by a QuantLinear; returns the number replaced."""
    swaps = []
    for name, m in layer.named_modules():
        for child_name, child in m.named_children():
            if isinstance(child, nn.Linear) and not isinstance(child, QuantLinear):
                act = args.act_down_proj_quant_params if (args.flex_linear_quant and child_name in DOWN_NAMES) \
                    else args.act_quant_params
                swaps.append((m, child_name, QuantLinear(child, args.weight_quant_params, act)))
    for parent, child_name, q in swaps:
        setattr(parent, child_name, q)
    return len(swaps)


@torch.no_grad()
def flexqllm(lm, args, logger=None):
    model = getattr(lm, "model", lm)
    dev = getattr(lm, "device", None) or next(model.parameters()).device
    layers, _ = decoder_layers(model)
    use_cache = getattr(getattr(model, "config", None), "use_cache", None)
    if use_cache is not None:
        model.config.use_cache = False
    for i in range(len(layers)):
        if logger:
            logger.info(f"=== Start quantize layer {i} ===")
        layer = layers[i].to(dev)
        quantize_layer_linears(layer, args)
        set_quant_state(layer, weight_quant=True, act_quant=True)
        weight_quant_inplace(layer, args)
        layer.half()
        register_scales_and_zeros(layer)
        if getattr(args, "engine", False):
            pack_for_engine(layer, strict=False)
        layers[i] = layer
    if use_cache is not None:
        model.config.use_cache = use_cache
    return model
