"""QuantLinear -- nn.Linear drop-in of FlexQ (algorithm/flexq_quantize/int_linear.py:20-76).

Two execution modes:
  * fake-quant (default): the reference's arithmetic in torch ops -- weight and activation pass
    through their UniformAffineQuantizer, then F.linear.  This is the accuracy path of FlexQ's
    `algorithm/`, reproduced bit-for-bit (golden vectors).
  * engine: `to_engine()` packs the weight once into the HIP engine's image and `forward` runs
    `fq_linear_w6ax` -- dynamic per-group activation quantization + int8-MFMA GEMM + dequant on
    the GPU with the serving engine's arithmetic (e2e .../flexqgemm).  There is no
    silent fallback: the engine mode raises when the extension, the device or the configuration
    does not fit it.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .quantizer import UniformAffineQuantizer


class QuantLinear(nn.Module):
    """Quantized linear layer; set_quant_state() switches weight / activation quantization on."""

    def __init__(self, org_module: nn.Linear, weight_quant_params: dict = None, act_quant_params: dict = None,
                 disable_input_quant=False):
        super().__init__()
        weight_quant_params = dict(weight_quant_params or {})
        act_quant_params = dict(act_quant_params or {})
        self.fwd_kwargs = dict()
        self.fwd_func = F.linear
        self.register_buffer("weight", org_module.weight)
        if org_module.bias is not None:
            self.register_buffer("bias", org_module.bias)
        else:
            self.bias = None
        self.in_features = org_module.in_features
        self.out_features = org_module.out_features
        self.use_weight_quant = False
        self.use_act_quant = False
        self.use_temporary_parameter = False
        self.disable_input_quant = disable_input_quant
        self.weight_quantizer = UniformAffineQuantizer(**weight_quant_params, shape=org_module.weight.shape)
        self.act_quantizer = None if disable_input_quant else UniformAffineQuantizer(**act_quant_params)
        self.engine = False
        self.image = None

    def set_quant_state(self, weight_quant: bool = False, act_quant: bool = False):
        self.use_weight_quant = weight_quant
        self.use_act_quant = act_quant

    # ------------------------------------------------------------------ fake-quant path
    def _fake_quant_forward(self, x):
        if self.use_temporary_parameter:
            weight, bias = self.temp_weight, self.temp_bias
        elif self.use_weight_quant:
            weight, bias = self.weight_quantizer(self.weight), self.bias
        else:
            weight, bias = self.weight, self.bias
        if self.use_act_quant and not self.disable_input_quant:
            x = self.act_quantizer(x)
        return self.fwd_func(x, weight, bias, **self.fwd_kwargs)

    # ------------------------------------------------------------------ engine path
    def engine_ready(self):
        """Whether this layer's configuration is the engine's: W6 g128 symmetric codes and a
        dynamic per-group-128 symmetric A6/A8 activation quantizer."""
        aq = self.act_quantizer
        return (self.weight_quantizer.engine_compatible(n_bits=(6,)) and aq is not None
                and aq.engine_compatible(n_bits=(6, 8)))

    @torch.no_grad()
    def to_engine(self):
        """Pack the (integer-valued) weight into the engine image; forward then runs on the HIP
        engine.  Uses the registered `scales` buffer when weight_quant_inplace +
        register_scales_and_zeros already ran, so the codes are exactly the fake-quant ones."""
        from .. import ops  # the HIP extension: raises FlexQExtensionError when it is missing
        if not self.engine_ready():
            raise ValueError("engine mode needs W6 g128 symmetric weights and A6/A8 g128 symmetric dynamic activations")
        if not self.weight.is_cuda:
            raise ValueError("engine mode needs the layer on a HIP device")
        wq = self.weight_quantizer
        scales = getattr(wq, "scales", None)
        w = self.weight.float()
        codes, ws = wq.codes_and_scales(w, scales.float() if scales is not None else None)
        self.image = ops.pack_w6(codes.contiguous(), ws.to(torch.float16).contiguous())
        self.engine = True
        return self

    def _engine_forward(self, x):
        from .. import ops
        if x.dtype != torch.float16:
            raise ValueError("engine mode computes on fp16 activations (the serving engine's input)")
        lead = x.shape[:-1]
        y = ops.linear_w6ax(x.reshape(-1, self.in_features).contiguous(), self.image, self.out_features,
                            self.act_quantizer.n_bits)
        if self.bias is not None:
            y = y + self.bias.to(y.dtype)
        return y.reshape(*lead, self.out_features)

    def forward(self, input: torch.Tensor):
        if self.engine:
            return self._engine_forward(input)
        return self._fake_quant_forward(input)
