"""QuantMatMul -- activation-activation matmul with optional fake quantization of both operands
(algorithm/flexq_quantize/int_matmul.py:21-61).  FlexQ runs attention matmuls at 16 bits
(main.py:297-319), i.e. these quantizers are identities in the shipped configuration."""
import torch
import torch.nn as nn

from .quantizer import UniformAffineQuantizer


class QuantMatMul(nn.Module):
    def __init__(self, x1_quant_params: dict = None, x2_quant_params: dict = None, disable_act_quant=False,
                 matmul_func=torch.bmm):
        super().__init__()
        self.use_act_quant = False
        self.use_weight_quant = False
        self.x1_quantizer = UniformAffineQuantizer(**dict(x1_quant_params or {}))
        self.x2_quantizer = UniformAffineQuantizer(**dict(x2_quant_params or {}))
        self.matmul_func = matmul_func
        self.x1_qunat_flag = False  # (sic) attribute names of the reference, kept for state compatibility
        self.x2_qunat_flag = False
        self.disable_act_quant = disable_act_quant

    def set_quant_state(self, weight_quant: bool = False, act_quant: bool = False):
        self.use_weight_quant = weight_quant
        self.use_act_quant = act_quant

    def quant_x1(self, x1):
        return self.x1_quantizer(x1) if self.use_act_quant else x1

    def quant_x2(self, x2):
        return self.x2_quantizer(x2) if self.use_act_quant else x2

    def forward(self, x1, x2):
        return self.matmul_func(self.quant_x1(x1), self.quant_x2(x2))
