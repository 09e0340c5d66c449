"""FlexQ's Python operator surface (algorithm/flexq_quantize), with the HIP W6Ax engine behind
QuantLinear.to_engine() / utils.pack_for_engine()."""
from .quantizer import CLIPMIN, UniformAffineQuantizer, round_ste
from .int_linear import QuantLinear
from .int_matmul import QuantMatMul
from .utils import (register_scales_and_zeros, set_quant_state, weight_quant_inplace, smooth_and_quant_temporary,
                    clear_temp_variable, pack_for_engine)
from .config import build_quant_params, make_arg_parser
from .flexqllm import flexqllm

__all__ = ["CLIPMIN", "UniformAffineQuantizer", "round_ste", "QuantLinear", "QuantMatMul",
           "register_scales_and_zeros", "set_quant_state", "weight_quant_inplace", "smooth_and_quant_temporary",
           "clear_temp_variable", "pack_for_engine", "build_quant_params", "make_arg_parser", "flexqllm"]
