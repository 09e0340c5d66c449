"""Model-level helpers of FlexQ's flexq_quantize package (algorithm/flexq_quantize/utils.py:14-131):
quant-state switches, in-place weight quantization, scale registration, and the parameter
filters used by the (out-of-scope) calibration loop.  `pack_for_engine` is this build's addition:
it moves every eligible QuantLinear onto the HIP engine."""
from collections import OrderedDict

import torch

from .int_linear import QuantLinear
from .int_matmul import QuantMatMul


def _params_matching(model, *keys):
    return iter([p for n, p in model.named_parameters() if any(k in n for k in keys)])


def let_parameters(model, use_shift=True):
    return _params_matching(model, "smooth" if use_shift else "smooth_scale")


def com_parameters(model, use_shift=True):
    return _params_matching(model, "compensation")


def lwc_parameters(model):
    return _params_matching(model, "bound_factor")


def get_abq_parameters(model, use_shift=True):
    return _params_matching(model, "bound_factor", "smooth" if use_shift else "smooth_scale", "compensation")


def abq_state_dict(model, destination=None, prefix="", keep_vars=False):
    destination = OrderedDict() if destination is None else destination
    for name, param in model.named_parameters():
        if "smooth" in name or "bound_factor" in name:
            destination[prefix + name] = param if keep_vars else param.detach()
    return destination


def register_scales_and_zeros(model):
    for m in model.modules():
        if isinstance(m, QuantLinear):
            m.weight_quantizer.register_scales_and_zeros()


class TruncateFunction(torch.autograd.Function):
    """Push |x| < threshold to sign(x) * threshold (AMP overflow guard); identity gradient."""

    @staticmethod
    def forward(ctx, input, threshold):
        out = input.clone()
        small = out.abs() < threshold
        out[small] = out[small].sign() * threshold
        return out

    @staticmethod
    def backward(ctx, grad_output):
        return grad_output.clone(), None


def truncate_number(number, threshold=1e-2):
    return TruncateFunction.apply(number, threshold)


def smooth_and_quant_temporary(model, args=None, isllama=None):
    """Quantize every QuantLinear's weight into temp_weight (plus an optional low-rank
    `<name>_compensation_left @ _right` term registered on the model) and use it."""
    for m in model.modules():
        if isinstance(m, QuantLinear):
            m.temp_weight = m.weight
    for name, m in model.named_modules():
        if not isinstance(m, QuantLinear):
            continue
        w = getattr(m, "temp_weight", m.weight)
        key = name.replace(".", "_")
        if hasattr(model, f"{key}_compensation_left"):
            w = w + getattr(model, f"{key}_compensation_left") @ getattr(model, f"{key}_compensation_right")
        m.temp_weight = m.weight_quantizer(w)
        if not hasattr(m, "temp_bias"):
            m.temp_bias = m.bias
        m.use_temporary_parameter = True


def clear_temp_variable(model):
    for m in model.modules():
        if isinstance(m, QuantLinear):
            for attr in ("temp_weight", "temp_bias"):
                if hasattr(m, attr):
                    delattr(m, attr)


@torch.no_grad()
def weight_quant_inplace(model, args=None, isllama=None):
    """Replace every QuantLinear's weight by its fake-quantized value (calibrating the quantizer)."""
    for m in model.modules():
        if isinstance(m, QuantLinear):
            m.weight = m.weight_quantizer(m.weight)
            m.use_temporary_parameter = False


def set_quant_state(self, weight_quant: bool = False, act_quant: bool = False):
    """Switch weight / activation quantization on every QuantLinear and QuantMatMul below `self`."""
    self.use_weight_quant = weight_quant
    self.use_act_quant = act_quant
    for m in self.modules():
        if isinstance(m, (QuantLinear, QuantMatMul)):
            m.set_quant_state(weight_quant, act_quant)


@torch.no_grad()
def pack_for_engine(model, strict=True):
    """Move every QuantLinear whose configuration the HIP engine implements onto it (to_engine).
    strict: raise if a QuantLinear with active quantization cannot move; otherwise leave it on
    the fake-quant path.  Returns the number of layers moved."""
    moved = 0
    for name, m in model.named_modules():
        if not isinstance(m, QuantLinear) or m.engine:
            continue
        if m.engine_ready():
            m.to_engine()
            moved += 1
        elif strict and (m.use_weight_quant or m.use_act_quant):
            raise ValueError(f"{name}: configuration not supported by the W6Ax engine")
    return moved
