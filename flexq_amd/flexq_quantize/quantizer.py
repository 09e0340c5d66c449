"""UniformAffineQuantizer -- FlexQ's fake-quant operator (algorithm/flexq_quantize/quantizer.py:37-177).

Same constructor, attributes and arithmetic as the reference, so `QuantLinear`/`flexqllm` code and
checkpoints written against it keep working; golden vectors generated from the reference pin the
behaviour (tests/test_flexq_quantize.py).  What this module adds is the bridge to the HIP engine:
`codes_and_scales()` returns the integer codes and per-group scales that the fake-quant path
represents, which `fq_pack_w6` turns into the engine's weight image.
"""
import torch
import torch.nn as nn

CLIPMIN = 1e-5
_METHODS = ("per_token", "per_channel", "per_group")


def round_ste(x: torch.Tensor):
    """Rounding with a straight-through gradient.  Kept as (round(x) - x) + x, not round(x): the
    float result differs in the sign of zero (-0 -> +0), and the reference's codes carry that."""
    return (x.round() - x).detach() + x


def _as_groups(x, group_size, deficiency=0):
    """[*, K] -> [-1, group_size] rows (2-D input; a leading batch dim of 1 is dropped), with the
    reference's zero padding of `deficiency` columns."""
    if deficiency:
        x = torch.cat((x, x.new_zeros((x.shape[0], deficiency))), dim=1)
    return x.reshape(-1, group_size)


class UniformAffineQuantizer(nn.Module):
    def __init__(self, n_bits: int = 8, symmetric: bool = False, per_channel_axes=(), metric="minmax",
                 dynamic=False, dynamic_method="per_group", group_size=None, shape=None,
                 disable_zero_point=False, flex_quant=False):
        super().__init__()
        self.symmetric = symmetric
        self.disable_zero_point = disable_zero_point
        self.flex_quant = flex_quant
        self.per_channel_axes = list(per_channel_axes)
        self.metric = metric
        self.dynamic = dynamic
        self.dynamic_method = dynamic_method
        self.group_size = group_size
        self.deficiency = 0
        self.enable = True
        self.scale = None
        self.zero_point = None
        self.round_zero_point = None
        self.cached_xmin = None
        self.cached_xmax = None
        self.sigmoid = nn.Sigmoid()
        self.change_n_bits(n_bits)

    # ------------------------------------------------------------------ configuration
    def change_n_bits(self, n_bits):
        """Signed range when there is no zero point, unsigned [0, 2^b - 1] otherwise."""
        self.n_bits = n_bits
        if self.disable_zero_point:
            self.qmin, self.qmax = -(2 ** (n_bits - 1)), 2 ** (n_bits - 1) - 1
        else:
            self.qmin, self.qmax = 0, 2 ** n_bits - 1

    # ------------------------------------------------------------------ math
    def per_token_dynamic_calibration(self, x):
        """Scale (and zero point) per row, or per `group_size` chunk of a row
        (reference quantizer.py:144-171)."""
        if self.group_size:
            x = _as_groups(x, self.group_size, self.deficiency)
        lo = x.amin([-1], keepdim=True)
        hi = x.amax([-1], keepdim=True)
        if self.symmetric:
            peak = torch.max(hi.abs(), lo.abs())
            self.scale = (peak / (2 ** (self.n_bits - 1) - 1)).clamp(min=CLIPMIN, max=1e4)
            zero_point = (2 ** (self.n_bits - 1) - 1) * torch.ones_like(self.scale)
        else:
            levels = 2 ** self.n_bits if self.n_bits in (1, 2) else 2 ** self.n_bits - 1
            self.scale = ((hi - lo) / levels).clamp(min=CLIPMIN, max=1e4)
            zero_point = -lo / self.scale
        self.round_zero_point = None if self.disable_zero_point else zero_point.clamp(min=-1e4, max=1e4).round()

    def _codes(self, x, scale, round_zero_point):
        q = round_ste(x / scale)
        if round_zero_point is not None:
            q = q.add(round_zero_point)
        return q.clamp(self.qmin, self.qmax)

    def fake_quant(self, x, scale, round_zero_point):
        """x -> dequantize(quantize(x)) with the given scale / zero point (quantizer.py:93-125)."""
        squeezed = False
        if self.group_size:
            if x.dim() == 3 and x.shape[0] == 1:
                squeezed, x = True, x.squeeze(0)
            assert x.dim() == 2, "only support linear layer now"
            rows, cols = x.shape
            if self.deficiency:
                x = torch.cat((x, x.new_zeros((rows, self.deficiency))), dim=1)
            x = x.reshape(-1, self.group_size)
        y = self._codes(x, scale, round_zero_point)
        if round_zero_point is not None:
            y = y.sub(round_zero_point)
        y = y.mul(scale)
        if self.group_size:
            y = y.reshape(rows, -1)
            if self.deficiency:
                y = y[:, :-self.deficiency]
            if squeezed:
                y = y.unsqueeze(0)
        return y

    def forward(self, x: torch.Tensor):
        if self.n_bits >= 16 or not self.enable:
            return x
        if self.metric == "fix0to1":
            x = x.mul_(2 ** self.n_bits - 1).round_().div_(2 ** self.n_bits - 1)
            if not self.flex_quant:
                return x
        if self.dynamic_method not in _METHODS:
            raise NotImplementedError(self.dynamic_method)
        self.per_token_dynamic_calibration(x)
        return self.fake_quant(x, self.scale, self.round_zero_point)

    def register_scales_and_zeros(self):
        """Move the calibrated scale / zero point into buffers `scales` / `zeros` (the form
        checkpoints carry; quantizer.py:173-177)."""
        self.register_buffer("scales", self.scale)
        self.register_buffer("zeros", self.round_zero_point)
        del self.scale
        del self.round_zero_point

    # ------------------------------------------------------------------ engine bridge
    def engine_compatible(self, n_bits=(6,)):
        """True when the integer form is what the HIP engine computes with: symmetric signed
        codes (no zero point), dynamic groups of 128."""
        return (self.disable_zero_point and self.group_size == 128 and self.n_bits in n_bits
                and self.dynamic_method == "per_group" and self.metric == "minmax" and self.enable)

    @torch.no_grad()
    def codes_and_scales(self, w: torch.Tensor, scales: torch.Tensor = None):
        """Integer codes int8 [N, K] and group scales [K/128, N] of a weight [N, K] under this
        quantizer (calibrated on `w` unless `scales` [N*K/128, 1] is given, e.g. the registered
        buffer after weight_quant_inplace).  Codes are the fake-quant path's own: w_hat = codes *
        scale."""
        assert self.engine_compatible(n_bits=(self.n_bits,)), "needs symmetric per-group-128 codes"
        N, K = w.shape
        if scales is None:
            self.per_token_dynamic_calibration(w)
            scales = self.scale
        g = _as_groups(w, self.group_size)
        codes = self._codes(g, scales, None).reshape(N, K).to(torch.int8)
        return codes, scales.reshape(N, K // self.group_size).t().contiguous()
