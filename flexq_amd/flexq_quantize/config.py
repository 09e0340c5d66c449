"""Command-line flags -> quantizer parameter dicts, as FlexQ's main.py builds them
(algorithm/main.py:177-202 flags, :222-319 mapping).  `build_quant_params(args)` fills the same
`args.*_quant_params` attributes; tests pin the dict contents against the reference's rules."""
import argparse


def make_arg_parser():
    p = argparse.ArgumentParser(description="FlexQ quantization flags (main.py subset on the W6Ax path)")
    p.add_argument("--model", type=str)
    p.add_argument("--net", type=str, default=None)
    p.add_argument("--wbits", type=int, default=16)
    p.add_argument("--w_group_size", type=int, default=None)
    p.add_argument("--abits", type=int, default=16)
    p.add_argument("--a_group_size", type=int, default=None)
    p.add_argument("--symmetric", default=False, action="store_true")
    p.add_argument("--disable_zero_point", default=False, action="store_true")
    p.add_argument("--a_dynamic_method", type=str, default="per_token", choices=["per_token", "per_group"])
    p.add_argument("--w_dynamic_method", type=str, default="per_channel", choices=["per_channel", "per_group"])
    p.add_argument("--flex_linear_quant", default=False, action="store_true",
                   help="down_proj uses W6A8, the other linears W6A6")
    p.add_argument("--engine", default=False, action="store_true",
                   help="run eligible QuantLinear layers on the HIP W6Ax engine after quantization")
    return p


def build_quant_params(args):
    """Mutates and returns args: symmetric implies no zero point, a group size implies per-group
    dynamic quantization, then the weight / activation / down_proj / attention parameter dicts."""
    if args.symmetric:
        args.disable_zero_point = True
    if args.w_group_size is not None:
        args.w_dynamic_method = "per_group"
    if args.a_group_size is not None:
        args.a_dynamic_method = "per_group"
    a_bits = args.abits if not args.flex_linear_quant else 6
    down_bits = args.abits if not args.flex_linear_quant else 8
    args.weight_quant_params = {
        "n_bits": args.wbits, "per_channel_axes": [0], "symmetric": args.symmetric,
        "dynamic_method": args.w_dynamic_method, "group_size": args.w_group_size,
        "disable_zero_point": args.disable_zero_point,
    }
    if args.a_group_size:
        grouped = {"per_channel_axes": [], "symmetric": args.symmetric, "dynamic_method": args.a_dynamic_method,
                   "group_size": args.a_group_size, "disable_zero_point": args.disable_zero_point}
        args.act_quant_params = {"n_bits": a_bits, **grouped}
        args.act_down_proj_quant_params = {"n_bits": down_bits, **grouped}
    else:
        plain = {"per_channel_axes": [], "symmetric": False, "dynamic_method": args.a_dynamic_method}
        args.act_quant_params = {"n_bits": a_bits, **plain}
        args.act_down_proj_quant_params = {"n_bits": down_bits, **plain}
    half = {"n_bits": 16, "per_channel_axes": [], "symmetric": args.symmetric, "dynamic_method": args.a_dynamic_method}
    args.q_quant_params = dict(half)
    args.k_quant_params = dict(half)
    args.v_quant_params = dict(half)
    args.p_quant_params = {"n_bits": 16, "metric": "fix0to1"}
    return args
