"""Generate golden vectors from the REFERENCE Python fake-quant path (run in the build container only).

Usage (from the repo root, reference mounted read-only at /root/reference):
    PYTHONPATH=/root/reference/algorithm python tests/golden/gen_golden.py

What it records (all inputs come from numpy's PCG64 with fixed seeds, so they are regenerated
bit-for-bit by tests/golden/inputs.py without the reference):
  * act_{dtype}_a{bits}.npz  -- UniformAffineQuantizer(n_bits, symmetric, per_group g=128,
    disable_zero_point) applied to activations (quantizer.py:128-171): scale, integer codes, x_hat.
  * wq_{dtype}.npz           -- the same quantizer on a weight matrix, as weight_quant_inplace does
    (flexq_quantize/utils.py:116-123).
  * linear_{dtype}_m{M}.npz  -- QuantLinear.forward with use_weight_quant=use_act_quant=True
    (int_linear.py:56-72) for the C1 shape M=1, K=N=4096 and for M=16 W6A8 (down_proj style).
    Large tensors are recorded as sha256 digests plus the output row(s).
  * edge_{dtype}.npz         -- all-zero groups, exact .5 ties, 3-D [1,S,K] input, outliers.

The reference source never leaves this container; only these data files are committed.
"""
import hashlib
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from inputs import act_input, weight_input, edge_inputs  # noqa: E402

from flexq_quantize.quantizer import UniformAffineQuantizer, round_ste  # noqa: E402  (reference)
from flexq_quantize.int_linear import QuantLinear  # noqa: E402  (reference)

DT = {"fp16": torch.float16, "fp32": torch.float32}


def qparams(bits):
    # main.py:273-286 with --symmetric (=> disable_zero_point, main.py:223-224) and a_group_size=128
    return dict(n_bits=bits, per_channel_axes=[], symmetric=True, dynamic_method="per_group",
                group_size=128, disable_zero_point=True)


def wparams():
    # main.py:256-263 with --wbits 6 --w_group_size 128 --symmetric
    return dict(n_bits=6, per_channel_axes=[0], symmetric=True, dynamic_method="per_group",
                group_size=128, disable_zero_point=True)


def run_quantizer(x, params):
    q = UniformAffineQuantizer(**params)
    xhat = q(x.clone())
    scale = q.scale.clone()
    # integer codes through the reference's own ops (fake_quant, quantizer.py:107-112)
    x2 = x.reshape(-1, 128) if x.dim() == 2 else x.squeeze(0).reshape(-1, 128)
    codes = round_ste(x2 / scale).clamp(q.qmin, q.qmax)
    return scale, codes, xhat


def sha(t):
    return hashlib.sha256(t.contiguous().view(torch.uint8).numpy().tobytes()).hexdigest()


def main():
    out = {}
    for dname, dt in DT.items():
        for bits in (6, 8):
            x = torch.from_numpy(act_input(16, 1024, seed=11 + bits)).to(dt)
            scale, codes, xhat = run_quantizer(x, qparams(bits))
            np.savez_compressed(os.path.join(HERE, f"act_{dname}_a{bits}.npz"),
                                scale=scale.numpy(), codes=codes.to(torch.int8).numpy(),
                                xhat=xhat.numpy())
        w = torch.from_numpy(weight_input(64, 512, seed=7)).to(dt)
        scale, codes, what = run_quantizer(w, wparams())
        np.savez_compressed(os.path.join(HERE, f"wq_{dname}.npz"), scale=scale.numpy(),
                            codes=codes.to(torch.int8).numpy(), what=what.numpy())

        # QuantLinear forward: C1 (M=1, K=N=4096, W6A6) and M=16 W6A8 (K=1024, N=256)
        for (M, K, N, abits, tag) in ((1, 4096, 4096, 6, "m1"), (16, 1024, 256, 8, "m16a8")):
            torch.manual_seed(0)
            lin = torch.nn.Linear(K, N, bias=False)
            lin.weight.data = torch.from_numpy(weight_input(N, K, seed=1)).to(dt)
            ql = QuantLinear(lin, wparams(), qparams(abits))
            ql.set_quant_state(True, True)
            x = torch.from_numpy(act_input(M, K, seed=2)).to(dt)
            with torch.no_grad():
                y = ql(x)
                wq_t = ql.weight_quantizer(ql.weight.clone())
            np.savez_compressed(os.path.join(HERE, f"linear_{dname}_{tag}.npz"), y=y.numpy(),
                                w_scale=ql.weight_quantizer.scale.numpy(),
                                w_hat_sha256=np.array(sha(wq_t)),
                                x_scale=ql.act_quantizer.scale.numpy())

        e = {}
        for name, arr in edge_inputs().items():
            x = torch.from_numpy(arr).to(dt)
            for bits in (6, 8):
                scale, codes, xhat = run_quantizer(x, qparams(bits))
                e[f"{name}_a{bits}_scale"] = scale.numpy()
                e[f"{name}_a{bits}_codes"] = codes.to(torch.int8).numpy()
                e[f"{name}_a{bits}_xhat"] = xhat.numpy()
        np.savez_compressed(os.path.join(HERE, f"edge_{dname}.npz"), **e)

        # other quantizer configurations of the operator surface (main.py:222-296 without
        # --symmetric, per-token activations, symmetric with a zero point, fix0to1)
        v = {}
        x = torch.from_numpy(act_input(8, 512, seed=31)).to(dt)
        for tag, params in (
                ("asym_g128_a6", dict(n_bits=6, symmetric=False, dynamic_method="per_group", group_size=128)),
                ("asym_g128_a8", dict(n_bits=8, symmetric=False, dynamic_method="per_group", group_size=128)),
                ("asym_tok_a8", dict(n_bits=8, symmetric=False, dynamic_method="per_token")),
                ("asym_g128_a2", dict(n_bits=2, symmetric=False, dynamic_method="per_group", group_size=128)),
                ("symzp_g128_a6", dict(n_bits=6, symmetric=True, dynamic_method="per_group", group_size=128)),
                ("sym_tok_a6", dict(n_bits=6, symmetric=True, dynamic_method="per_token", disable_zero_point=True)),
                ("a16", dict(n_bits=16, symmetric=False, dynamic_method="per_group", group_size=128))):
            q = UniformAffineQuantizer(**params)
            with torch.no_grad():
                v[f"{tag}_xhat"] = q(x.clone()).numpy()
            if q.scale is not None:
                v[f"{tag}_scale"] = q.scale.numpy()
            if q.round_zero_point is not None:
                v[f"{tag}_zero"] = q.round_zero_point.numpy()
        p01 = torch.from_numpy(np.abs(act_input(4, 256, seed=5)) / 8).to(dt).clamp(0, 1)
        q = UniformAffineQuantizer(n_bits=8, metric="fix0to1")
        with torch.no_grad():
            v["fix0to1_a8_xhat"] = q(p01.clone()).numpy()
        np.savez_compressed(os.path.join(HERE, f"variants_{dname}.npz"), **v)
    print("golden vectors written to", HERE)


if __name__ == "__main__":
    main()
