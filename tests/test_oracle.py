"""CPU tests of the oracle itself: pinned against the reference's golden vectors and its own KATs.

* Python fake-quant restatement vs tests/golden/*.npz (generated from the reference by
  tests/golden/gen_golden.py): bit-exact scales / codes / x_hat, QuantLinear output within
  fp tolerance.
* Packing KAT mirroring engine/test_packing_kernel.cu:131-148 (FlexQ layout vs ABQ layout).
* The contract GEMM (fqo_gemm) vs the reference's own compute_ref (test_bgemm_kernel.cu:113-146)
  within the reference tolerance (test_kernel.h:59-69) and within 1e-3 relative.
"""
import os

import numpy as np
import pytest
import torch

from common import ROOT, kat_operands, oracle, rng
from inputs import act_input, edge_inputs, weight_input

GOLD = os.path.join(ROOT, "tests", "golden")
DT = {"fp16": torch.float16, "fp32": torch.float32}


def load(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


@pytest.mark.parametrize("dname", ["fp16", "fp32"])
@pytest.mark.parametrize("bits", [6, 8])
def test_act_fakequant_matches_reference(dname, bits):
    g = load(f"act_{dname}_a{bits}.npz")
    x = torch.from_numpy(act_input(16, 1024, seed=11 + bits)).to(DT[dname])
    xhat, scale, codes = oracle.fake_quant_per_group(x, bits)
    np.testing.assert_array_equal(scale.numpy(), g["scale"])
    np.testing.assert_array_equal(codes.to(torch.int8).numpy(), g["codes"])
    np.testing.assert_array_equal(xhat.numpy(), g["xhat"])


@pytest.mark.parametrize("dname", ["fp16", "fp32"])
def test_weight_fakequant_matches_reference(dname):
    g = load(f"wq_{dname}.npz")
    w = torch.from_numpy(weight_input(64, 512, seed=7)).to(DT[dname])
    what, scale, codes = oracle.fake_quant_per_group(w, 6)
    np.testing.assert_array_equal(scale.numpy(), g["scale"])
    np.testing.assert_array_equal(codes.to(torch.int8).numpy(), g["codes"])
    np.testing.assert_array_equal(what.numpy(), g["what"])


@pytest.mark.parametrize("dname", ["fp16", "fp32"])
def test_edge_cases_match_reference(dname):
    g = load(f"edge_{dname}.npz")
    for name, arr in edge_inputs().items():
        x = torch.from_numpy(arr).to(DT[dname])
        for bits in (6, 8):
            xhat, scale, codes = oracle.fake_quant_per_group(x, bits)
            np.testing.assert_array_equal(scale.numpy(), g[f"{name}_a{bits}_scale"], err_msg=name)
            np.testing.assert_array_equal(codes.to(torch.int8).numpy(), g[f"{name}_a{bits}_codes"], err_msg=name)
            np.testing.assert_array_equal(xhat.numpy(), g[f"{name}_a{bits}_xhat"], err_msg=name)


@pytest.mark.parametrize("dname", ["fp16", "fp32"])
@pytest.mark.parametrize("case", [(1, 4096, 4096, 6, "m1"), (16, 1024, 256, 8, "m16a8")])
def test_quant_linear_forward_matches_reference(dname, case):
    M, K, N, abits, tag = case
    g = load(f"linear_{dname}_{tag}.npz")
    w = torch.from_numpy(weight_input(N, K, seed=1)).to(DT[dname])
    x = torch.from_numpy(act_input(M, K, seed=2)).to(DT[dname])
    w_hat, w_scale, _ = oracle.fake_quant_per_group(w, 6)
    np.testing.assert_array_equal(w_scale.numpy(), g["w_scale"])
    import hashlib
    assert hashlib.sha256(w_hat.contiguous().view(torch.uint8).numpy().tobytes()).hexdigest() == str(g["w_hat_sha256"])
    y = oracle.quant_linear_forward(x, w, 6, abits)
    # F.linear's CPU reduction order may differ between hosts; the inputs to it are bit-exact above
    rtol = 2e-3 if dname == "fp16" else 1e-5
    np.testing.assert_allclose(y.float().numpy(), g["y"].astype(np.float32), rtol=rtol,
                               atol=rtol * float(np.abs(g["y"].astype(np.float32)).max()))


# ----------------------------------------------------------------- bit-plane layout KAT

@pytest.mark.parametrize("R,K,bits", [(1, 128, 6), (2, 256, 6), (4, 512, 8), (8, 384, 6), (16, 256, 8), (24, 128, 6)])
def test_packing_kat_flexq_vs_abq(R, K, bits):
    """test_packing_kernel.cu:131-148: ABQ [bits][R][K/32] re-indexed into FlexQ layout."""
    vals = rng(R * K + bits).integers(0, 1 << bits, size=(R, K), dtype=np.int32)
    fq = oracle.pack_bitplanes(vals, bits)
    abq = oracle.pack_abq(vals, bits).view(np.int32)
    chunk = min(R, 8)
    for b in range(bits):
        for m in range(R):
            for kt in range(K // 32):
                idx = (kt // 4) * (R * bits * 4) + (m // chunk) * (bits * chunk * 4) + b * (chunk * 4) + (m % chunk) * 4 + kt % 4
                assert abq[b * (R * K // 32) + m * (K // 32) + kt] == fq[idx]


@pytest.mark.parametrize("R,K,bits", [(1, 128, 6), (3, 256, 6), (8, 512, 8), (32, 256, 6)])
def test_bitplane_roundtrip(R, K, bits):
    v = rng(7).integers(-(1 << (bits - 1)), 1 << (bits - 1), size=(R, K), dtype=np.int32)
    back = oracle.unpack_bitplanes(oracle.pack_bitplanes(v, bits), R, K, bits)
    np.testing.assert_array_equal(back, v)


def test_bitplane_rejects_hazard_rows():
    with pytest.raises(ValueError):
        oracle.pack_bitplanes(np.zeros((12, 128), np.int32), 6)


@pytest.mark.parametrize("N,K", [(32, 128), (64, 384), (40, 256), (1, 128), (17, 128)])
def test_fq6_roundtrip(N, K):
    r = rng(N + K)
    wq = r.integers(-32, 32, size=(N, K)).astype(np.int8)
    ws = (r.random((K // 128, N)) * 0.1).astype(np.float16)
    pk = oracle.pack_fq6(wq, ws)
    assert pk.size == ((N + 15) // 16) * (K // 128) * (1536 + 32)  # codes + blocked scales
    wq2, ws2 = oracle.unpack_fq6(pk, N, K, want_ws=True)
    np.testing.assert_array_equal(wq2, wq)
    np.testing.assert_array_equal(ws2.view(np.uint16), ws.view(np.uint16))
    # the scale region: fp16 [N/16][K/128][16], pad columns 0
    sc = pk[((N + 15) // 16) * (K // 128) * 1536:].view(np.uint16).reshape((N + 15) // 16, K // 128, 16)
    assert sc[0, 0, 0] == ws.view(np.uint16)[0, 0]
    if N % 16:
        assert np.all(sc[-1, :, N % 16:] == 0)


def test_fq6_unpack_rule_gives_4w():
    """The documented register unpack (out_r = P_r & 0xFC.., out_3 from the low bit pairs) yields
    4*w per byte for every lane and k-step of one (tile, group) block [3 planes][64 lanes][2 steps]:
    lane l, step s = the v_mfma_i32_16x16x64_i8 B operand, column l&15, k = 64s + 16(l>>4) + j."""
    wq = rng(3).integers(-32, 32, size=(16, 128)).astype(np.int8)
    pk = oracle.pack_fq6(wq)[:1536].view(np.uint32).reshape(3, 64, 2)
    for s in range(2):
        for lane in range(64):
            p0, p1, p2 = (int(pk[r, lane, s]) for r in range(3))
            o = [p0 & 0xFCFCFCFC, p1 & 0xFCFCFCFC, p2 & 0xFCFCFCFC,
                 ((p0 & 0x03030303) << 2) | ((p1 & 0x03030303) << 4) | ((p2 & 0x03030303) << 6)]
            bts = np.frombuffer(np.array(o, dtype=np.uint32).tobytes(), dtype=np.int8)
            n = lane & 15
            k0 = 64 * s + 16 * (lane >> 4)
            np.testing.assert_array_equal(bts.astype(np.int32), 4 * wq[n, k0:k0 + 16].astype(np.int32))


# ----------------------------------------------------------------- the GEMM contract vs compute_ref

@pytest.mark.parametrize("M,N,K,abits", [(1, 64, 256, 6), (2, 32, 128, 6), (4, 64, 384, 8), (8, 64, 256, 6), (16, 32, 256, 8)])
def test_contract_gemm_vs_reference_compute_ref(M, N, K, abits):
    xraw, wraw, xq, wq, xs, ws = kat_operands(M, N, K, abits, seed=M * 1000 + N + K)
    xp = oracle.pack_bitplanes(xraw, abits)
    wp = oracle.pack_bitplanes(wraw, 6)
    dup = oracle.xs_to_ref_dup(xs, M, K)
    ref = oracle.compute_ref(wp, ws, xp, dup, M, N, K, 6, abits)
    out, acc, mag = oracle.gemm(xq, xs, wq, ws, want_acc=True)
    # the reference's own tolerance (test_kernel.h:64): |d| <= 1e-4 * 65504
    assert np.max(np.abs(out.astype(np.float32) - ref.astype(np.float32))) <= 1e-4 * 65504
    # and 1e-3 relative once compute_ref's own float accumulation noise is budgeted: it adds
    # 36*K signed bit-pair terms into a float, so its error scales with the unsigned magnitude
    # sum_g s_g * sum_k xraw*wraw (random-walk bound, sqrt(#terms) * 2^-24 * 8)
    G = K // 128
    s = xs.astype(np.float64).T[:, None, :] * ws.astype(np.float64).T[None, :, :]
    u = (xraw.astype(np.float64).reshape(M, 1, G, 128) * wraw.astype(np.float64).reshape(1, N, G, 128)).sum(-1)
    noise = np.sqrt(36 * K) * 2.0 ** -24 * 8 * (s * u).sum(-1)
    err = np.abs(out.astype(np.float64) - ref.astype(np.float64))
    assert np.all(err <= 1e-3 * np.abs(ref.astype(np.float64)) + noise)
    # the integer accumulators are exactly the sum of int products
    assert acc.shape == (M, N, K // 128)
    manual = (xq.astype(np.int64).reshape(M, 1, K // 128, 128) * wq.astype(np.int64).reshape(1, N, K // 128, 128)).sum(-1)
    np.testing.assert_array_equal(acc, manual)
    # the unpacked operands are the two's complement reading of the raw patterns
    np.testing.assert_array_equal(oracle.unpack_bitplanes(xp, M, K, abits), xq.astype(np.int32))


def test_engine_quantizer_scales_match_python_scales():
    """engine-style and Python-style scales are bit-identical on fp16 inputs;
    codes differ on a small fraction (fp16 division + tie rule)."""
    x = act_input(16, 4096, seed=5).astype(np.float16)
    for bits, maxfrac in ((6, 0.01), (8, 0.03)):
        q, xs = oracle.quantize_engine(x, bits)
        xhat, scale, codes = oracle.fake_quant_per_group(torch.from_numpy(x), bits)
        np.testing.assert_array_equal(xs.T.reshape(-1), scale.numpy().reshape(-1))
        diff = np.mean(q.reshape(-1) != codes.to(torch.int8).numpy().reshape(-1))
        assert diff < maxfrac
        assert np.all(np.abs(q.astype(np.int32).reshape(-1) - codes.numpy().astype(np.int32).reshape(-1)) <= 1)


def test_engine_quantizer_edge_semantics():
    x = np.zeros((2, 256), np.float16)
    x[0, 128:] = np.float16(1.0)
    x[1, :128] = np.float16(6e-8)  # scale underflows to 0 -> saturating conversion
    q, xs = oracle.quantize_engine(x, 6)
    assert np.all(q[0, :128] == 0) and xs[0, 0] == 0  # all-zero group: NaN path -> 0
    assert np.all(q[0, 128:] == 31)
    assert xs[1, 0] == np.float16(np.float32(1.0) / np.float32(31))  # xs is [K/128][M]
    assert np.all(q[1, :128] == 31)  # x/0 = +inf -> saturate -> clamp to hi


def test_f16_conversion_rounding():
    L = oracle.lib()
    for f, h in ((1.0, 0x3C00), (65504.0, 0x7BFF), (65520.0, 0x7C00), (5.960464477539063e-08, 0x0001),
                 (2.9802322387695312e-08, 0x0000), (1.0 + 2 ** -11, 0x3C00), (1.0 + 3 * 2 ** -11, 0x3C02),
                 (-2.0, 0xC000), (6.097555160522461e-05, 0x03FF), (6.103515625e-05, 0x0400)):
        assert L.fqo_f32_to_f16(f) == h, (f, hex(L.fqo_f32_to_f16(f)), hex(h))
    vals = rng(1).standard_normal(100000).astype(np.float32) * 100
    got = np.array([L.fqo_f32_to_f16(float(v)) for v in vals[:5000]], dtype=np.uint16)
    np.testing.assert_array_equal(got, vals[:5000].astype(np.float16).view(np.uint16))


@pytest.mark.parametrize("hi", [31, 127])
def test_quantizer_division_by_constant_is_exact(hi):
    """The device quantizer replaces absmax / (2^(b-1)-1) by a Newton-corrected product with the
    rounded reciprocal constant; over every fp16 absmax it is bit-identical to IEEE division."""
    assert oracle.check_div_by_const(hi) == 0


@pytest.mark.parametrize("bits", [6, 8])
@pytest.mark.parametrize("rc_ulp", [0, 1, -1, 4, -4])
def test_quantizer_fma_rounding_is_exact(bits, rc_ulp):
    """The device quantizer's element step -- trunc(RN(x * rcb + copysign(0.5, x))) with the
    reciprocal of the fp16 scale biased by 2^-20 -- gives roundf(x / s)'s code for every fp16
    absmax and every element of such a group, whatever the hardware reciprocal's last bits
    (v_rcp_f32 is within 1 ulp; checked to 4)."""
    assert oracle.check_quant_fma(bits, rc_ulp) == 0
