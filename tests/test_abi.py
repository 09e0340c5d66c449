"""CPU checks of the C ABI: the built library loads, exports exactly what include/flexq_hip.h
declares, reports its status strings, and the Python wrappers validate on the host (no GPU
calls here; CPU tensors must be rejected -- there is no CPU path)."""
import ctypes
import os
import re
import subprocess

import pytest
import torch

from common import ROOT

HEADER = os.path.join(ROOT, "include", "flexq_hip.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = set(re.findall(r"\b(fq_[a-z0-9_]+)\s*\(", text))
    return sorted(names - {"fq_stream_t"})


def test_library_exports_every_header_symbol():
    from flexq_amd import _lib
    assert os.path.exists(_lib.LIB_PATH), "build first: __graft_entry__.build()"
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True)
    exported = set(re.findall(r"\bT\s+(fq_\w+)", nm.stdout))
    declared = set(header_functions())
    assert declared, "no declarations parsed"
    assert declared <= exported, f"declared but not exported: {sorted(declared - exported)}"
    assert set(_lib.EXPORTED) == declared, f"ctypes table vs header: {set(_lib.EXPORTED) ^ declared}"


def test_library_loads_and_reports():
    from flexq_amd import _lib
    lib = _lib.load()
    assert b"gfx950" in lib.fq_version()
    for code, word in [(0, b"ok"), (2, b"shape"), (3, b"bit"), (4, b"workspace"), (5, b"HIP")]:
        assert word in lib.fq_status_string(code)
    # size queries are pure host functions
    assert lib.fq_packed_w_bytes(4096, 4096) == 256 * 32 * (1536 + 32)
    assert lib.fq_packed_w_bytes(17, 128) == 2 * 1 * (1536 + 32)
    assert lib.fq_packed_w_bytes(16, 100) == 0  # K % 128
    assert lib.fq_gemm_workspace_bytes(1024, 28672, 4096) == 0  # prefill, many tiles: no split-K slabs
    # few tiles (M = 200, N = 4096: 64 WGs): split-K slabs after the ticket region, fp32 [S][M][Npad]
    ws = lib.fq_gemm_workspace_bytes(200, 4096, 4096)
    assert ws > 256 * 1024 and (ws - 256 * 1024) % (200 * 4096 * 4) == 0
    assert lib.fq_gemm_workspace_bytes(64, 4096, 4096) == 0  # the decode kernel's 64-row tile
    assert lib.fq_gemm_workspace_bytes(96, 4096, 4096) == 0  # two row chunks of 64


def test_null_and_shape_errors_are_status_codes():
    from flexq_amd import _lib
    lib = _lib.load()
    P = ctypes.c_void_p
    assert lib.fq_quantize_act(None, 1, 128, 6, None, None, None) == 1          # FQ_ERR_NULL
    assert lib.fq_quantize_act(P(16), 1, 100, 6, P(16), P(16), None) == 2      # K % 128
    assert lib.fq_quantize_act(P(16), 1, 128, 7, P(16), P(16), None) == 3      # bits
    assert lib.fq_ref_bit_packing(P(16), P(16), 12, 128, 6, None) == 2         # rows 9..15 unsupported
    # the GEMM and the linear: empty or ragged-K shapes, bad bits and null operands are status codes,
    # checked before any device call (an empty M, N or K is FQ_ERR_SHAPE, never an empty launch)
    g = lambda M, N, K, b=6, d=P(16): lib.fq_gemm_w6ax(P(16), P(16), P(16), M, N, K, b, d,  # noqa: E731
                                                        None, None, 0, None)
    assert g(1, 4096, 4096, d=None) == 1
    assert [g(0, 4096, 4096), g(1, 0, 4096), g(1, 4096, 0), g(1, 4096, 100), g(-1, 4096, 4096)] == [2] * 5
    assert g(1, 1 << 21, 4096) == 2                                              # tiles past the ticket region
    assert g(1, 4096, 4096, b=7) == 3
    ln = lambda M, N, K, b=6: lib.fq_linear_w6ax(P(16), M, N, K, b, P(16), P(16), P(16), None, None, 0,  # noqa: E731
                                                 None)
    assert [ln(0, 4096, 4096), ln(1, 0, 4096), ln(1, 4096, 0), ln(1, 4096, 200)] == [2] * 4
    assert ln(1, 4096, 4096, b=4) == 3


def test_missing_extension_fails_loudly():
    """No CPU or eager fallback: with the shared object absent, every op raises
    FlexQExtensionError (a fresh interpreter, so the already-loaded library is not reused)."""
    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "from flexq_amd import _lib\n"
        "_lib.LIB_PATH = '/nonexistent/libflexq_hip.so'\n"
        "from flexq_amd import ops\n"
        "import torch\n"
        "for fn in (lambda: _lib.load(), lambda: _lib.version(),\n"
        "           lambda: ops.act_scratch_bytes(1, 4096, 4096)):\n"
        "    try:\n"
        "        fn()\n"
        "    except _lib.FlexQExtensionError as e:\n"
        "        assert 'not built' in str(e)\n"
        "    else:\n"
        "        raise SystemExit('no error')\n"
        "print('raised')\n" % ROOT)
    r = subprocess.run([os.sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "raised" in r.stdout, r.stdout + r.stderr


def test_wrappers_reject_cpu_tensors():
    from flexq_amd import ops
    with pytest.raises(ValueError, match="HIP device"):
        ops.quantize_act(torch.zeros(1, 128, dtype=torch.float16), 6)
    with pytest.raises(ValueError, match="HIP device"):
        ops.pack_w6(torch.zeros(16, 128, dtype=torch.int8), torch.zeros(1, 16, dtype=torch.float16))


def test_abi_version_matches_header():
    from flexq_amd import _lib
    m = re.search(r"#define FQ_ABI_VERSION (\d+)", open(HEADER).read())
    assert m and _lib.load().fq_abi_version() == int(m.group(1))


def test_fqbmma_instances_exported_with_reference_names():
    """include/flexq_bmma_op.hpp: the eight FQBMMA init/exec function pointers the reference's
    FLEXQGEMMWrapper names (flexq_gemm_wrapper.cu:53-84) are data symbols of the library, under the
    reference's FQ_NAME_FUN spelling (common/base.h:286-289), so its wrapper links unchanged."""
    from flexq_amd import _lib
    hpp = open(os.path.join(ROOT, "include", "flexq_bmma_op.hpp")).read()
    names = re.findall(r"FQ_AMD_DECL_INSTANCE\((FQBMMA_\w+)\)", hpp)
    assert len(names) == 8
    for n in names:  # <X_BITS>x<W_BITS>xtrue_<BLOCK>_<WARP>_<MMA>_<NSTAGE>_<STRIDE>
        assert re.fullmatch(r"FQBMMA_[68]x6xtrue_\d+x\d+x\d+_\d+x\d+x\d+_8x8x128_\d_1", n), n
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True)
    data = set(re.findall(r"\b[DdBb]\s+(FQBMMA_\w+)", nm.stdout))
    for n in names:
        assert {n + "_InitFn", n + "_ExecFn"} <= data, n
    funcs = set(re.findall(r"\bT\s+(fq_bmma_op_\w+)", nm.stdout))
    assert {"fq_bmma_op_forget_weight", "fq_bmma_op_device_bytes"} <= funcs


def test_chain_host_side():
    """fq_linear_chain_w6ax's host contract (no GPU calls): the ctypes link struct matches the
    header's layout, the chain workspace is the sync block plus one hand-off region per link whose
    output the next link reads (4 B per output element, 256-B rounded) plus one per RMSNorm link with
    an input (its residual output's granules), and bad arguments are status codes."""
    from flexq_amd import _lib, ops
    lib = _lib.load()
    L = ops._ChainLink
    assert ctypes.sizeof(L) == 72
    assert [L.N.offset, L.pro.offset, L.in_.offset, L.gamma.offset, L.eps.offset, L.ldh.offset] == [24, 36, 40, 48, 64, 68]
    sync = 4096
    links = (L * 3)()
    for i, (n, k) in enumerate([(4096, 4096), (22016, 4096), (4096, 11008)]):
        links[i].N, links[i].K, links[i].abits = n, k, 6
    assert lib.fq_chain_workspace_bytes(links, 3, 1) == sync + 4096 * 4 + 22016 * 4
    assert lib.fq_chain_workspace_bytes(links, 3, 3) == sync + 3 * 4096 * 4 + ((3 * 22016 * 4 + 255) // 256) * 256
    links[1].pro, links[1].in_ = 1, 16  # an RMSNorm link with an input: + its residual's granules
    assert lib.fq_chain_workspace_bytes(links, 3, 1) == sync + 4096 * 4 + 22016 * 4 + 4096 * 4
    assert lib.fq_chain_workspace_bytes(links, 1, 1) == sync
    assert lib.fq_chain_error_offset() == 4 * 32 * 9
    assert lib.fq_linear_chain_w6ax(None, 1, 1, None, 0, None, None, None, 0, None) == 1  # FQ_ERR_NULL
    assert lib.fq_linear_chain_w6ax(links, 3, 33, None, 0, None, None, None, 0, None) == 2  # M > 32
    assert lib.fq_linear_chain_w6ax(links, 3, 1, None, 0, None, None, None, 0, None) == 1  # null x / w / d
    assert lib.fq_chain_workspace_init(None, 0, None) == 0
    assert lib.fq_chain_workspace_init(None, 64, None) == 1


def test_prefill_quantized_output_host_checks():
    """fq_gemm_w6ax_u8_q's host-side validation (no GPU calls): null next-input buffers, a next
    input that is not a prefix of the output or has K % 128 != 0, bad bits, and next-input buffers
    overlapping the operands or the output are status codes."""
    from flexq_amd import _lib
    lib = _lib.load()
    P = ctypes.c_void_p
    M, N, K = 4096, 4096, 4096
    xq, xs, w, wu, d = P(1 << 32), P(2 << 32), P(3 << 32), P(4 << 32), P(5 << 32)
    qx, qs = P(6 << 32), P(7 << 32)
    call = lambda qxq, qxs, qM, qK, qb: lib.fq_gemm_w6ax_u8_q(xq, xs, w, wu, M, N, K, 8, d, qxq, qxs, qM, qK, qb,  # noqa: E731
                                                                None, 0, None)
    assert call(None, qs, M, K, 8) == 1
    assert call(qx, qs, M, 100, 8) == 2
    assert call(qx, qs, 2 * M, N, 8) == 2          # more than the output holds
    assert call(qx, qs, M, K, 7) == 3
    assert call(xq, qs, M, K, 8) == 2              # codes over the operand codes
    assert call(qx, P(5 << 32), M, K, 8) == 2      # scales over the output


def test_decode_quantized_output_host_checks():
    """fq_gemm_w6ax_q (the next input's codes from the decode GEMM's epilogue): the same host-side
    validation as fq_gemm_w6ax_u8_q before any device call, and its workspace -- the group tickets on
    top of the GEMM's own -- only where the one-launch form runs (M <= 16, N % 128 == 0, no k-split)."""
    from flexq_amd import _lib
    lib = _lib.load()
    P = ctypes.c_void_p
    M, N, K = 16, 4096, 4096
    xq, xs, w, d = P(1 << 32), P(2 << 32), P(3 << 32), P(5 << 32)
    qx, qs = P(6 << 32), P(7 << 32)
    call = lambda qxq, qxs, qM, qK, qb, ab=6: lib.fq_gemm_w6ax_q(xq, xs, w, M, N, K, ab, d, qxq, qxs, qM, qK, qb,  # noqa: E731
                                                                   None, 0, None)
    assert lib.fq_gemm_w6ax_q(None, xs, w, M, N, K, 6, d, qx, qs, M, K, 6, None, 0, None) == 1
    assert call(None, qs, M, K, 6) == 1
    assert call(qx, qs, M, 100, 6) == 2
    assert call(qx, qs, 2 * M, N, 6) == 2           # more than the output holds
    assert call(qx, qs, M, K, 7) == 3
    assert call(qx, qs, M, K, 6, ab=5) == 3
    assert call(xq, qs, M, K, 6) == 2               # codes over the operand codes
    assert call(qx, P(5 << 32), M, K, 6) == 2       # scales over the output
    tickets = lib.fq_gemm_q_workspace_bytes(1, 12288, 4096)
    assert tickets >= 4 * (12288 // 128) and lib.fq_gemm_workspace_bytes(1, 12288, 4096) == 0
    assert lib.fq_gemm_q_workspace_bytes(16, 22016, 4096) == tickets
    assert lib.fq_gemm_q_workspace_bytes(17, 4096, 4096) == lib.fq_gemm_workspace_bytes(17, 4096, 4096)
    assert lib.fq_gemm_q_workspace_bytes(16, 4112, 4096) == lib.fq_gemm_workspace_bytes(16, 4112, 4096)
    assert lib.fq_gemm_q_workspace_bytes(16, 4096, 100) == 0
