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
    # few tiles (M = 96, N = 4096: 32 WGs): split-K slabs after the ticket region, fp32 [S][M][Npad]
    ws = lib.fq_gemm_workspace_bytes(96, 4096, 4096)
    assert ws > 256 * 1024 and (ws - 256 * 1024) % (96 * 4096 * 4) == 0
    assert lib.fq_gemm_workspace_bytes(64, 4096, 4096) == 0  # two row chunks of the decode kernel


def test_null_and_shape_errors_are_status_codes():
    from flexq_amd import _lib
    lib = _lib.load()
    P = ctypes.c_void_p
    assert lib.fq_quantize_act(None, 1, 128, 6, None, None, None) == 1          # FQ_ERR_NULL
    assert lib.fq_quantize_act(P(16), 1, 100, 6, P(16), P(16), None) == 2      # K % 128
    assert lib.fq_quantize_act(P(16), 1, 128, 7, P(16), P(16), None) == 3      # bits
    assert lib.fq_ref_bit_packing(P(16), P(16), 12, 128, 6, None) == 2         # rows 9..15 unsupported


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
