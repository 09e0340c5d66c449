"""The inline-asm LDS reads of the prefill kernels are never touched before their lgkmcnt wait
(tools/lds_hazard_check.py): the compiler takes an asm read's destination as written at the asm
statement, so a spill, copy or reuse of that register ahead of the wait would race the read.  Round 5
met it once: the debug variant of the 256 x 256 kernel spilled x-scale registers still in flight.
CPU-only: compiles fq_gemm.hip to gfx950 assembly (hipcc cross-compiles) and lints it."""
import hashlib
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "flexq_amd", "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _asm():
    srcs = [os.path.join(CSRC, f) for f in ("fq_gemm.hip", "fq_common.h", "fq_lds.h")]
    h = hashlib.sha256(b"".join(open(f, "rb").read() for f in srcs)).hexdigest()[:16]
    out = os.path.join("/tmp", f"fq_gemm_lint_{h}.s")
    if not os.path.exists(out):
        tmp = out + f".{os.getpid()}"
        subprocess.run([HIPCC, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-fno-fast-math",
                        "-fno-slp-vectorize", "-mllvm", "-amdgpu-kernarg-preload-count=16", "--cuda-device-only",
                        "-S", "-I", os.path.join(ROOT, "include"), os.path.join(CSRC, "fq_gemm.hip"), "-o", tmp],
                       check=True, capture_output=True, cwd=CSRC, timeout=600)
        os.replace(tmp, out)
    return out


@pytest.mark.skipif(not shutil.which(HIPCC) and not os.path.exists(HIPCC), reason="hipcc not available")
def test_prefill_kernels_never_touch_an_lds_read_in_flight():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import lds_hazard_check
    r = subprocess.run([sys.executable, lds_hazard_check.__file__, _asm(), "fq_gemm_prefill"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:]
    assert r.stdout.strip().endswith("0 hazard(s)")


@pytest.mark.skipif(not shutil.which(HIPCC) and not os.path.exists(HIPCC), reason="hipcc not available")
def test_no_lds_dma_buffer_load_has_an_immediate_offset():
    """A buffer_load ... lds adds its immediate offset to the LDS destination as well as to the memory
    address (round 5: the second half of each unpacked weight piece landed 1 KiB too far); the kernels
    put every such offset in the SGPR offset instead."""
    import re
    bad = [ln.strip() for ln in open(_asm()) if re.search(r"buffer_load_\w+ .*\boffset:\d+.*\blds\b", ln)]
    assert not bad, bad[:10]
