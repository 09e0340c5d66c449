"""ctypes binding of libflexq_hip.so (the C ABI declared in include/flexq_hip.h).

The library is the product path: there is no CPU or eager fallback.  If the shared object is
missing, every op raises `FlexQExtensionError` (build it with `python -c "import
__graft_entry__ as g; g.build()"` or `make -C flexq_amd/csrc`).

torch is imported before the library is loaded so that the HIP runtime torch already mapped
(soname libamdhip64.so.7) is the one our code object registers with.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libflexq_hip.so")
# development A/B only (tools/ab_decode.sh): another build of the same library
if os.environ.get("FLEXQ_AMD_LIB"):
    LIB_PATH = os.path.abspath(os.environ["FLEXQ_AMD_LIB"])

FQ_OK = 0
FQ_ERR_TIMEOUT = 6
_STATUS = {1: "FQ_ERR_NULL", 2: "FQ_ERR_SHAPE", 3: "FQ_ERR_BITS", 4: "FQ_ERR_WORKSPACE", 5: "FQ_ERR_HIP",
           6: "FQ_ERR_TIMEOUT"}


class FlexQExtensionError(RuntimeError):
    """The HIP extension is missing or failed to load."""


class FlexQError(RuntimeError):
    """A C-ABI entry point returned a non-zero fq_status."""

    def __init__(self, fn, status):
        super().__init__(f"{fn} failed: {_STATUS.get(status, status)} ({status})")
        self.status = status


class ChainTimeoutError(FlexQError):
    """FQ_ERR_TIMEOUT: a decode chain's in-kernel wait timed out on this chain workspace earlier; that
    launch's results and every later one's are undefined until ops.chain_reset()."""


P = ctypes.c_void_p
I = ctypes.c_int
SZ = ctypes.c_size_t

# name -> (argtypes, restype)   -- mirrors include/flexq_hip.h
_SIGS = {
    "fq_version": ([], ctypes.c_char_p),
    "fq_abi_version": ([], I),
    "fq_status_string": ([I], ctypes.c_char_p),
    "fq_packed_w_bytes": ([I, I], SZ),
    "fq_gemm_workspace_bytes": ([I, I, I], SZ),
    "fq_workspace_init": ([P, SZ, P], I),
    "fq_pack_w6": ([P, P, I, I, P, P], I),
    "fq_unpack_w6": ([P, I, I, P, P, P], I),
    "fq_quantize_pack_w6": ([P, I, I, P, P, P, P], I),
    "fq_quantize_act": ([P, I, I, I, P, P, P], I),
    "fq_gemm_w6ax": ([P, P, P, I, I, I, I, P, P, P, SZ, P], I),
    "fq_linear_w6ax": ([P, I, I, I, I, P, P, P, P, P, SZ, P], I),
    "fq_linear_act_scratch_bytes": ([I, I, I], SZ),
    "fq_linear_chain_w6ax": ([P, I, I, P, SZ, P, P, P, SZ, P], I),
    "fq_chain_workspace_init": ([P, SZ, P], I),
    "fq_chain_error_offset": ([], SZ),
    "fq_chain_workspace_bytes": ([P, I, I], SZ),
    "fq_chain_bind_status": ([P, SZ, P, P], I),
    "fq_chain_status": ([P], I),
    "fq_chain_reset": ([P, SZ, P], I),
    "fq_ref_bit_packing": ([P, P, I, I, I, P], I),
    "fq_ref_quantize_bit_packing": ([P, P, P, I, I, I, P], I),
    "fq_import_ref_w": ([P, P, I, I, P, P], I),
    "fq_import_ref_x": ([P, P, I, I, I, P, P, P], I),
    "fq_planes_act_scratch_bytes": ([I, I, I], SZ),
    "fq_gemm_w6ax_planes": ([P, P, P, I, I, I, I, P, P, P, P, SZ, P], I),
    "fq_bmma_scratch_bytes": ([I, I, I], SZ),
    "fq_bmma_image_scratch_bytes": ([I, I, I], SZ),
    "fq_rmsnorm_quantize": ([P, P, P, ctypes.c_float, I, I, I, P, P, P, P], I),
    "fq_silu_mul_quantize": ([P, P, I, I, I, I, P, P, P, P], I),
    "fq_layernorm_quantize": ([P, P, P, P, P, P, ctypes.c_float, I, I, I, P, P, P, P], I),
    "fq_prefill_weight_bytes": ([I, I], SZ),
    "fq_linear_w6ax_gather_after": ([P, P, P, I, I, I, I, P, P, P, P, P, SZ, P], I),
    "fq_prefill_unpack_weights": ([P, I, I, P, P], I),
    "fq_gemm_w6ax_u8": ([P, P, P, P, I, I, I, I, P, P, P, SZ, P], I),
    "fq_gemm_w6ax_u8_q": ([P, P, P, P, I, I, I, I, P, P, P, I, I, I, P, SZ, P], I),
    "fq_gemm_q_workspace_bytes": ([I, I, I], SZ),
    "fq_gemm_w6ax_q": ([P, P, P, I, I, I, I, P, P, P, I, I, I, P, SZ, P], I),
    "fq_linear_w6ax_gather": ([P, I, I, I, I, P, P, P, P, P, SZ, P], I),
    "fq_gather_wait": ([P, P, P], I),
    "fq_rmsnorm_linear_scratch_bytes": ([I, I, I], SZ),
    "fq_silu_linear_scratch_bytes": ([I, I, I], SZ),
    "fq_rmsnorm_linear_w6ax": ([P, P, P, P, ctypes.c_float, I, I, I, I, P, P, P, P, P, SZ, P], I),
    "fq_silu_linear_w6ax": ([P, P, I, I, I, I, I, P, P, P, P, P, SZ, P], I),
    "fq_layernorm_linear_scratch_bytes": ([I, I, I], SZ),
    "fq_layernorm_linear_w6ax": ([P, P, P, P, P, P, ctypes.c_float, I, I, I, I, P, P, P, P, P, SZ, P], I),
}


class BmmaState(ctypes.Structure):
    """fq_bmma_state (include/flexq_hip.h; FQBMMAOpState, flexq_bmma_op.h:19-34)."""
    _fields_ = [("init_success", I), ("M", I), ("N", I), ("K", I), ("x_bits", I), ("w_bits", I),
                ("group_size", I), ("w_format", I), ("prepared", I), ("X", P), ("W", P), ("X_SCALE", P),
                ("W_SCALE", P), ("D", P), ("scratch", P), ("scratch_bytes", SZ)]


_STRUCT_SIGS = {
    "fq_bmma_init": ([P, P, P, P, I, I, I, P, I, I, I, I, P, SZ], BmmaState),
    "fq_bmma_init_image": ([P, P, P, I, I, I, P, I, I, I, I, P, SZ], BmmaState),
    "fq_bmma_exec": ([ctypes.POINTER(BmmaState), P], I),
}
EXPORTED = tuple(_SIGS) + tuple(_STRUCT_SIGS)

_lib = None


def load():
    """Load (once) and return the CDLL.  Raises FlexQExtensionError if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise FlexQExtensionError(
            f"{LIB_PATH} not found: the HIP extension is not built (run __graft_entry__.build())")
    try:
        lib = ctypes.CDLL(LIB_PATH)
    except OSError as e:  # pragma: no cover - depends on the box
        raise FlexQExtensionError(f"failed to load {LIB_PATH}: {e}") from e
    ab = LIB_PATH != os.path.join(_HERE, "libflexq_hip.so")  # an older A/B build may lack new entries
    for name, (args, res) in list(_SIGS.items()) + list(_STRUCT_SIGS.items()):
        if ab and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    _lib = lib
    return lib


def call(name, *args):
    """Invoke an fq_status-returning entry point and raise on failure."""
    rc = getattr(load(), name)(*args)
    if rc == FQ_ERR_TIMEOUT:
        raise ChainTimeoutError(name, rc)
    if rc != FQ_OK:
        raise FlexQError(name, rc)


def version():
    return load().fq_version().decode()
