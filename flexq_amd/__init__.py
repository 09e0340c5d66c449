"""flexq_amd -- MI355X-native (gfx950) W6Ax quantized-linear engine.

Layers:
  include/flexq_hip.h + csrc/*.hip  the C ABI and its HIP kernels (libflexq_hip.so)
  flexq_amd._lib / flexq_amd.ops    ctypes binding and torch-facing wrappers
  flexq_amd.flexq_quantize          FlexQ's Python operator surface (QuantLinear drop-in ...)
  flexq_amd.dist                    column-parallel sharding with one RCCL all-gather
  flexq_amd.convert                 offline converter, .fqw6 packed-weight files
  flexq_amd.layers                  W6Linear, FlexQFfn (FT FfnLayer int8_mode 5)
"""
__version__ = "0.1.0"

from ._lib import ChainTimeoutError, FlexQError, FlexQExtensionError  # noqa: F401
