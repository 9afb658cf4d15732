"""leo_erasure_amd — MI355X-native erasure-coding engine for leo_erasure.

Drop-in for the encode / decode / repair hot path of leo-project/leo_erasure
(c_src/{rscoding,cauchycoding,liberationcoding,irscoding}.cpp behind
c_src/leo_erasure_nif.cpp).  The engine is libleoec.so (HIP kernels for
gfx950 + C++ host, C ABI in include/leoec.h); this package mirrors the
reference's Erlang API over it (``api``) and exposes the batched
device-resident entry points (``device``).
"""
from ._lib import LeoecError, lib, strerror, version  # noqa: F401
from .api import (  # noqa: F401
    CODING_CLASS_CAUCHYRS, CODING_CLASS_ISA_VANDRS, CODING_CLASS_LIBERATION,
    CODING_CLASS_VANDRS, DEF_CODING_CLASS, DEF_CODING_PARAMS, decode, encode,
    env_default_coder, gf_init, layout, nif_decode, nif_encode, nif_repair, repair,
    set_default_coder, write_blocks, encode_file, decode_file,
)
from . import device  # noqa: F401

__all__ = [
    "encode", "decode", "repair", "gf_init", "layout", "nif_encode", "nif_decode", "nif_repair",
    "set_default_coder", "env_default_coder", "device", "LeoecError", "version",
    "write_blocks", "encode_file", "decode_file",
]
