"""ctypes binding of libleoec.so, the C-ABI engine (include/leoec.h).

The engine is native code: HIP kernels for gfx950 plus the C++ host side.
There is no Python or CPU fallback for the data path — if the library is
missing, importing this package fails loudly, and if no gfx950 device is
present the data-path calls return LEOEC_E_NO_DEVICE.
"""
import ctypes
import os

try:  # share torch's HIP runtime when torch is present (same soname, loaded first)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the host API
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libleoec.so")

CAUCHYRS, VANDRS, LIBERATION, ISARS = 1, 2, 3, 4
CODING_IDS = {"cauchyrs": CAUCHYRS, "vandrs": VANDRS, "liberation": LIBERATION, "isars": ISARS}

OK = 0
E_INVALID_CODING = -1
E_NOT_ENOUGH_BLOCKS = -9
E_NOT_UNIQUE = -10
E_NO_DEVICE = -16

# Every symbol declared in include/leoec.h (tests check the export table).
EXPORTS = (
    "leoec_strerror", "leoec_gf_init", "leoec_check_params", "leoec_layout", "leoec_encode",
    "leoec_decode", "leoec_repair", "leoec_encode_dev", "leoec_decode_dev", "leoec_repair_dev",
    "leoec_coding_matrix", "leoec_device", "leoec_version",
)


class LeoecError(Exception):
    """A negative leoec_status; str() is the reference's message text."""

    def __init__(self, code):
        self.code = code
        super().__init__(strerror(code))


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build the HIP engine first "
            "(python -c 'import __graft_entry__ as g; g.build()' or make -C leo_erasure_amd/csrc)")
    L = ctypes.CDLL(LIB_PATH)
    c_int, u64 = ctypes.c_int, ctypes.c_uint64
    vp, u8p = ctypes.c_void_p, ctypes.c_void_p
    L.leoec_strerror.restype = ctypes.c_char_p
    L.leoec_strerror.argtypes = [c_int]
    L.leoec_version.restype = ctypes.c_char_p
    L.leoec_gf_init.argtypes = []
    L.leoec_device.argtypes = []
    L.leoec_check_params.argtypes = [c_int] * 4
    L.leoec_layout.argtypes = [c_int] * 4 + [u64, ctypes.POINTER(u64), ctypes.POINTER(c_int)]
    L.leoec_encode.argtypes = [c_int] * 4 + [u8p, u64, u8p, u64]
    L.leoec_decode.argtypes = [c_int] * 4 + [ctypes.POINTER(vp), ctypes.POINTER(c_int), c_int, u64,
                                             u64, u8p]
    L.leoec_repair.argtypes = [c_int] * 4 + [ctypes.POINTER(vp), ctypes.POINTER(c_int), c_int, u64,
                                             ctypes.POINTER(c_int), c_int, u8p]
    L.leoec_encode_dev.argtypes = [c_int] * 4 + [vp, u64, u64, u64, vp, u64, vp]
    L.leoec_decode_dev.argtypes = [c_int] * 4 + [vp, u64, u64, u64, vp, u64,
                                                 ctypes.POINTER(c_int), c_int, vp]
    L.leoec_repair_dev.argtypes = [c_int] * 4 + [ctypes.POINTER(vp), u64, u64, u64,
                                                 ctypes.POINTER(c_int), c_int, ctypes.POINTER(vp),
                                                 u64, vp]
    L.leoec_coding_matrix.argtypes = [c_int] * 4 + [ctypes.POINTER(ctypes.c_uint32), c_int,
                                                    ctypes.POINTER(c_int)]
    return L


lib = _load()


def strerror(code):
    return lib.leoec_strerror(code).decode("latin-1")


def check(rc):
    if rc != OK:
        raise LeoecError(rc)
    return rc


def version():
    return lib.leoec_version().decode()
