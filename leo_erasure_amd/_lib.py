"""ctypes binding of libleoec.so, the C-ABI engine (include/leoec.h).

The engine is native code: HIP kernels for gfx950 plus the C++ host side.
There is no Python or CPU fallback for the data path — if the library is
missing, importing this package fails loudly, and if no gfx950 device is
present the data-path calls return LEOEC_E_NO_DEVICE.
"""
import ctypes
import os

# Share torch's HIP runtime when torch is present (same soname, loaded
# first).  LEOEC_NO_TORCH=1 keeps torch out of the process, so the library
# binds the system runtime (its RUNPATH, /opt/rocm) as under an Erlang VM
# loading the NIF: bench.py's host-memory leg runs in such a child process.
torch = None
if os.environ.get("LEOEC_NO_TORCH") != "1":
    try:
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch is optional for the host API
        torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libleoec.so")
# The measurement build (every A/B kernel form, LEOEC_* knobs read once at
# first use, or set with measure_set_knob): `make -C leo_erasure_amd/csrc
# measure`.  Tools and the form-parity tests' own process select it with
# LEOEC_LIBRARY=measure, so a process loads one HIP library.
MEASURE_LIB_PATH = os.path.join(_HERE, "libleoec_measure.so")

CAUCHYRS, VANDRS, LIBERATION, ISARS = 1, 2, 3, 4
CODING_IDS = {"cauchyrs": CAUCHYRS, "vandrs": VANDRS, "liberation": LIBERATION, "isars": ISARS}

OK = 0
E_INVALID_CODING = -1
E_NOT_ENOUGH_BLOCKS = -9
E_NOT_UNIQUE = -10
E_NO_DEVICE = -16
E_HIP = -17

# Every symbol declared in include/leoec.h (tests check the export table).
EXPORTS = (
    "leoec_strerror", "leoec_gf_init", "leoec_check_params", "leoec_layout", "leoec_encode",
    "leoec_decode", "leoec_repair", "leoec_encode_dev", "leoec_decode_dev", "leoec_repair_dev",
    "leoec_coding_matrix", "leoec_device", "leoec_host_lanes", "leoec_host_spread",
    "leoec_version",
)


class LeoecError(Exception):
    """A negative leoec_status; str() is the reference's message text."""

    def __init__(self, code):
        self.code = code
        super().__init__(strerror(code))


_loaded = {}


def _load(path=LIB_PATH):
    if path in _loaded:
        return _loaded[path]
    if not os.path.exists(path):
        raise ImportError(
            f"{path} is missing: build the HIP engine first "
            "(python -c 'import __graft_entry__ as g; g.build()' or make -C leo_erasure_amd/csrc)")
    L = ctypes.CDLL(path)
    c_int, u64 = ctypes.c_int, ctypes.c_uint64
    vp, u8p = ctypes.c_void_p, ctypes.c_void_p
    L.leoec_strerror.restype = ctypes.c_char_p
    L.leoec_strerror.argtypes = [c_int]
    L.leoec_version.restype = ctypes.c_char_p
    L.leoec_gf_init.argtypes = []
    L.leoec_device.argtypes = []
    if hasattr(L, "leoec_host_lanes"):  # (absent from pre-round-3 builds, A/B tools)
        L.leoec_host_lanes.argtypes = [ctypes.POINTER(c_int), c_int]
    if hasattr(L, "leoec_host_spread"):  # (absent from pre-round-4 builds)
        L.leoec_host_spread.argtypes = [ctypes.POINTER(c_int), c_int]
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
    if hasattr(L, "leoec_measure_reload"):
        L.leoec_measure_reload.argtypes = []
        L.leoec_measure_reload.restype = None
        L.leoec_measure_set_knob.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        L.leoec_measure_set_knob.restype = ctypes.c_int
        L.leoec_measure_reset_knobs.argtypes = []
        L.leoec_measure_reset_knobs.restype = None
    if hasattr(L, "leoec_measure_warm_state"):
        L.leoec_measure_warm_state.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        L.leoec_measure_warm_state.restype = None
    if hasattr(L, "leoec_measure_reclaim_state"):
        L.leoec_measure_reclaim_state.argtypes = [ctypes.POINTER(ctypes.c_long)]
        L.leoec_measure_reclaim_state.restype = None
    if hasattr(L, "leoec_measure_xor_pattern_dev"):  # measurement build (xor_pattern.hip)
        L.leoec_measure_xor_pattern_dev.argtypes = [
            ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p,
            ctypes.c_uint64, ctypes.c_void_p]
        L.leoec_measure_xor_pattern_dev.restype = ctypes.c_int
    if hasattr(L, "leoec_measure_stream_half_dev"):
        L.leoec_measure_stream_half_dev.argtypes = [
            ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
            ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        L.leoec_measure_stream_half_dev.restype = ctypes.c_int
    _loaded[path] = L
    return L


_current = _load(MEASURE_LIB_PATH if os.environ.get("LEOEC_LIBRARY") == "measure" else LIB_PATH)


class _LibProxy:
    """`lib.leoec_*` resolves against the library in use (use_library)."""
    __slots__ = ()

    def __getattr__(self, name):
        return getattr(_current, name)


lib = _LibProxy()


def library_path():
    return _current._name


def use_library(path):
    """Route every later call through the library at `path`; returns the
    previous library's path."""
    global _current
    prev = _current._name
    _current = _load(path)
    return prev


def measure_library():
    """The measurement build (libleoec_measure.so), loaded beside whatever
    library is in use, for its measurement-only entry points
    (leoec_measure_xor_pattern_dev); raises if it was not built."""
    if not os.path.exists(MEASURE_LIB_PATH):
        raise RuntimeError(f"{MEASURE_LIB_PATH} not built (make -C leo_erasure_amd/csrc measure)")
    return _load(MEASURE_LIB_PATH)


def is_measure_build():
    return hasattr(_current, "leoec_measure_reload")


def _need_measure():
    if not is_measure_build():
        raise RuntimeError(f"{library_path()} is the product build: it has no LEOEC_* knobs")


def measure_reload():
    """Measurement build only: re-read the LEOEC_* knobs from the environment."""
    _need_measure()
    _current.leoec_measure_reload()


def measure_set_knob(name, value):
    """Measurement build only: set knob `name` (LEOEC_*) to `value`, or drop
    its override with None; the library never reads a changed environment,
    so nothing calls setenv while its threads run."""
    _need_measure()
    rc = _current.leoec_measure_set_knob(name.encode(),
                                         None if value is None else str(value).encode())
    if rc != 0:
        raise ValueError(f"not a knob: {name}")


def measure_warm_state(dev):
    """Measurement build only: what the warm-up left on device `dev`:
    {pool_streams, pool_mapped, queue (every lane of the device has its
    batching queue), queues_built (by the process)}."""
    _need_measure()
    out = (ctypes.c_int * 4)()
    _current.leoec_measure_warm_state(dev, out)
    return {"pool_streams": out[0], "pool_mapped": out[1], "queue": bool(out[2]),
            "queues_built": out[3]}


def measure_reclaim_state():
    """Measurement build only: the per-thread staging of exited threads
    (engine.cpp Staging::hand_off / reclaim_drain) and the warm-up threads:
    {handed_off, drained, busy (handed off with work in flight: 0),
    warm_threads_started, warm_threads_done}."""
    _need_measure()
    out = (ctypes.c_long * 5)()
    _current.leoec_measure_reclaim_state(out)
    return {"handed_off": out[0], "drained": out[1], "busy": out[2],
            "warm_threads_started": out[3], "warm_threads_done": out[4]}


def measure_reset_knobs():
    """Measurement build only: drop every measure_set_knob override."""
    _need_measure()
    _current.leoec_measure_reset_knobs()


def strerror(code):
    return lib.leoec_strerror(code).decode("latin-1")


def check(rc):
    if rc != OK:
        raise LeoecError(rc)
    return rc


def version():
    return lib.leoec_version().decode()


def host_spread(devices):
    """Spread host-memory calls over these device ordinals ([] restores the
    default: each call on the caller's current device); returns the count."""
    arr = (ctypes.c_int * max(len(devices), 1))(*devices)
    n = lib.leoec_host_spread(arr, len(devices))
    if n < 0:
        raise LeoecError(n)
    return n


def host_lanes():
    """Device ordinal of each dispatcher lane (one per gfx950 device)."""
    n = lib.leoec_host_lanes(None, 0)
    if n < 0:
        raise LeoecError(n)
    arr = (ctypes.c_int * max(n, 1))()
    check(min(0, lib.leoec_host_lanes(arr, n)))
    return list(arr[:n])
