"""Python mirror of the reference's public API, over the C-ABI engine.

Two layers, like the reference:

* ``nif_*`` — the NIF surface ``gf_init/0``, ``encode/4``, ``decode/5``,
  ``repair/5`` (c_src/leo_erasure_nif.cpp:122-353): same argument meaning and
  validation order, same return shapes ``("ok", X)`` / ``("error", Reason)``.
* ``encode`` / ``decode`` / ``repair`` — the wrappers of src/leo_erasure.erl
  (default class and W filling, ``{Id, Block}`` zipping), dispatched on the
  number of arguments the way Erlang dispatches on arity.

Coding classes are the reference's atoms as strings: ``"vandrs"``,
``"cauchyrs"``, ``"liberation"``, ``"isars"`` (include/leo_erasure.hrl:23-31).
Blocks are ``bytes``.  All block arithmetic runs on the GPU (libleoec.so).
"""
import ctypes
import os

import numpy as np

from . import _lib
from ._lib import lib

# include/leo_erasure.hrl:23-51
CODING_CLASS_VANDRS = "vandrs"
CODING_CLASS_CAUCHYRS = "cauchyrs"
CODING_CLASS_LIBERATION = "liberation"
CODING_CLASS_ISA_VANDRS = "isars"
DEF_CODING_CLASS = CODING_CLASS_VANDRS
DEF_CODING_PARAMS = (10, 4, 8)
DEF_K = {"vandrs": 10, "cauchyrs": 4, "liberation": 4, "isars": 10}
DEF_M = {"vandrs": 4, "cauchyrs": 2, "liberation": 2, "isars": 4}
DEF_W = {"vandrs": 8, "cauchyrs": 3, "liberation": 7, "isars": 8}

_default_coder = None


def set_default_coder(coding_class):
    """application:set_env(leo_erasure, default_coder, Class) analogue."""
    global _default_coder
    _default_coder = coding_class


def env_default_coder():
    """?env_default_coder() (include/leo_erasure.hrl:88-94)."""
    if _default_coder is not None:
        return _default_coder
    return os.environ.get("LEO_ERASURE_DEFAULT_CODER", CODING_CLASS_VANDRS)


def coding_params_w(coding_class):
    """?coding_params_w(Class) (include/leo_erasure.hrl:74-84)."""
    return DEF_W[coding_class]


def _err(reason):
    return ("error", reason)


def _as_bytes(x):
    """enif_inspect_iolist_as_binary: a binary, or a (nested) list of binaries
    and bytes 0..255.  Tuples and out-of-range integers are not iolists."""
    if isinstance(x, (bytes, bytearray, memoryview)):
        return bytes(x)
    if not isinstance(x, list):
        return None
    out = bytearray()
    for p in x:
        if isinstance(p, int) and not isinstance(p, bool):
            if not 0 <= p <= 255:
                return None
            out.append(p)
        else:
            b = _as_bytes(p)
            if b is None:
                return None
            out += b
    return bytes(out)


def _c_int(v):
    """enif_get_int: an integer that fits a C int."""
    return isinstance(v, int) and not isinstance(v, bool) and -(1 << 31) <= v < (1 << 31)


def _coding_params(params):
    """{K,M,W} parsing of the NIF (leo_erasure_nif.cpp:144-153)."""
    if not isinstance(params, tuple):
        return None, "Expect tuple for coding parameters"
    names = ("Invalid K", "Invalid M", "Invalid W")
    vals = []
    for i in range(3):
        if i >= len(params) or not _c_int(params[i]):
            return None, names[i]
        vals.append(params[i])
    return tuple(vals), None


def _coding_id(coding):
    if not isinstance(coding, str):
        return None, "Expect coding"
    cid = _lib.CODING_IDS.get(coding)
    if cid is None:
        return None, "Invalid Coding"
    return cid, None


def gf_init():
    """gf_init/0 (leo_erasure_nif.cpp:122-128)."""
    rc = lib.leoec_gf_init()
    return "ok" if rc == 0 else _err(_lib.strerror(rc))


def layout(coding_class, params, size):
    """(block_size, filled) of the stripe geometry (c_src/rscoding.cpp:44-54)."""
    cid, e = _coding_id(coding_class)
    if e:
        raise _lib.LeoecError(_lib.E_INVALID_CODING)
    k, m, w = params
    bs = ctypes.c_uint64()
    filled = ctypes.c_int()
    _lib.check(lib.leoec_layout(cid, k, m, w, size, ctypes.byref(bs), ctypes.byref(filled)))
    return bs.value, filled.value


# ---------------------------------------------------------------------------
# NIF surface
def nif_encode(coding_class, params, data, total_size=None):
    """encode/4 (leo_erasure_nif.cpp:130-166).  TotalSize is ignored, as there."""
    data = _as_bytes(data)
    if data is None:
        return _err("Expected Input Bin")
    cid, e = _coding_id(coding_class) if isinstance(coding_class, str) else (None, "Expect coding")
    if e == "Expect coding":
        return _err(e)
    p, pe = _coding_params(params)
    if pe:
        return _err(pe)
    if cid is None:
        return _err("Invalid Coding")
    k, m, w = p
    bs = ctypes.c_uint64()
    filled = ctypes.c_int()
    rc = lib.leoec_layout(cid, k, m, w, len(data), ctypes.byref(bs), ctypes.byref(filled))
    if rc:
        return _err(_lib.strerror(rc))
    bs, filled = bs.value, filled.value
    nout = (k + m - filled) * bs
    out = np.empty(max(nout, 1), dtype=np.uint8)
    src = np.frombuffer(data, dtype=np.uint8) if data else np.zeros(1, dtype=np.uint8)
    rc = lib.leoec_encode(cid, k, m, w, src.ctypes.data, len(data), out.ctypes.data, nout)
    if rc:
        return _err(_lib.strerror(rc))
    blocks = [data[i * bs:(i + 1) * bs] for i in range(filled)]
    blocks += [out[i * bs:(i + 1) * bs].tobytes() for i in range(k + m - filled)]
    return ("ok", blocks)


def _parse_blocks(block_list, id_list):
    """Block / id list parsing shared by decode and repair (nif.cpp:173-206)."""
    if not isinstance(block_list, list):
        return None, None, "Block List Needed"
    if not isinstance(id_list, list):
        return None, None, "ID List Needed"
    if len(block_list) != len(id_list):
        return None, None, "Block List and ID List does not match (different Len)"
    blocks, ids = [], []
    for b, i in zip(block_list, id_list):
        bb = _as_bytes(b)
        if bb is None:
            return None, None, "Invalid Block"
        if not _c_int(i):
            return None, None, "Invalid ID"
        blocks.append(bb)
        ids.append(i)
    return blocks, ids, None


def _ptr_array(blocks):
    arrs = [np.frombuffer(b, dtype=np.uint8) if len(b) else np.zeros(1, np.uint8) for b in blocks]
    ptrs = (ctypes.c_void_p * max(len(arrs), 1))(*[a.ctypes.data for a in arrs])
    return arrs, ptrs


def nif_decode(coding_class, params, block_list, id_list, obj_size):
    """decode/5 (leo_erasure_nif.cpp:169-249)."""
    blocks, ids, e = _parse_blocks(block_list, id_list)
    if e:
        return _err(e)
    if not isinstance(obj_size, int) or obj_size < 0 or obj_size >= 1 << 64:
        return _err("Expect data size")
    if not isinstance(coding_class, str):
        return _err("Expect coding")
    p, pe = _coding_params(params)
    if pe:
        return _err(pe)
    cid, ce = _coding_id(coding_class)
    if ce:
        return _err(ce)
    k, m, w = p
    bs = len(blocks[-1]) if blocks else 0  # blockSize of the last listed block (rscoding.cpp:102)
    if any(len(b) != bs for b in blocks):
        return _err(_lib.strerror(-13))
    keep, ptrs = _ptr_array(blocks)
    idv = (ctypes.c_int * max(len(ids), 1))(*ids)
    out = np.empty(max(obj_size, 1), dtype=np.uint8)
    rc = lib.leoec_decode(cid, k, m, w, ptrs, idv, len(ids), bs, obj_size, out.ctypes.data)
    del keep
    if rc:
        return _err(_lib.strerror(rc))
    return ("ok", out[:obj_size].tobytes())


def nif_repair(coding_class, params, block_list, id_list, repair_id_list):
    """repair/5 (leo_erasure_nif.cpp:252-344)."""
    blocks, ids, e = _parse_blocks(block_list, id_list)
    if e:
        return _err(e)
    if not isinstance(repair_id_list, list):
        return _err("Repair ID List Needed")
    for r in repair_id_list:
        if not _c_int(r):
            return _err("Invalid Repair ID")
    if not isinstance(coding_class, str):
        return _err("Expect coding")
    p, pe = _coding_params(params)
    if pe:
        return _err(pe)
    cid, ce = _coding_id(coding_class)
    if ce:
        return _err(ce)
    k, m, w = p
    bs = len(blocks[-1]) if blocks else 0
    if any(len(b) != bs for b in blocks):
        return _err(_lib.strerror(-13))
    keep, ptrs = _ptr_array(blocks)
    idv = (ctypes.c_int * max(len(ids), 1))(*ids)
    rep = (ctypes.c_int * max(len(repair_id_list), 1))(*repair_id_list)
    nrep = len(repair_id_list)
    out = np.empty(max(nrep * bs, 1), dtype=np.uint8)
    rc = lib.leoec_repair(cid, k, m, w, ptrs, idv, len(ids), bs, rep, nrep, out.ctypes.data)
    del keep
    if rc:
        return _err(_lib.strerror(rc))
    return ("ok", [out[i * bs:(i + 1) * bs].tobytes() for i in range(nrep)])


# ---------------------------------------------------------------------------
# src/leo_erasure.erl wrappers (arity dispatch)
def encode(*args):
    """encode/2, encode/3, encode/4 (src/leo_erasure.erl:145-171)."""
    if len(args) == 2:
        (k, m), data = args
        cls = env_default_coder()
        return encode(cls, (k, m, coding_params_w(cls)), data)
    if len(args) == 3:
        cls, params, data = args
        if isinstance(params, tuple) and len(params) == 3 and isinstance(params[2], int) \
                and params[2] < 1 and cls in DEF_W:
            return encode(cls, (params[0], params[1], coding_params_w(cls)), data)
        res = nif_encode(cls, params, data, len(data) if hasattr(data, "__len__") else 0)
        if res[0] == "ok":
            return ("ok", list(enumerate(res[1])))
        return res
    if len(args) == 4:
        return nif_encode(*args)
    raise TypeError("encode/%d is undefined" % len(args))


def decode(*args):
    """decode/3, decode/4, decode/5 (src/leo_erasure.erl:182-208)."""
    if len(args) == 3:
        (k, m), id_with_block, obj_size = args
        cls = env_default_coder()
        return decode(cls, (k, m, coding_params_w(cls)), id_with_block, obj_size)
    if len(args) == 4:
        cls, params, id_with_block, obj_size = args
        if isinstance(params, tuple) and len(params) == 3 and isinstance(params[2], int) \
                and params[2] < 1 and cls in DEF_W:
            params = (params[0], params[1], coding_params_w(cls))
        ids = [i for i, _ in id_with_block]
        blocks = [b for _, b in id_with_block]
        return nif_decode(cls, params, blocks, ids, obj_size)
    if len(args) == 5:
        return nif_decode(*args)
    raise TypeError("decode/%d is undefined" % len(args))


def repair(*args):
    """repair/2, repair/3, repair/5 (src/leo_erasure.erl:217-245).

    repair/2 always uses the default class vandrs, not the env default
    (src/leo_erasure.erl:218)."""
    if len(args) == 2:
        (k, m), id_with_block = args
        cls = DEF_CODING_CLASS
        return repair(cls, (k, m, coding_params_w(cls)), id_with_block)
    if len(args) == 3:
        cls, params, id_with_block = args
        k, m = params[0], params[1]
        ids = [i for i, _ in id_with_block]
        blocks = [b for _, b in id_with_block]
        repair_ids = [i for i in range(k + m) if i not in ids]  # lists:subtract
        res = nif_repair(cls, params, blocks, ids, repair_ids)
        if res[0] == "ok":
            return ("ok", list(zip(repair_ids, res[1])))
        return res
    if len(args) == 5:
        return nif_repair(*args)
    raise TypeError("repair/%d is undefined" % len(args))


# ---------------------------------------------------------------------------
# File helpers of src/leo_erasure.erl:63-136,255-279 (blocks/<File>.<Id>).
BLOCKSTOR = "blocks/"


def write_blocks(file_name, blocks, cnt):
    """write_blocks/3: blocks/<FileName>.<Cnt>, Cnt counting up; returns the next Cnt."""
    os.makedirs(BLOCKSTOR, exist_ok=True)
    for b in blocks:
        with open(os.path.join(BLOCKSTOR, "%s.%d" % (file_name, cnt)), "wb") as fh:
            fh.write(b)
        cnt += 1
    return cnt


def encode_file(*args):
    """encode_file/1, encode_file/3 (src/leo_erasure.erl:63-96)."""
    if len(args) == 1:
        return encode_file(env_default_coder(), DEF_CODING_PARAMS, args[0])
    coding_class, params, file_name = args
    try:
        with open(file_name, "rb") as fh:
            data = fh.read()
    except OSError as e:
        return _err(e.strerror)
    res = nif_encode(coding_class, params, data, len(data))
    if res[0] != "ok":
        return res
    return write_blocks(file_name, res[1], 0)


def _check_available_blocks(file_name, cnt):
    """check_available_blocks/3: ids cnt..0 present on disk, ascending."""
    avail = []
    for i in range(cnt, -1, -1):
        if os.path.isfile(os.path.join(BLOCKSTOR, "%s.%d" % (file_name, i))):
            avail.insert(0, i)
    return avail


def decode_file(*args):
    """decode_file/2, decode_file/4 (src/leo_erasure.erl:102-136): reads the
    blocks of ids 14..0 present on disk (as the reference does) and writes
    <FileName>.dec."""
    if len(args) == 2:
        return decode_file(env_default_coder(), DEF_CODING_PARAMS, args[0], args[1])
    coding_class, params, file_name, obj_size = args
    id_with_block = []
    for i in _check_available_blocks(file_name, 14):  # read_blocks/3 builds the list reversed
        with open(os.path.join(BLOCKSTOR, "%s.%d" % (file_name, i)), "rb") as fh:
            id_with_block.insert(0, (i, fh.read()))
    res = decode(coding_class, params, id_with_block, obj_size)
    if res[0] != "ok":
        return res
    with open(file_name + ".dec", "wb") as fh:
        fh.write(res[1])
    return "ok"
