"""Device-resident, batched form of encode / decode / repair (leoec_*_dev).

Buffers are torch uint8 CUDA(HIP) tensors used only as device memory; work
is enqueued on the current torch stream and not synchronised.  Layout of a
batch of ``n`` objects of ``size`` bytes:

* ``objs``   — ``[n, obj_stride]``: object o's data block j at byte j*bs of row o
               (the unpadded object; bytes past ``size`` are treated as zero);
* ``parity`` — ``[n, parity_stride]``: coding block i at byte i*bs of row o.
"""
import ctypes

from . import _lib
from ._lib import lib
from .api import layout  # noqa: F401  (re-exported)

torch = _lib.torch  # (None under LEOEC_NO_TORCH=1: the device API then needs explicit streams)


def _stream(stream):
    if stream is not None:
        return ctypes.c_void_p(stream)
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _cid(coding):
    cid = _lib.CODING_IDS.get(coding)
    if cid is None:
        raise _lib.LeoecError(_lib.E_INVALID_CODING)
    return cid


def _row_stride(t):
    if t.dtype != torch.uint8 or not t.is_cuda:
        raise ValueError("uint8 device tensor expected")
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError("2-D row-contiguous tensor expected")
    if t.device.index != torch.cuda.current_device():
        raise ValueError(f"tensor on {t.device}, current device is cuda:{torch.cuda.current_device()}")
    return t.stride(0)


def _rows(t, nobj, cols, what):
    """The kernels read / write `cols` bytes of each of `nobj` rows: the
    tensor must hold them (the C ABI sees only pointers and strides)."""
    if nobj < 0 or nobj > t.shape[0]:
        raise ValueError(f"{what}: nobj {nobj} outside [0, {t.shape[0]}]")
    if nobj and t.shape[1] < cols:
        raise ValueError(f"{what}: rows of {t.shape[1]} B, {cols} B needed")


def encode(coding, params, objs, size, parity, nobj=None, stream=None):
    """leoec_encode_dev: coding blocks of every object of the batch."""
    k, m, w = params
    nobj = objs.shape[0] if nobj is None else nobj
    bs, _ = layout(coding, params, size)
    _rows(objs, nobj, size, "objs")
    _rows(parity, nobj, m * bs, "parity")
    _lib.check(lib.leoec_encode_dev(_cid(coding), k, m, w, objs.data_ptr(), _row_stride(objs),
                                    size, nobj, parity.data_ptr(), _row_stride(parity),
                                    _stream(stream)))


def decode(coding, params, objs, size, parity, erased, nobj=None, stream=None):
    """leoec_decode_dev: rebuild the erased data blocks in place in ``objs``."""
    k, m, w = params
    nobj = objs.shape[0] if nobj is None else nobj
    bs, _ = layout(coding, params, size)
    _rows(objs, nobj, size, "objs")
    _rows(parity, nobj, m * bs, "parity")
    er = (ctypes.c_int * max(len(erased), 1))(*erased)
    _lib.check(lib.leoec_decode_dev(_cid(coding), k, m, w, objs.data_ptr(), _row_stride(objs),
                                    size, nobj, parity.data_ptr(), _row_stride(parity), er,
                                    len(erased), _stream(stream)))


def repair(coding, params, blocks, block_size, repair_ids, out, nobj, stream=None):
    """leoec_repair_dev.  ``blocks``: list of k+m tensors-or-None, each
    ``[nobj, stride]`` with the block at byte 0 of every row (all the same
    row stride); ``out``: list of tensors (same shape rules), one per id."""
    k, m, w = params
    strides = {_row_stride(b) for b in blocks if b is not None}
    ostrides = {_row_stride(o) for o in out}
    if len(strides) != 1 or len(ostrides) != 1:
        raise ValueError("one row stride per side expected")
    if len(blocks) != k + m:
        raise ValueError(f"blocks: {k + m} entries (tensor or None) expected")
    for b in blocks:
        if b is not None:
            _rows(b, nobj, block_size, "block")
    for o in out:
        _rows(o, nobj, block_size, "out")
    ptrs = (ctypes.c_void_p * (k + m))(*[b.data_ptr() if b is not None else None for b in blocks])
    optrs = (ctypes.c_void_p * max(len(out), 1))(*[o.data_ptr() for o in out])
    rep = (ctypes.c_int * max(len(repair_ids), 1))(*repair_ids)
    _lib.check(lib.leoec_repair_dev(_cid(coding), k, m, w, ptrs, strides.pop(), block_size, nobj,
                                    rep, len(repair_ids), optrs, ostrides.pop(), _stream(stream)))
