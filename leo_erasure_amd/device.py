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

try:
    import torch
except Exception:  # pragma: no cover
    torch = None


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
    assert t.dtype == torch.uint8 and t.is_cuda, "uint8 device tensor expected"
    assert t.dim() == 2 and t.stride(1) == 1, "2-D row-contiguous tensor expected"
    return t.stride(0)


def encode(coding, params, objs, size, parity, nobj=None, stream=None):
    """leoec_encode_dev: coding blocks of every object of the batch."""
    k, m, w = params
    nobj = objs.shape[0] if nobj is None else nobj
    _lib.check(lib.leoec_encode_dev(_cid(coding), k, m, w, objs.data_ptr(), _row_stride(objs),
                                    size, nobj, parity.data_ptr(), _row_stride(parity),
                                    _stream(stream)))


def decode(coding, params, objs, size, parity, erased, nobj=None, stream=None):
    """leoec_decode_dev: rebuild the erased data blocks in place in ``objs``."""
    k, m, w = params
    nobj = objs.shape[0] if nobj is None else nobj
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
    assert len(strides) == 1 and len(ostrides) == 1, "one row stride per side expected"
    ptrs = (ctypes.c_void_p * (k + m))(*[b.data_ptr() if b is not None else None for b in blocks])
    optrs = (ctypes.c_void_p * max(len(out), 1))(*[o.data_ptr() for o in out])
    rep = (ctypes.c_int * max(len(repair_ids), 1))(*repair_ids)
    _lib.check(lib.leoec_repair_dev(_cid(coding), k, m, w, ptrs, strides.pop(), block_size, nobj,
                                    rep, len(repair_ids), optrs, ostrides.pop(), _stream(stream)))
