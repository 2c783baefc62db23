"""JSON wire format — mirror of `CRDTree.Operation.encoder` / `decoder`
(src/CRDTree/Operation.elm:109-159), implemented natively (csrc/json_codec.cpp).

`encoder(op, value_encoder)` returns the exact bytes `Json.Encode.encode 0`
produces; `decoder(text, value_decoder)` returns the Operation (nested Batches
kept as one flat Batch: `apply` is identical either way). Values cross as JSON
text; the defaults mirror Encode.value / Decode.value via Python's json.
"""
from __future__ import annotations

import ctypes as C
import json

import numpy as np

from . import _native as N
from .operation import Add, Batch, Delete, flatten


class DecodeError(ValueError):
    pass


def _take(ptr, n):
    s = C.string_at(ptr, n).decode("utf-8")
    N.lib().crdtm_free(ptr)
    return s


def canonical_value(text: str) -> str:
    """JSON.stringify(JSON.parse(text))."""
    b = text.encode("utf-8")
    out = C.c_void_p()
    n = C.c_size_t()
    r = N.lib().crdtm_json_canonical(b, len(b), C.byref(out), C.byref(n))
    if r != 0:
        raise DecodeError(f"not a JSON value: {text!r}")
    return _take(out, n.value)


def _default_encode(v):
    return json.dumps(v, ensure_ascii=False, allow_nan=False, separators=(",", ":"))


def encoder(op, value_encoder=_default_encode) -> str:
    leaves = flatten(op) if op.kind == "batch" else [op]
    is_batch = op.kind == "batch"
    vals = []
    voff = [0]
    for o in leaves:
        if o.kind == "add":
            t = canonical_value(value_encoder(o.val)).encode("utf-8")
            vals.append(t)
            voff.append(voff[-1] + len(t))
    n = len(leaves)
    kind = np.zeros(n + 1, np.uint8)
    ts = np.zeros(n + 1, np.int64)
    off = np.zeros(n + 1, np.uint32)
    val = np.zeros(n + 1, np.uint32)
    path = []
    h = 0
    for i, o in enumerate(leaves):
        if o.kind == "add":
            ts[i] = o.ts
            val[i] = h
            h += 1
        else:
            kind[i] = 1
        path.extend(o.path)
        off[i + 1] = len(path)
    parr = np.array(path + [0], np.int64)
    vb = b"".join(vals) + b"\0"
    vo = np.array(voff, np.uint64)
    p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    ops = N.Ops(n, len(path), p(kind), p(ts), p(off), p(parr), p(val), None)
    out = C.c_void_p()
    ln = C.c_size_t()
    N.check(N.lib().crdtm_json_encode(C.byref(ops), 1 if is_batch else 0, vb, p(vo), C.byref(out), C.byref(ln)),
            "crdtm_json_encode")
    return _take(out, ln.value)


def decoder(text: str, value_decoder=json.loads):
    """Decode one Operation; unknown "op" -> Batch [] (src/CRDTree/Operation.elm:158-159)."""
    b = text.encode("utf-8")
    ops = C.POINTER(N.Ops)()
    vb = C.c_void_p()
    vo = C.c_void_p()
    nv = C.c_uint64()
    isb = C.c_int()
    r = N.lib().crdtm_json_decode(b, len(b), C.byref(ops), C.byref(vb), C.byref(vo), C.byref(nv), C.byref(isb))
    if r != 0:
        raise DecodeError(f"invalid operation JSON ({N.CODES.get(r, r)})")
    o = ops.contents
    n, npth = o.n_ops, o.n_path

    def arr(ptr, dt, cnt):
        if not ptr or cnt == 0:
            return np.zeros(0, dt)
        return np.frombuffer((C.c_char * (cnt * np.dtype(dt).itemsize)).from_address(ptr), dtype=dt,
                             count=cnt).copy()

    kind = arr(o.kind, np.uint8, n)
    ts = arr(o.ts, np.int64, n)
    off = arr(o.path_off, np.uint32, n + 1)
    path = arr(o.path, np.int64, npth)
    val = arr(o.val, np.uint32, n)
    voff = arr(vo.value, np.uint64, nv.value + 1)
    vbytes = C.string_at(vb.value, int(voff[-1]) if nv.value else 0) if vb.value else b""
    out = []
    for i in range(n):
        pth = [int(x) for x in path[off[i]:off[i + 1]]]
        if kind[i] == 0:
            h = int(val[i])
            txt = vbytes[int(voff[h]):int(voff[h + 1])].decode("utf-8")
            out.append(Add(int(ts[i]), pth, value_decoder(txt)))
        else:
            out.append(Delete(pth))
    N.lib().crdtm_ops_free(ops)
    N.lib().crdtm_free(vb)
    N.lib().crdtm_free(vo)
    if isb.value:
        return Batch(out)
    return out[0]
