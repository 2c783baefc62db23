"""ctypes binding of libcrdtm.so (the C ABI in include/crdtm.h).

The product path has no CPU fallback: if the HIP library is missing or no
device is present, calls raise. PyTorch (when installed) is imported first so
that the process uses one HIP runtime for torch tensors and the engine.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# CRDTM_LIB: load another build of the engine (same-box A/B measurements)
LIB_PATH = os.environ.get("CRDTM_LIB") or os.path.join(_HERE, "libcrdtm.so")

CRDTM_OK = 0
PATH_CLOSED_FORM = 1
PATH_REPLAY = 2
PATH_DICT_REPLAY = 3
FLAG_REMERGE = 1  # non-fresh tree merged as init ++ log ++ batch on the parallel paths
FLAG_INCREMENTAL = 2  # adds-only batch merged into a clean flat document in place (incr.hip)
FLAG_INCR_WINDOWS = 4  # ... and blocks of its gapped order were spread over rebalance windows
FLAG_INCR_DENSE = 8  # ... and no window could take it: merged densely, the blocks rebuilt
FLAG_INCR_TOUR = 32  # ... and some gap was ordered as its tree's DFS (keys growing along its anchors)
FLAG_DICT_INCR = 16  # non-fresh tree: replayed per children dict on the state itself, level by level (ilr.hip)
REF_NONE = 2 ** 64 - 1
REF_ROOT = 2 ** 64 - 2
REL_PARENT, REL_NEXT, REL_PREV, REL_HEAD = 0, 1, 2, 3
CODES = {0: "Ok", 1: "InvalidPath", 2: "NotFound", 3: "OperationFailed", -1: "E_ARG", -2: "E_HIP", -3: "E_NOMEM", -7: "E_STATE",
         -4: "E_RANGE", -5: "E_NODEVICE", -6: "E_PARSE"}


class Ops(C.Structure):
    _fields_ = [("n_ops", C.c_uint64), ("n_path", C.c_uint64), ("kind", C.c_void_p), ("ts", C.c_void_p),
                ("path_off", C.c_void_p), ("path", C.c_void_p), ("val", C.c_void_p), ("tree", C.c_void_p)]


class Result(C.Structure):
    _fields_ = [("code", C.c_int32), ("path_taken", C.c_int32), ("err_index", C.c_int64),
                ("n_applied", C.c_uint64), ("n_already", C.c_uint64), ("timestamp", C.c_int64),
                ("n_slots", C.c_uint64), ("guard", C.c_uint32), ("flags", C.c_uint32),
                ("serial_ops", C.c_uint64), ("serial_dicts", C.c_uint64), ("serial_max", C.c_uint64)]


class SynthParams(C.Structure):
    _fields_ = [("n_ops", C.c_uint64), ("n_docs", C.c_uint64), ("replicas", C.c_uint32), ("window", C.c_uint32),
                ("p_delete", C.c_double), ("p_branch", C.c_double), ("p_continue", C.c_double),
                ("max_depth", C.c_uint32), ("max_children", C.c_uint32), ("deletes_last", C.c_uint32),
                ("seed", C.c_uint64), ("doc_base", C.c_uint64)]


# every function the header declares: (name, restype, argtypes)
P = C.c_void_p
SIGNATURES = [
    ("crdtm_version", C.c_int, []),
    ("crdtm_device_count", C.c_int, [C.POINTER(C.c_int)]),
    ("crdtm_ctx_create", C.c_int, [C.c_int, P, C.POINTER(P)]),
    ("crdtm_ctx_destroy", C.c_int, [P]),
    ("crdtm_ctx_stream", P, [P]),
    ("crdtm_ctx_sync", C.c_int, [P]),
    ("crdtm_tree_create", C.c_int, [P, C.c_int64, C.POINTER(P)]),
    ("crdtm_tree_destroy", C.c_int, [P]),
    ("crdtm_tree_reset", C.c_int, [P, C.c_int64]),
    ("crdtm_tree_clone", C.c_int, [P, C.POINTER(P)]),
    ("crdtm_apply", C.c_int, [P, C.POINTER(Ops), C.c_int, C.c_int, P, C.POINTER(Result)]),
    ("crdtm_tree_timestamp", C.c_int, [P, C.POINTER(C.c_int64)]),
    ("crdtm_tree_replicas", C.c_int, [P, P, P, C.c_uint64, C.POINTER(C.c_uint64)]),
    ("crdtm_tree_ops", C.c_int, [P, C.c_int, C.POINTER(Ops), C.POINTER(C.c_int)]),
    ("crdtm_tree_ops_since", C.c_int, [P, C.c_int64, C.POINTER(Ops)]),
    ("crdtm_shard_assemble", C.c_int, [P, P, C.c_uint64, C.c_int32, C.c_int32, C.c_uint64, C.POINTER(Ops)]),
    ("crdtm_tree_get", C.c_int, [P, P, C.c_uint64, C.POINTER(C.c_uint64)]),
    ("crdtm_node_info", C.c_int, [P, C.c_uint64, C.POINTER(C.c_int32), C.POINTER(C.c_uint32), C.POINTER(C.c_int32),
                                  C.POINTER(C.c_int64), P, C.c_uint64, C.POINTER(C.c_uint64)]),
    ("crdtm_tree_relative", C.c_int, [P, C.c_uint64, C.c_int, C.POINTER(C.c_uint64)]),
    ("crdtm_node_children", C.c_int, [P, C.c_uint64, P, C.c_uint64, C.POINTER(C.c_uint64)]),
    ("crdtm_tree_walk", C.c_int, [P, C.c_uint64, P, C.c_uint64, C.POINTER(C.c_uint64)]),
    ("crdtm_tree_canonical", C.c_int, [P, C.c_int, P, C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    ("crdtm_tree_document", C.c_int, [P, P, C.c_uint64, C.POINTER(C.c_uint64)]),
    ("crdtm_forest_apply", C.c_int, [P, C.c_int64, C.POINTER(Ops), P, C.c_uint64, C.c_int, P, P, P, P, P, P]),
    ("crdtm_synth", C.c_int, [C.POINTER(SynthParams), C.POINTER(C.POINTER(Ops))]),
    ("crdtm_ops_free", C.c_int, [C.POINTER(Ops)]),
    ("crdtm_json_decode", C.c_int, [C.c_char_p, C.c_size_t, C.POINTER(C.POINTER(Ops)), C.POINTER(C.c_void_p),
                                    C.POINTER(C.c_void_p), C.POINTER(C.c_uint64), C.POINTER(C.c_int)]),
    ("crdtm_json_encode", C.c_int, [C.POINTER(Ops), C.c_int, C.c_char_p, P, C.POINTER(C.c_void_p),
                                    C.POINTER(C.c_size_t)]),
    ("crdtm_json_canonical", C.c_int, [C.c_char_p, C.c_size_t, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]),
    ("crdtm_free", None, [P]),
    ("crdtm_ctx_guard_stats", C.c_int, [P, P]),
    ("crdtm_debug_poke", C.c_int, [P, C.c_int, C.c_uint64, C.c_uint32]),
    ("crdtm_ctx_profile", C.c_int, [P, C.c_int]),
    ("crdtm_ctx_phase_times", C.c_int, [P, C.c_char_p, C.c_size_t, P, C.c_int]),
]

_lib = None


class CrdtmError(RuntimeError):
    pass


def lib():
    """Load libcrdtm.so (raises if it was not built — there is no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise CrdtmError(f"{LIB_PATH} missing: build it with `make -C crdt-graph_amd` "
                             "(or __graft_entry__.build()); the merge engine has no CPU fallback")
        try:  # one HIP runtime per process: let torch load it first when present
            import torch  # noqa: F401
        except Exception:  # pragma: no cover
            pass
        L = C.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(code, what="crdtm"):
    if code < 0:
        raise CrdtmError(f"{what} failed: {CODES.get(code, code)}")
    return code


_CTX = {}


def context(device=0):
    """Process-wide engine context per device (own HIP stream)."""
    if device not in _CTX:
        h = C.c_void_p()
        check(lib().crdtm_ctx_create(device, None, C.byref(h)), "crdtm_ctx_create")
        _CTX[device] = h
    return _CTX[device]


def synth(n_ops, n_docs=1, replicas=2, window=8, p_delete=0.0, p_branch=0.0, p_continue=0.9, max_depth=1,
          max_children=0, deletes_last=0, seed=1, doc_base=0):
    """Generate a synthetic op stream (host numpy arrays, copied out of the engine)."""
    import numpy as np
    p = SynthParams(n_ops, n_docs, replicas, window, p_delete, p_branch, p_continue, max_depth, max_children,
                    deletes_last, seed, doc_base)
    out = C.POINTER(Ops)()
    check(lib().crdtm_synth(C.byref(p), C.byref(out)), "crdtm_synth")
    o = out.contents
    n, npth = o.n_ops, o.n_path

    def arr(ptr, dtype, count):
        if not ptr or count == 0:
            return np.zeros(0, dtype)
        buf = (C.c_char * (count * np.dtype(dtype).itemsize)).from_address(ptr)
        return np.frombuffer(buf, dtype=dtype, count=count).copy()

    res = dict(kind=arr(o.kind, np.uint8, n), ts=arr(o.ts, np.int64, n), path_off=arr(o.path_off, np.uint32, n + 1),
               path=arr(o.path, np.int64, npth), val=arr(o.val, np.uint32, n),
               tree=arr(o.tree, np.uint32, n) if o.tree else None)
    lib().crdtm_ops_free(out)
    return res
