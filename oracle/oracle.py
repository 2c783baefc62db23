"""ctypes front-end of the CPU restatement oracle (oracle/crdtree_oracle.cpp).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py — never by the product package.

`OTree` mirrors the Elm `CRDTree` API (src/CRDTree.elm:1-26) closely enough
that the reference's own tests (tests/CRDTreeTest.elm, tests/NodeTest.elm)
transcribe one-to-one. Operations are duck-typed: anything with
`kind in ("add", "del", "batch")` and `ts/path/val` or `ops` attributes.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle.so")
_lib = None

ERR_NAMES = {0: "Ok", 1: "InvalidPath", 2: "NotFound", 3: "OperationFailed"}
MASK32 = 2 ** 32


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB) or os.path.getmtime(_LIB) < os.path.getmtime(
                os.path.join(_HERE, "crdtree_oracle.cpp")):
            build()
        L = C.CDLL(_LIB)
        P = C.c_void_p
        L.orc_init.restype = P
        L.orc_init.argtypes = [C.c_int64]
        L.orc_clone.restype = P
        L.orc_clone.argtypes = [P]
        L.orc_free.argtypes = [P]
        L.orc_apply.restype = C.c_int
        L.orc_apply.argtypes = [P, C.c_int, C.c_int, C.c_uint64, P, P, P, P, P, C.POINTER(C.c_int64)]
        L.orc_timestamp.restype = C.c_int64
        L.orc_timestamp.argtypes = [P]
        L.orc_guard_stats.restype = None
        L.orc_guard_stats.argtypes = [P]
        L.orc_cursor.restype = C.c_uint64
        L.orc_cursor.argtypes = [P, P, C.c_uint64]
        L.orc_set_cursor.argtypes = [P, P, C.c_uint64]
        L.orc_replicas.restype = C.c_uint64
        L.orc_replicas.argtypes = [P, P, P, C.c_uint64]
        L.orc_ops.restype = C.c_uint64
        L.orc_ops.argtypes = [P, C.c_int, P, P, P, P, P, P, P]
        L.orc_canonical.restype = C.c_uint64
        L.orc_canonical.argtypes = [P, C.c_int, P, C.c_uint64, P]
        L.orc_get_value.restype = C.c_int
        L.orc_get_value.argtypes = [P, P, C.c_uint64, P, P]
        L.orc_get_path.restype = C.c_uint64
        L.orc_get_path.argtypes = [P, P, C.c_uint64, P, C.c_uint64]
        L.orc_node_get.restype = C.c_uint64
        L.orc_node_get.argtypes = [P, P, C.c_uint64, P, C.c_uint64]
        L.orc_node_query.restype = C.c_uint64
        L.orc_node_query.argtypes = [P, C.c_int, P, C.c_uint64, P, C.c_uint64]
        L.orc_flat_replay.restype = C.c_int
        L.orc_flat_replay.argtypes = [C.c_uint64, P, P, P, P, P, C.POINTER(C.c_int64), P, P, C.POINTER(C.c_uint64)]
        L.orc_flat_replay_literal.restype = C.c_int
        L.orc_flat_replay_literal.argtypes = L.orc_flat_replay.argtypes
        L.orc_flat_check.restype = C.c_uint64
        L.orc_flat_check.argtypes = [C.c_uint64, P, C.c_uint64, P, P, P]
        L.orc_reset_last.argtypes = [P]
        L.orc_merge_last.argtypes = [P, P]
        L.orc_forest_apply.restype = None
        L.orc_forest_apply.argtypes = [C.c_uint64, P, C.c_int64, P, P, P, P, P, P, P, P, P, P]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None and a.size else None


class Values:
    """Interning table: opaque Elm values <-> u32 handles."""

    def __init__(self):
        self.to_handle = {}
        self.values = []

    def handle(self, v):
        key = (type(v).__name__, v)
        h = self.to_handle.get(key)
        if h is None:
            h = len(self.values)
            self.values.append(v)
            self.to_handle[key] = h
        return h

    def value(self, h):
        return self.values[h]


VALUES = Values()


def flatten(op, out):
    """Leaves of a (possibly nested) Batch in order (empty Batches vanish)."""
    if op.kind == "batch":
        for o in op.ops:
            flatten(o, out)
    else:
        out.append(op)
    return out


def pack(leaves, values=VALUES):
    n = len(leaves)
    kind = np.zeros(max(n, 1), np.uint8)
    ts = np.zeros(max(n, 1), np.int64)
    val = np.zeros(max(n, 1), np.uint32)
    off = np.zeros(n + 1, np.uint32)
    paths = []
    for i, o in enumerate(leaves):
        kind[i] = 0 if o.kind == "add" else 1
        if o.kind == "add":
            ts[i] = o.ts
            val[i] = values.handle(o.val)
        paths.extend(o.path)
        off[i + 1] = len(paths)
    path = np.array(paths if paths else [0], np.int64)
    return kind, ts, off, path, val


class OTree:
    """CRDTree a, restated (src/CRDTree.elm:112-120)."""

    def __init__(self, replica_id=0, _h=None):
        self._h = _h if _h is not None else lib().orc_init(replica_id)
        self.err_index = -1

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.orc_free(self._h)
            self._h = None

    def clone(self):
        return OTree(_h=lib().orc_clone(self._h))

    # ---- merge path ----
    def _apply(self, op, local):
        leaves = flatten(op, []) if op.kind == "batch" else [op]
        is_batch = 1 if op.kind == "batch" else 0
        kind, ts, off, path, val = pack(leaves)
        new = self.clone()
        err = C.c_int64(-1)
        r = lib().orc_apply(new._h, is_batch, 1 if local else 0, len(leaves), _ptr(kind), _ptr(ts), _ptr(off),
                            _ptr(path), _ptr(val), C.byref(err))
        if r != 0:
            return ERR_NAMES[r], leaves[err.value] if err.value >= 0 else None
        return "Ok", new

    def apply(self, op):
        """CRDTree.apply (src/CRDTree.elm:265-269): ('Ok', tree) | (errname, op)."""
        return self._apply(op, local=False)

    def apply_local(self, op):
        return self._apply(op, local=True)

    # ---- local editing (src/CRDTree.elm:151-216), used by the transcribed tests ----
    def next_timestamp(self):
        return self.timestamp() + 1

    def add(self, v):
        return self.add_after(self.cursor(), v)

    def add_after(self, path, v):
        from types import SimpleNamespace as NS
        return self.apply_local(NS(kind="add", ts=self.next_timestamp(), path=list(path), val=v))

    def add_branch(self, v):
        r, t = self.add(v)
        if r == "Ok":
            c = t.cursor() + [0]
            lib().orc_set_cursor(t._h, _ptr(np.array(c, np.int64)), len(c))
        return r, t

    def delete(self, path):
        from types import SimpleNamespace as NS
        # cursor bookkeeping of the local delete (previous sibling's path) is
        # not on the merge path; the Delete itself is what the tests pin.
        r, t = self.apply_local(NS(kind="del", path=list(path)))
        if r == "Ok":
            lib().orc_set_cursor(t._h, _ptr(np.array(path, np.int64)), len(path))
        return r, t

    def batch(self, funcs):
        """CRDTree.batch (src/CRDTree.elm:224-232) over local functions."""
        cur = self.clone()
        lib().orc_reset_last(cur._h)
        for f in funcs:
            r, nxt = f(cur)
            if r != "Ok":
                return r, nxt
            lib().orc_merge_last(nxt._h, cur._h)
            cur = nxt
        return "Ok", cur

    # ---- traversal (src/CRDTree.elm:421-625): node descriptors
    #      (kind, value, path tuple, next) with kind in node/tombstone/root ----
    raw_values = False  # True: descriptors carry value handles (engine parity tests)

    def _nodes(self, words):
        out, k = [], 0
        while k < len(words):
            kind, val, hn, nx, pl = (int(x) for x in words[k:k + 5])
            path = tuple(int(x) for x in words[k + 5:k + 5 + pl])
            kd = {1: "node", 2: "tombstone", 3: "root"}[kind]
            v = (val if self.raw_values else VALUES.value(val)) if kd == "node" else None
            out.append((kd, v, path, nx if hn else None))
            k += 5 + pl
        return out

    def _words(self, fn, *args):
        n = fn(self._h, *args, None, 0)
        buf = np.zeros(max(n, 1), np.int64)
        fn(self._h, *args, _ptr(buf), n)
        return buf[:n]

    def node(self, path):
        """get path tree -> descriptor or None."""
        p = np.array(list(path) or [0], np.int64)
        r = self._nodes(self._words(lib().orc_node_get, _ptr(p), len(path)))
        return r[0] if r else None

    def node_query(self, which, path=None):
        """which: parent, next, prev, children, walk (from the node at path), walk_start."""
        code = {"parent": 0, "next": 1, "prev": 2, "children": 3, "walk": 4, "walk_start": 5}[which]
        p = np.array(list(path or []) or [0], np.int64)
        r = self._nodes(self._words(lib().orc_node_query, code, _ptr(p), len(path or [])))
        return r if which in ("children", "walk", "walk_start") else (r[0] if r else None)

    # ---- queries ----
    def timestamp(self):
        return lib().orc_timestamp(self._h)

    def cursor(self):
        buf = np.zeros(64, np.int64)
        n = lib().orc_cursor(self._h, _ptr(buf), 64)
        return [int(x) for x in buf[:n]]

    def replicas(self):
        n = lib().orc_replicas(self._h, None, None, 0)
        ids = np.zeros(max(n, 1), np.int64)
        tss = np.zeros(max(n, 1), np.int64)
        lib().orc_replicas(self._h, _ptr(ids), _ptr(tss), n)
        return {int(a): int(b) for a, b in zip(ids[:n], tss[:n])}

    def last_replica_timestamp(self, rid):
        return self.replicas().get(rid, 0)

    def _ops(self, which):
        L = lib()
        pt = C.c_uint64(0)
        isb = C.c_int(0)
        n = L.orc_ops(self._h, which, None, None, None, None, None, C.byref(pt), C.byref(isb))
        kind = np.zeros(max(n, 1), np.uint8)
        ts = np.zeros(max(n, 1), np.int64)
        off = np.zeros(n + 1, np.uint32)
        path = np.zeros(max(pt.value, 1), np.int64)
        val = np.zeros(max(n, 1), np.uint32)
        L.orc_ops(self._h, which, _ptr(kind), _ptr(ts), _ptr(off), _ptr(path), _ptr(val), None, None)
        out = []
        for i in range(n):
            p = [int(x) for x in path[off[i]:off[i + 1]]]
            if kind[i] == 0:
                out.append(("add", int(ts[i]), p, VALUES.value(int(val[i]))))
            else:
                out.append(("del", p))
        return out, bool(isb.value)

    def operations(self):
        """The log oldest-first (= operationsSince 0, src/CRDTree.elm:408-414)."""
        return self._ops(0)[0]

    def last_operation(self):
        """('batch', [ops]) or the single op tuple (src/CRDTree.elm:371-373)."""
        ops, isb = self._ops(1)
        return ("batch", ops) if isb else ops[0]

    def operations_since(self, ts):
        """CRDTree.operationsSince (src/CRDTree.elm:408-418) + Operation.since
        (src/Internal/Operation.elm:25-53): inclusive of the Add with that ts,
        [] when absent; Batch entries never reach the log."""
        log = self.operations()
        if ts == 0:
            return log
        acc = []
        for o in reversed(log):  # newest-first walk, prepending
            acc.insert(0, o)
            if o[0] == "add" and o[1] == ts:
                return acc
        return []

    def get_value(self, path):
        v = C.c_uint32(0)
        ex = C.c_int(0)
        p = np.array(path if path else [0], np.int64)
        r = lib().orc_get_value(self._h, _ptr(p), len(path), C.byref(v), C.byref(ex))
        return VALUES.value(v.value) if r else None

    def get_path(self, path):
        p = np.array(path if path else [0], np.int64)
        buf = np.zeros(64, np.int64)
        n = lib().orc_get_path(self._h, _ptr(p), len(path), _ptr(buf), 64)
        return None if n == 2 ** 64 - 1 else [int(x) for x in buf[:n]]

    def canonical(self, which=0, full=True):
        """Canonical dump words (which=0 structure, 1 visible order) and FNV hash."""
        h = C.c_uint64(0)
        n = lib().orc_canonical(self._h, which, None, 0, C.byref(h))
        if not full:
            return None, n, h.value
        buf = np.zeros(max(n, 1), np.int64)
        lib().orc_canonical(self._h, which, _ptr(buf), n, None)
        return buf[:n], n, h.value

    def visible_values(self, depth0_only=True):
        """Values of the visible document (Node.map Node.value of the root level)."""
        words, n, _ = self.canonical(1)
        out = []
        i = 0
        while i < n:
            d, v, pl = int(words[i]), int(words[i + 1]), int(words[i + 2])
            if d == 0 or not depth0_only:
                out.append(VALUES.value(v))
            i += 3 + pl
        return out


def replica_id(ts):
    """Timestamp.replicaId (src/CRDTree/Timestamp.elm:16-18): trunc(ts / 2^32)."""
    q = abs(ts) // MASK32
    return q if ts >= 0 else -q
