"""CRDTree — host mirror of the reference's public module (src/CRDTree.elm:1-26),
backed by the gfx950 merge engine through the C ABI.

Names and meaning follow the Elm API: `init`, `apply`, `batch`, `add`,
`add_after`, `add_branch`, `delete`, `last_operation`, `operations_since`,
`timestamp`, `id`, `last_replica_timestamp`, `get_value`. `apply` keeps the
Elm persistence contract (the input tree stays valid): it clones the device
state first; `apply_in_place` is the linear-use variant for throughput.
Results are `Ok(tree)` / `Err(error)` like Elm's `Result (Error a) (CRDTree a)`.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Any

import numpy as np

from . import _native as N
from .operation import Add, Batch, Delete, flatten
from .timestamp import TWO32, replica_id


# ---- Result / Error (src/CRDTree.elm:104-107) ----
@dataclass(frozen=True)
class Ok:
    value: Any
    ok = True


@dataclass(frozen=True)
class Err:
    error: Any
    ok = False


@dataclass(frozen=True)
class InvalidPath:
    pass


@dataclass(frozen=True)
class NotFound:
    pass


@dataclass(frozen=True)
class OperationFailed:
    operation: Any


class Values:
    """Opaque Elm values <-> u32 handles (the engine orders by timestamp only)."""

    def __init__(self):
        self._h = {}
        self._v = []

    def handle(self, v):
        k = (type(v).__name__, v)
        h = self._h.get(k)
        if h is None:
            h = len(self._v)
            self._v.append(v)
            self._h[k] = h
        return h

    def value(self, h):
        return self._v[h]


VALUES = Values()



class NodeView:
    """A node of CRDTree a as the reference exposes it (src/Internal/Node.elm:29-32)."""
    __slots__ = ("ref", "kind", "value", "path", "next")

    def __init__(self, ref, kind, value, path, next_):
        self.ref, self.kind, self.value, self.path, self.next = ref, kind, value, path, next_

    def key(self):
        return (self.kind, self.value, tuple(self.path), self.next)

    def __repr__(self):
        return f"NodeView({self.kind}, {self.value!r}, {self.path}, next={self.next})"

def pack(leaves, values=VALUES):
    """Flattened Add/Delete leaves -> SoA numpy arrays (crdtm_ops layout)."""
    n = len(leaves)
    kind = np.zeros(n + 1, np.uint8)
    ts = np.zeros(n + 1, np.int64)
    val = np.zeros(n + 1, np.uint32)
    off = np.zeros(n + 1, np.uint32)
    path = []
    for i, o in enumerate(leaves):
        if o.kind == "add":
            ts[i] = o.ts
            val[i] = values.handle(o.val)
        else:
            kind[i] = 1
        path.extend(o.path)
        off[i + 1] = len(path)
    return dict(kind=kind, ts=ts, path_off=off, path=np.array(path + [0], np.int64), val=val)


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def ops_struct(arrs, n):
    return N.Ops(n, int(arrs["path_off"][n]), _ptr(arrs["kind"]), _ptr(arrs["ts"]), _ptr(arrs["path_off"]),
                 _ptr(arrs["path"]), _ptr(arrs["val"]), None)


class CRDTree:
    """CRDTree a (src/CRDTree.elm:112-120), device resident."""

    def __init__(self, handle, device=0, cursor=(0,)):
        self._h = handle
        self.device = device
        self._cursor = list(cursor)
        self.last_result = None

    # ---- lifecycle ----
    @staticmethod
    def init(replica_id_: int, device: int = 0) -> "CRDTree":
        """CRDTree.init (src/CRDTree.elm:130-139)."""
        ctx = N.context(device)
        h = C.c_void_p()
        N.check(N.lib().crdtm_tree_create(ctx, int(replica_id_), C.byref(h)), "crdtm_tree_create")
        return CRDTree(h, device)

    def clone(self) -> "CRDTree":
        h = C.c_void_p()
        N.check(N.lib().crdtm_tree_clone(self._h, C.byref(h)), "crdtm_tree_clone")
        return CRDTree(h, self.device, self._cursor)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and N._lib is not None:
            N._lib.crdtm_tree_destroy(h)
            self._h = None

    # ---- merge path ----
    def apply_arrays(self, arrs, n, is_batch=True, on_device=False, status=None):
        """Apply packed ops in place (crdtm_apply); returns the crdtm_result."""
        res = N.Result()
        ops = arrs if isinstance(arrs, N.Ops) else ops_struct(arrs, n)
        st = _ptr(status) if status is not None else None
        N.check(N.lib().crdtm_apply(self._h, C.byref(ops), 1 if on_device else 0, 1 if is_batch else 0, st,
                                    C.byref(res)), "crdtm_apply")
        self.last_result = res
        return res

    def _apply(self, op, in_place):
        leaves = flatten(op) if op.kind == "batch" else [op]
        is_batch = op.kind == "batch"
        target = self if in_place else self.clone()
        res = target.apply_arrays(pack(leaves), len(leaves), is_batch=is_batch)
        if res.code == 0:
            return Ok(target)
        if res.code == 1:
            return Err(InvalidPath())
        return Err(OperationFailed(leaves[res.err_index]))

    def apply(self, op) -> Any:
        """CRDTree.apply (src/CRDTree.elm:265-269): Ok(new tree) | Err(error)."""
        return self._apply(op, in_place=False)

    def apply_in_place(self, op):
        return self._apply(op, in_place=True)

    # ---- local editing (src/CRDTree.elm:142-216) ----
    def _local(self, op):
        r = self.apply(op)
        if r.ok:
            t = r.value
            # applyLocal sets the cursor to buildPath ts path (src/CRDTree.elm:310, :628-632)
            path = list(op.path)
            t._cursor = path[:-1] + [op.ts if op.kind == "add" else (path[-1] if path else 0)]
        return r

    def add(self, value):
        return self.add_after(self._cursor, value)

    def add_after(self, path, value):
        """CRDTree.addAfter: Add (nextTimestamp tree) path value."""
        return self._local(Add(self.timestamp() + 1, path, value))

    def add_branch(self, value):
        r = self.add(value)
        if r.ok:
            r.value._cursor = r.value._cursor + [0]
        return r

    def delete(self, path):
        return self._local(Delete(path))

    def batch(self, funcs):
        """CRDTree.batch (src/CRDTree.elm:224-232) over functions tree -> Result."""
        cur = self
        ops = []
        for f in funcs:
            r = f(cur)
            if not r.ok:
                return r
            nxt = r.value
            lo = nxt.last_operation()
            ops.extend(lo.ops if lo.kind == "batch" else [lo])
            cur = nxt
        cur._last_override = Batch(ops)
        return Ok(cur)

    # ---- queries ----
    def cursor(self):
        return list(self._cursor)

    def timestamp(self) -> int:
        v = C.c_int64()
        N.check(N.lib().crdtm_tree_timestamp(self._h, C.byref(v)))
        return v.value

    def id(self) -> int:
        return replica_id(self.timestamp())

    def next_timestamp(self) -> int:
        return self.timestamp() + 1

    def replicas(self) -> dict:
        n = C.c_uint64()
        N.check(N.lib().crdtm_tree_replicas(self._h, None, None, 0, C.byref(n)))
        ids = np.zeros(max(n.value, 1), np.int64)
        tss = np.zeros(max(n.value, 1), np.int64)
        N.check(N.lib().crdtm_tree_replicas(self._h, _ptr(ids), _ptr(tss), n.value, C.byref(n)))
        return {int(a): int(b) for a, b in zip(ids[:n.value], tss[:n.value])}

    def last_replica_timestamp(self, rid: int) -> int:
        """CRDTree.lastReplicaTimestamp (src/CRDTree.elm:637-639)."""
        return self.replicas().get(rid, 0)

    def _ops(self, which, since=None):
        o = N.Ops()
        isb = C.c_int(1)

        def fetch(ops):
            if since is None:
                N.check(N.lib().crdtm_tree_ops(self._h, which, C.byref(ops), C.byref(isb)))
            else:
                N.check(N.lib().crdtm_tree_ops_since(self._h, since, C.byref(ops)))

        fetch(o)
        n, npth = o.n_ops, o.n_path
        kind = np.zeros(n + 1, np.uint8)
        ts = np.zeros(n + 1, np.int64)
        off = np.zeros(n + 1, np.uint32)
        path = np.zeros(npth + 1, np.int64)
        val = np.zeros(n + 1, np.uint32)
        o2 = N.Ops(n, npth, _ptr(kind), _ptr(ts), _ptr(off), _ptr(path), _ptr(val), None)
        fetch(o2)
        out = []
        for i in range(n):
            p = [int(x) for x in path[off[i]:off[i + 1]]]
            out.append(Add(int(ts[i]), p, VALUES.value(int(val[i]))) if kind[i] == 0 else Delete(p))
        return out, bool(isb.value)

    def operations(self) -> list:
        """The log oldest-first (operationsSince 0)."""
        return self._ops(0)[0]

    def last_operation(self):
        """CRDTree.lastOperation (src/CRDTree.elm:371-373)."""
        ov = getattr(self, "_last_override", None)
        if ov is not None:
            return ov
        ops, isb = self._ops(1)
        return Batch(ops) if isb else ops[0]

    def operations_since(self, ts: int) -> Batch:
        """CRDTree.operationsSince (src/CRDTree.elm:408-418): inclusive of the
        newest logged Add with that ts, [] when absent (crdtm_tree_ops_since)."""
        return Batch(self._ops(0, since=ts)[0])

    # ---- traversal (src/CRDTree.elm:421-625, src/CRDTree/Node.elm:96-174) ----
    # Nodes are returned as NodeView(ref, kind, value, path, next); refs stay
    # valid until the next apply.
    def _view(self, ref):
        if ref == N.REF_NONE:
            return None
        kind = C.c_int32()
        val = C.c_uint32()
        hn = C.c_int32()
        nx = C.c_int64()
        pl = C.c_uint64()
        buf = np.zeros(64, np.int64)
        N.check(N.lib().crdtm_node_info(self._h, ref, C.byref(kind), C.byref(val), C.byref(hn), C.byref(nx),
                                        _ptr(buf), 64, C.byref(pl)), "crdtm_node_info")
        if pl.value > 64:
            buf = np.zeros(pl.value, np.int64)
            N.check(N.lib().crdtm_node_info(self._h, ref, None, None, None, None, _ptr(buf), pl.value, C.byref(pl)))
        k = {1: "node", 2: "tombstone", 3: "root"}[kind.value]
        return NodeView(ref, k, VALUES.value(val.value) if k == "node" else None,
                        [int(x) for x in buf[:pl.value]], int(nx.value) if hn.value else None)

    def get(self, path):
        """CRDTree.get (src/CRDTree.elm:468-470): the Node / Tombstone at path, or None."""
        ref = C.c_uint64()
        p = np.array(list(path) or [0], np.int64)
        N.check(N.lib().crdtm_tree_get(self._h, _ptr(p), len(path), C.byref(ref)), "crdtm_tree_get")
        return self._view(ref.value)

    def get_value(self, path):
        """CRDTree.getValue (src/CRDTree.elm:486-488)."""
        v = self.get(path)
        return v.value if v is not None and v.kind == "node" else None

    def root(self):
        return self._view(N.REF_ROOT)

    def _rel(self, node, which):
        out = C.c_uint64()
        N.check(N.lib().crdtm_tree_relative(self._h, node.ref, which, C.byref(out)), "crdtm_tree_relative")
        return self._view(out.value)

    def parent(self, node):
        """CRDTree.parent (src/CRDTree.elm:425-441)."""
        return self._rel(node, N.REL_PARENT)

    def next(self, node):
        """CRDTree.next (src/CRDTree.elm:560-566)."""
        return self._rel(node, N.REL_NEXT)

    def prev(self, node):
        """CRDTree.prev (src/CRDTree.elm:569-575)."""
        return self._rel(node, N.REL_PREV)

    def head(self, node):
        """CRDTree.Node.head (src/CRDTree/Node.elm:165-167)."""
        return self._rel(node, N.REL_HEAD)

    def _refs(self, fn, ref):
        n = C.c_uint64()
        N.check(fn(self._h, ref, None, 0, C.byref(n)))
        buf = np.zeros(max(n.value, 1), np.uint64)
        N.check(fn(self._h, ref, _ptr(buf), n.value, C.byref(n)))
        return [self._view(int(r)) for r in buf[:n.value]]

    def children(self, node):
        """CRDTree.Node.children (src/CRDTree/Node.elm:96-98): live children in order."""
        return self._refs(N.lib().crdtm_node_children, node.ref)

    def walk(self, func, acc, start=None):
        """CRDTree.walk (src/CRDTree.elm:583-625): func(node, acc) -> ("take", acc) | ("done", acc)."""
        for node in self._refs(N.lib().crdtm_tree_walk, N.REF_NONE if start is None else start.ref):
            step, acc = func(node, acc)
            if step == "done":
                return acc
        return acc

    def walk_nodes(self, start=None):
        """The visit order of walk when func always Takes."""
        return self._refs(N.lib().crdtm_tree_walk, N.REF_NONE if start is None else start.ref)

    def canonical(self, which=0, full=True):
        n = C.c_uint64()
        h = C.c_uint64()
        if not full:
            N.check(N.lib().crdtm_tree_canonical(self._h, which, None, 0, C.byref(n), C.byref(h)))
            return None, n.value, h.value
        N.check(N.lib().crdtm_tree_canonical(self._h, which, None, 0, C.byref(n), C.byref(h)))
        buf = np.zeros(max(n.value, 1), np.int64)
        N.check(N.lib().crdtm_tree_canonical(self._h, which, _ptr(buf), n.value, C.byref(n), C.byref(h)))
        return buf[:n.value], n.value, h.value

    def document_handles(self) -> np.ndarray:
        """Value handles of the visible nodes in document order (device linearisation)."""
        n = C.c_uint64()
        N.check(N.lib().crdtm_tree_document(self._h, None, 0, C.byref(n)))
        out = np.zeros(max(n.value, 1), np.uint32)
        N.check(N.lib().crdtm_tree_document(self._h, _ptr(out), n.value, C.byref(n)))
        return out[:n.value]

    def document(self) -> list:
        return [VALUES.value(int(h)) for h in self.document_handles()]

    def visible_values(self, depth0_only=True):
        words, n, _ = self.canonical(1)
        out = []
        i = 0
        while i < n:
            d, v, pl = int(words[i]), int(words[i + 1]), int(words[i + 2])
            if d == 0 or not depth0_only:
                out.append(VALUES.value(v))
            i += 3 + pl
        return out


def init(replica_id_: int, device: int = 0) -> CRDTree:
    return CRDTree.init(replica_id_, device)


__all__ = ["CRDTree", "init", "Ok", "Err", "InvalidPath", "NotFound", "OperationFailed", "TWO32"]


def forest_apply(arrs, doc_off, replica_id=0, device=0, on_device=False):
    """crdtm_forest_apply: every document fresh, `apply (Batch ops_d)` each.
    Returns dict of per-document numpy arrays (code, err, applied, hash, words, timestamp)."""
    n_docs = len(doc_off) - 1
    ctx = N.context(device)
    doc_off = np.ascontiguousarray(doc_off, dtype=np.uint32)
    out = dict(code=np.zeros(n_docs, np.int32), err=np.zeros(n_docs, np.int64), applied=np.zeros(n_docs, np.uint32),
               hash=np.zeros(n_docs, np.uint64), words=np.zeros(n_docs, np.uint64),
               timestamp=np.zeros(n_docs, np.int64))
    ops = arrs if isinstance(arrs, N.Ops) else ops_struct(arrs, int(doc_off[-1]))
    rc = N.lib().crdtm_forest_apply(ctx, int(replica_id), C.byref(ops), _ptr(doc_off), n_docs, 1 if on_device else 0,
                                    _ptr(out["code"]), _ptr(out["err"]), _ptr(out["applied"]), _ptr(out["hash"]),
                                    _ptr(out["words"]), _ptr(out["timestamp"]))
    out["rc"] = rc
    return out
