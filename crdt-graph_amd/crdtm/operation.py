"""Operation algebra — host mirror of `CRDTree.Operation` / `Internal.Operation`.

Reference: src/Internal/Operation.elm:17-119 (type, since, toList, fromList,
merge, replicaId, timestamp, path) and src/CRDTree/Operation.elm:53-159
(public re-exports, JSON encoder/decoder). The JSON codec itself is native
(crdt-graph_amd/csrc/json_codec.cpp) and reached through `crdtm._native`.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, List, Optional

from .timestamp import replica_id as _replica_id


@dataclass(frozen=True)
class Add:
    """Add Int (List Int) a (src/Internal/Operation.elm:18)."""
    ts: int
    path: tuple
    val: Any
    kind = "add"

    def __init__(self, ts, path, val):
        object.__setattr__(self, "ts", int(ts))
        object.__setattr__(self, "path", tuple(int(x) for x in path))
        object.__setattr__(self, "val", val)


@dataclass(frozen=True)
class Delete:
    """Delete (List Int) (src/Internal/Operation.elm:19)."""
    path: tuple
    kind = "del"

    def __init__(self, path):
        object.__setattr__(self, "path", tuple(int(x) for x in path))


@dataclass(frozen=True)
class Batch:
    """Batch (List (Operation a)) (src/Internal/Operation.elm:20)."""
    ops: tuple = field(default_factory=tuple)
    kind = "batch"

    def __init__(self, ops=()):
        object.__setattr__(self, "ops", tuple(ops))


Operation = Any  # Add | Delete | Batch


def to_list(op) -> List:
    """Operation.toList (src/Internal/Operation.elm:58-68)."""
    return list(op.ops) if op.kind == "batch" else [op]


def from_list(ops) -> Batch:
    """Operation.fromList (src/Internal/Operation.elm:73-75)."""
    return Batch(ops)


def merge(a, b) -> Batch:
    """Operation.merge a b = Batch (toList a ++ toList b) (src/Internal/Operation.elm:80-82)."""
    return Batch(to_list(a) + to_list(b))


def timestamp(op) -> Optional[int]:
    """Operation.timestamp (src/Internal/Operation.elm:94-104): Delete -> last path element."""
    if op.kind == "add":
        return op.ts
    if op.kind == "del":
        return op.path[-1] if op.path else None
    return None


def path(op) -> Optional[list]:
    """Operation.path (src/Internal/Operation.elm:109-119)."""
    return None if op.kind == "batch" else list(op.path)


def replica_id(op) -> Optional[int]:
    """Operation.replicaId (src/Internal/Operation.elm:87-89)."""
    t = timestamp(op)
    return None if t is None else _replica_id(t)


def since(ts: int, operations_newest_first: list) -> list:
    """Operation.since / sinceFold (src/Internal/Operation.elm:25-53)."""
    acc = []
    for o in operations_newest_first:
        if o.kind == "batch":
            continue
        acc.insert(0, o)
        if o.kind == "add" and o.ts == ts:
            return acc
    return []


def flatten(op, out=None) -> list:
    """Leaves of nested Batches in application order. `apply (Batch ops)` is
    equivalent to applying the flattened leaves in order (src/CRDTree.elm:224-232,
    :294-295; lastOperation is always flat via merge/toList)."""
    if out is None:
        out = []
    if op.kind == "batch":
        for o in op.ops:
            flatten(o, out)
    else:
        out.append(op)
    return out
