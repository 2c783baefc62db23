"""Helpers comparing the HIP engine with the CPU oracle on identical inputs."""
import ctypes as C

import numpy as np

from oracle.oracle import lib as olib, _ptr as optr


def oracle_apply_arrays(arrs, n, replica=0, is_batch=True, tree=None):
    L = olib()
    t = tree if tree is not None else L.orc_init(replica)
    err = C.c_int64(-1)
    r = L.orc_apply(t, 1 if is_batch else 0, 0, n, optr(arrs["kind"]), optr(arrs["ts"]), optr(arrs["path_off"]),
                    optr(arrs["path"]), optr(arrs["val"]), C.byref(err))
    return t, r, err.value


def oracle_summary(t):
    L = olib()
    out = {}
    for which in (0, 1):
        h = C.c_uint64()
        n = L.orc_canonical(t, which, None, 0, C.byref(h))
        out[which] = (n, h.value)
    out["ts"] = L.orc_timestamp(t)
    n = L.orc_replicas(t, None, None, 0)
    ids = np.zeros(max(n, 1), np.int64)
    tss = np.zeros(max(n, 1), np.int64)
    L.orc_replicas(t, optr(ids), optr(tss), n)
    out["replicas"] = {int(a): int(b) for a, b in zip(ids[:n], tss[:n])}
    return out


def oracle_log(t, which=0):
    """(kind, ts, path tuple, val) tuples of the log (0) or lastOperation (1), plus is_batch."""
    L = olib()
    pt = C.c_uint64(0)
    isb = C.c_int(0)
    n = L.orc_ops(t, which, None, None, None, None, None, C.byref(pt), C.byref(isb))
    kind = np.zeros(max(n, 1), np.uint8)
    ts = np.zeros(max(n, 1), np.int64)
    off = np.zeros(n + 1, np.uint32)
    path = np.zeros(max(pt.value, 1), np.int64)
    val = np.zeros(max(n, 1), np.uint32)
    L.orc_ops(t, which, optr(kind), optr(ts), optr(off), optr(path), optr(val), None, None)
    return log_tuples(kind, ts, off, path, val, n), bool(isb.value)


def log_tuples(kind, ts, off, path, val, n):
    return [(int(kind[i]), int(ts[i]) if kind[i] == 0 else 0, tuple(int(x) for x in path[off[i]:off[i + 1]]),
             int(val[i]) if kind[i] == 0 else 0) for i in range(n)]


def oracle_since(t, ts):
    """Operation.since (src/Internal/Operation.elm:25-53) over the oracle's log:
    newest-first walk, inclusive of the first Add with that ts; [] when absent;
    operationsSince 0 = the whole log (src/CRDTree.elm:408-418)."""
    log, _ = oracle_log(t, 0)
    if ts == 0:
        return log
    for j in range(len(log) - 1, -1, -1):
        if log[j][0] == 0 and log[j][1] == ts:
            return log[j:]
    return []


def engine_log(tree, which=0, since=None):
    import crdtm._native as N
    from crdtm.tree import _ptr
    o = N.Ops()
    isb = C.c_int(1)

    def fetch(ops):
        if since is None:
            N.check(N.lib().crdtm_tree_ops(tree._h, which, C.byref(ops), C.byref(isb)))
        else:
            N.check(N.lib().crdtm_tree_ops_since(tree._h, since, C.byref(ops)))

    fetch(o)
    n, npth = o.n_ops, o.n_path
    kind = np.zeros(n + 1, np.uint8)
    ts = np.zeros(n + 1, np.int64)
    off = np.zeros(n + 1, np.uint32)
    path = np.zeros(npth + 1, np.int64)
    val = np.zeros(n + 1, np.uint32)
    o2 = N.Ops(n, npth, _ptr(kind), _ptr(ts), _ptr(off), _ptr(path), _ptr(val), None)
    fetch(o2)
    return log_tuples(kind, ts, off, path, val, n), bool(isb.value)


def engine_log_arrays(tree, which=0):
    """The log (0) or lastOperation (1) as packed numpy arrays (kind, ts,
    path_off, path, val) plus is_batch, for full-size comparisons."""
    import crdtm._native as N
    from crdtm.tree import _ptr
    o = N.Ops()
    isb = C.c_int(1)
    N.check(N.lib().crdtm_tree_ops(tree._h, which, C.byref(o), C.byref(isb)))
    n, npth = o.n_ops, o.n_path
    out = dict(kind=np.zeros(n + 1, np.uint8), ts=np.zeros(n + 1, np.int64), path_off=np.zeros(n + 1, np.uint32),
               path=np.zeros(npth + 1, np.int64), val=np.zeros(n + 1, np.uint32))
    o2 = N.Ops(n, npth, _ptr(out["kind"]), _ptr(out["ts"]), _ptr(out["path_off"]), _ptr(out["path"]),
               _ptr(out["val"]), None)
    N.check(N.lib().crdtm_tree_ops(tree._h, which, C.byref(o2), C.byref(isb)))
    return dict(kind=out["kind"][:n], ts=out["ts"][:n], path_off=out["path_off"][:n + 1], path=out["path"][:npth],
                val=out["val"][:n]), bool(isb.value)


def engine_summary(tree):
    out = {}
    for which in (0, 1):
        _, n, h = tree.canonical(which, full=False)
        out[which] = (n, h)
    out["ts"] = tree.timestamp()
    out["replicas"] = tree.replicas()
    return out


def oracle_visible_vals(t):
    """Value handles of the visible document (pre-order) from the oracle dump."""
    L = olib()
    h = C.c_uint64()
    n = L.orc_canonical(t, 1, None, 0, C.byref(h))
    buf = np.zeros(max(n, 1), np.int64)
    L.orc_canonical(t, 1, optr(buf), n, None)
    vals = []
    i = 0
    while i < n:
        pl = int(buf[i + 2])
        vals.append(int(buf[i + 1]))
        i += 3 + pl
    return np.array(vals, np.uint32)
