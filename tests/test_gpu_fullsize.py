"""Full-size GPU checks (BASELINE.json config 3: 10M flat inserts, 64
replicas) through size-independent properties, where the general CPU
restatement would take hours (its findInsertion walks grow with the
document).

* every op applies, the document holds each key once, the visible-order
  walk of the committed `next` chain (host) and the device linearisation
  (`doc`) give the same values;
* the RGA order properties of oracle/crdtree_oracle.cpp `orc_flat_check`:
  each key after its anchor, every key between them larger (what every
  findInsertion walk guarantees for an Adds-only flat batch);
* exact parity over all 10M ops: canonical structure and visible digests
  and their word counts equal the searched flat restatement's
  (`orc_flat_replay`: findInsertion's stop node through a treap, pinned
  against the literal walk in tests/test_oracle_flat.py, which
  tests/test_oracle_kat.py pins against the general restatement); the
  reference behaviour is src/Internal/Node.elm:93-104 over 10M siblings;
* the merge's other outputs at 10M, derived in numpy for an Adds-only batch
  on a fresh tree (src/CRDTree.elm:298-325, :337-343): the op log and
  lastOperation are the batch itself (every op Applied, in batch order), the
  replicas table holds each replica's last Add (last writer), and the
  timestamp counts the observer's own-replica Adds.
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from crdtm import _native as N  # noqa: E402
from crdtm.tree import CRDTree  # noqa: E402
from oracle.oracle import _ptr, lib as olib  # noqa: E402
from parity_util import engine_log_arrays  # noqa: E402

CFG3 = dict(replicas=64, window=256, seed=0xC0FFEE03)


def test_flat10m_order_properties():
    n = 10_000_000
    s = N.synth(n_ops=n, **CFG3)
    t = CRDTree.init(0)
    res = t.apply_arrays(s, n)
    assert res.code == 0 and res.path_taken == N.PATH_CLOSED_FORM
    assert res.n_applied == n
    words, nw, _ = t.canonical(1, full=True)
    assert nw == 4 * n
    keys = words[3::4].copy()
    assert np.array_equal(words[2::4], np.ones(n, np.int64)) and not words[0::4].any()
    # device linearisation == host walk of the next chain
    assert np.array_equal(t.document_handles().astype(np.int64), words[1::4])
    bad = olib().orc_flat_check(n, _ptr(keys), n, _ptr(s["ts"]), _ptr(s["path_off"]), _ptr(s["path"]))
    assert bad == 0, bad
    # exact: the whole batch through the searched restatement (~15 s on one core)
    h = np.zeros(2, np.uint64)
    w = np.zeros(2, np.uint64)
    err = C.c_int64(-1)
    na = C.c_uint64()
    rc = olib().orc_flat_replay(n, _ptr(s["kind"]), _ptr(s["ts"]), _ptr(s["path_off"]), _ptr(s["path"]),
                                _ptr(s["val"]), C.byref(err), _ptr(h), _ptr(w), C.byref(na))
    assert rc == 0 and na.value == n
    for which in (0, 1):
        _, enw, eh = t.canonical(which, full=False)
        assert (enw, eh) == (int(w[which]), int(h[which])), which
    check_flat_outputs(t, s, n)


def check_flat_outputs(t, s, n, replica=0):
    """Log, lastOperation, replicas and timestamp of an Adds-only batch merged
    into a fresh `init replica` tree, every op Applied."""
    for which in (0, 1):  # operations (oldest first) and lastOperation (src/CRDTree.elm:311, :328-334)
        lg, isb = engine_log_arrays(t, which)
        assert isb
        for f in ("kind", "ts", "path_off", "path", "val"):
            assert np.array_equal(lg[f], s[f][:len(lg[f])]) and len(lg[f]) == len(s[f][:n + (f == "path_off")]), \
                (which, f)
    rid = s["ts"][:n] >> 32  # Timestamp.replicaId (src/CRDTree/Timestamp.elm:16-18): ts >= 0 here
    ids, first_rev = np.unique(rid[::-1], return_index=True)
    last = n - 1 - first_rev  # each replica's last Add in batch order: replicas[r] := ts (last writer)
    assert t.replicas() == {int(r): int(s["ts"][i]) for r, i in zip(ids, last)}
    assert t.timestamp() == replica * 2 ** 32 + int(np.count_nonzero(rid == replica))


def test_flat1m_matches_fast_restatement():
    m = 1_000_000
    s = N.synth(n_ops=m, **CFG3)
    t = CRDTree.init(0)
    assert t.apply_arrays(s, m).code == 0
    h = np.zeros(2, np.uint64)
    w = np.zeros(2, np.uint64)
    err = C.c_int64(-1)
    na = C.c_uint64()
    rc = olib().orc_flat_replay(m, _ptr(s["kind"]), _ptr(s["ts"]), _ptr(s["path_off"]), _ptr(s["path"]),
                                _ptr(s["val"]), C.byref(err), _ptr(h), _ptr(w), C.byref(na))
    assert rc == 0 and na.value == m
    for which in (0, 1):
        _, enw, eh = t.canonical(which, full=False)
        assert (enw, eh) == (int(w[which]), int(h[which])), which
    check_flat_outputs(t, s, m)
