"""GPU parity: the HIP engine (through the C ABI) against the CPU oracle.

Bit-exact on every output the reference defines: dict structure (every entry,
incl. tombstones, sentinels and copy-quirk orphans), visible document order,
operation log, lastOperation, timestamp and replicas; plus the device
document-order linearisation against the oracle's pre-order.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from crdtm import _native as N  # noqa: E402
from crdtm.operation import flatten  # noqa: E402
from crdtm.tree import CRDTree, pack  # noqa: E402
from kat_cases import SCENARIOS  # noqa: E402
from parity_util import (engine_log, engine_summary, oracle_apply_arrays, oracle_log, oracle_since,  # noqa: E402
                         oracle_summary, oracle_visible_vals)


def run_both(replica, calls):
    """Apply each top-level op to a fresh oracle tree and a fresh engine tree."""
    from oracle.oracle import lib as olib
    ot = olib().orc_init(replica)
    et = CRDTree.init(replica)
    results = []
    for op in calls:
        leaves = flatten(op) if op.kind == "batch" else [op]
        arrs = pack(leaves)
        n = len(leaves)
        _, rc, oerr = oracle_apply_arrays(arrs, n, is_batch=op.kind == "batch", tree=ot)
        res = et.apply_arrays(arrs, n, is_batch=op.kind == "batch")
        results.append((rc, oerr, res.code, res.err_index, res.path_taken))
    return ot, et, results


@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_scenarios(name):
    replica, calls = SCENARIOS[name]
    ot, et, results = run_both(replica, calls)
    for rc, oerr, code, eerr, _ in results:
        assert code == rc, (name, results)
        if rc != 0:
            assert eerr == oerr
    assert engine_summary(et) == oracle_summary(ot)
    assert engine_log(et, 0) == oracle_log(ot, 0)
    assert engine_log(et, 1) == oracle_log(ot, 1)
    assert np.array_equal(et.document_handles(), oracle_visible_vals(ot))


def synth_case(**kw):
    s = N.synth(**kw)
    return s, len(s["kind"])


CASES = {
    # config 1 (2 replicas, 70/30 interleaved, depth <= 3): quirks fire -> exact replay
    "cfg1": dict(n_ops=10000, replicas=2, window=8, p_delete=0.3, p_branch=0.05, max_depth=3, seed=0xC0FFEE01),
    # config 2 shape at reduced size (16 replicas, 80/20, branches, depth <= 4)
    "cfg2_small": dict(n_ops=20000, replicas=16, window=64, p_delete=0.2, p_branch=0.1, max_depth=4,
                       seed=0xC0FFEE02),
    # config 3 shape (flat, adds only, 64 replicas): closed form
    "cfg3_small": dict(n_ops=50000, replicas=64, window=256, seed=0xC0FFEE03),
    # config 4 shape (depth 12, <= 8 children, deletes after adds): closed form with tombstones
    "cfg4_small": dict(n_ops=60000, replicas=16, p_delete=1 / 3, max_depth=12, max_children=8, deletes_last=1,
                       seed=0xC0FFEE04),
    # flat with deletes after adds
    "flat_deletes_last": dict(n_ops=30000, replicas=8, window=32, p_delete=0.4, deletes_last=1, seed=7),
    # nested, adds only
    "nested_adds": dict(n_ops=30000, replicas=8, window=16, p_branch=0.2, max_depth=6, seed=11),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_synthetic_streams(name):
    s, n = synth_case(**CASES[name])
    ot, rc, oerr = oracle_apply_arrays(s, n)
    et = CRDTree.init(0)
    res = et.apply_arrays(s, n)
    assert res.code == rc
    if rc == 0:
        assert engine_summary(et) == oracle_summary(ot)
        assert engine_log(et, 0) == oracle_log(ot, 0)
        assert np.array_equal(et.document_handles(), oracle_visible_vals(ot))
    if name in ("cfg3_small", "cfg4_small", "flat_deletes_last", "nested_adds"):
        assert res.path_taken == N.PATH_CLOSED_FORM, f"expected the closed form, guard={res.guard}"


@pytest.mark.parametrize("lane", ["32", "0"])
@pytest.mark.parametrize("chunk", range(8))
def test_adversarial_streams(monkeypatch, chunk, lane):
    """Interleaved Deletes and tombstone walks (copy quirks, nested dicts):
    the per-dict replay, its conflict fallback and the sequential replay all
    match the oracle. lane: dicts of at most that many slots replay one per
    lane (k_pdr_lane, the default), or (0) every dict on a wave (pdr_serial)."""
    from adversarial import adversarial
    monkeypatch.setenv("CRDTM_PDR_LANE", lane)
    paths = {}
    for seed in range(16 * chunk, 16 * chunk + 16):
        n = [40, 120, 400, 1500][seed % 4]
        ops = adversarial(seed, n, replicas=2 + seed % 3, max_depth=1 + seed % 4)
        arrs = pack(ops)
        ot, rc, oerr = oracle_apply_arrays(arrs, n)
        et = CRDTree.init(0)
        res = et.apply_arrays(arrs, n)
        paths[res.path_taken] = paths.get(res.path_taken, 0) + 1
        assert res.code == rc, (seed, res.code, rc)
        if rc != 0:
            assert res.err_index == oerr, seed
            continue
        assert engine_summary(et) == oracle_summary(ot), seed
        assert engine_log(et, 0) == oracle_log(ot, 0), seed
        assert np.array_equal(et.document_handles(), oracle_visible_vals(ot)), seed
    assert paths.get(N.PATH_DICT_REPLAY, 0) > 0, paths


def test_snapshots_from_change_logs(monkeypatch):
    """Copy-quirk snapshots rebuilt from every dict's change log (forced on
    for all dict sizes) match the oracle like the re-replayed ones."""
    from adversarial import adversarial
    monkeypatch.setenv("CRDTM_PDR_LOG_MIN", "1")
    for seed in range(0, 128, 3):
        n = [40, 120, 400, 1500][seed % 4]
        ops = adversarial(seed, n, replicas=2 + seed % 3, max_depth=1 + seed % 4)
        arrs = pack(ops)
        ot, rc, oerr = oracle_apply_arrays(arrs, n)
        et = CRDTree.init(0)
        res = et.apply_arrays(arrs, n)
        assert res.code == rc, seed
        if rc == 0:
            assert engine_summary(et) == oracle_summary(ot), seed
    s, n = synth_case(**CASES["cfg2_small"])
    ot, rc, _ = oracle_apply_arrays(s, n)
    et = CRDTree.init(0)
    assert et.apply_arrays(s, n).code == rc == 0
    assert engine_summary(et) == oracle_summary(ot)


def test_operations_since_matches_oracle():
    """operationsSince through the device search (crdtm_tree_ops_since) against
    the oracle's newest-first walk (src/Internal/Operation.elm:25-53), incl. the
    reference test's vectors (tests/CRDTreeTest.elm:592-658)."""
    replica, calls = SCENARIOS["operations_since"]
    ot, et, results = run_both(replica, calls)
    full = tuple(et.operations())
    assert et.operations_since(0).ops == full
    assert et.operations_since(2).ops == full[1:]
    assert et.operations_since(6).ops == full[-1:]
    assert et.operations_since(10).ops == ()
    s, n = synth_case(n_ops=5000, replicas=4, window=16, p_delete=0.2, p_branch=0.1, max_depth=3, seed=21)
    ot, rc, _ = oracle_apply_arrays(s, n)
    et = CRDTree.init(0)
    assert et.apply_arrays(s, n).code == rc == 0
    rng = np.random.default_rng(3)
    adds = s["ts"][s["kind"] == 0]
    for want in list(rng.choice(adds, 16)) + [0, 12345]:
        assert engine_log(et, since=int(want))[0] == oracle_since(ot, int(want)), int(want)


def test_incremental_batches():
    """Successive applies of chunks equal one apply of the whole stream's chunks on the oracle."""
    s, n = synth_case(n_ops=20000, replicas=8, window=16, p_delete=0.2, p_branch=0.1, max_depth=3, seed=5)
    from oracle.oracle import lib as olib
    ot = olib().orc_init(0)
    et = CRDTree.init(0)
    off = s["path_off"]
    for a in range(0, n, 5000):
        b = min(n, a + 5000)
        chunk = dict(kind=s["kind"][a:b].copy(), ts=s["ts"][a:b].copy(), val=s["val"][a:b].copy(),
                     path_off=(off[a:b + 1] - off[a]).astype(np.uint32), path=s["path"][off[a]:off[b]].copy())
        _, rc, _ = oracle_apply_arrays(chunk, b - a, tree=ot)
        res = et.apply_arrays(chunk, b - a)
        assert res.code == rc == 0
        assert engine_summary(et) == oracle_summary(ot)
    assert engine_log(et, 0) == oracle_log(ot, 0)
    assert engine_log(et, 1) == oracle_log(ot, 1)


def test_error_leaves_tree_unchanged():
    et = CRDTree.init(0)
    from crdtm.operation import Add, Batch
    r = et.apply_in_place(Batch([Add(1, [0], "a"), Add(2, [1], "b")]))
    assert r.ok
    before = engine_summary(et)
    r = et.apply_in_place(Batch([Add(3, [2], "c"), Add(4, [99], "d")]))
    assert not r.ok and type(r.error).__name__ == "OperationFailed"
    assert engine_summary(et) == before


def test_forest_matches_oracle_per_document():
    """Config 5 shape: many independent documents, exact replay per document."""
    import ctypes as C
    from crdtm.tree import forest_apply
    from oracle.oracle import lib as olib, _ptr as optr
    n_docs, per = 300, 1000
    s = N.synth(n_ops=per, n_docs=n_docs, replicas=8, window=16, p_delete=0.2, seed=0xC0FFEE05)
    doc_off = np.searchsorted(s["tree"], np.arange(n_docs + 1)).astype(np.uint32)
    out = forest_apply(s, doc_off)
    assert out["rc"] == 0
    L = olib()
    for d in range(0, n_docs, 7):
        a, b = int(doc_off[d]), int(doc_off[d + 1])
        off = s["path_off"]
        sub = dict(kind=s["kind"][a:b].copy(), ts=s["ts"][a:b].copy(), val=s["val"][a:b].copy(),
                   path_off=(off[a:b + 1] - off[a]).astype(np.uint32), path=s["path"][off[a]:off[b]].copy())
        t, rc, err = oracle_apply_arrays(sub, b - a)
        assert out["code"][d] == rc
        h = C.c_uint64()
        nw = L.orc_canonical(t, 1, None, 0, C.byref(h))
        assert (int(out["words"][d]), int(out["hash"][d])) == (nw, h.value), f"document {d}"
        assert int(out["timestamp"][d]) == L.orc_timestamp(t)
        L.orc_free(t)
    # the same document through the single-tree API gives the same visible hash
    d = 5
    a, b = int(doc_off[d]), int(doc_off[d + 1])
    off = s["path_off"]
    sub = dict(kind=s["kind"][a:b].copy(), ts=s["ts"][a:b].copy(), val=s["val"][a:b].copy(),
               path_off=(off[a:b + 1] - off[a]).astype(np.uint32), path=s["path"][off[a]:off[b]].copy())
    et = CRDTree.init(0)
    et.apply_arrays(sub, b - a)
    _, nw, hh = et.canonical(1, full=False)
    assert (nw, hh) == (int(out["words"][d]), int(out["hash"][d]))


def _forest_doc(seed, n_ops, fmap=None, edits=()):
    """One flat synthetic document as rows (kind, ts, path, val); `fmap` remaps
    every key (timestamps and path keys alike, 0 stays the sentinel)."""
    s = N.synth(n_ops=n_ops, n_docs=1, replicas=8, window=16, p_delete=0.2, seed=seed)
    f = (lambda k: k if k == 0 else fmap(k)) if fmap else (lambda k: k)
    off = s["path_off"]
    rows = [(int(s["kind"][i]), f(int(s["ts"][i])), [f(int(x)) for x in s["path"][off[i]:off[i + 1]]], int(s["val"][i]))
            for i in range(len(s["kind"]))]
    for at, row in sorted(edits, key=lambda e: -e[0]):
        rows.insert(at, row)
    return rows


@pytest.mark.parametrize("layout", ["dense", "holes", "big_replica", "wide_range", "negative", "mixed"])
def test_forest_slot_map_edges(layout):
    """k_forest_prep's two slot maps (dense per-replica ranges; bitonic sort when
    a key is negative, a replica id >= 64 or the ranges exceed 1,024 slots) and
    the ops they must agree on -- duplicate keys, ts 0, anchors and deletes of
    in-range keys no Add owns, empty paths -- against the oracle per document."""
    import ctypes as C
    from crdtm.tree import forest_apply
    from oracle.oracle import lib as olib
    R = lambda r, c: (r << 32) | c
    maps = {"dense": None, "holes": lambda k: R(k >> 32, (k & 0xFFFFFFFF) * 3 + 7),
            "big_replica": lambda k: k + (100 << 32), "wide_range": lambda k: k + (5000 if (k >> 32) == 3 else 0),
            "negative": None, "mixed": None}
    docs = []
    for j in range(12):
        fm = maps[layout]
        if layout == "mixed":
            fm = [None, maps["holes"], maps["big_replica"], maps["wide_range"]][j % 4]
        base = _forest_doc(0xF0 + j, 300, fm)
        add0 = [r for r in base if r[0] == 0]
        k = j % 6
        if k == 1:  # duplicate of an earlier Add, later in the stream
            base.insert(250, add0[40])
        elif k == 2:  # ts 0 Add (collides with the sentinel: AlreadyApplied)
            base.insert(100, (0, 0, [0], 9))
        elif k == 3 and layout in ("holes", "mixed"):  # anchor on a hole key (NotFound)
            a = add0[10][1]
            base.insert(200, (0, R(7, 999999), [a + 1], 9))
        elif k == 4:  # empty path (InvalidPath)
            base.insert(150, (0, R(7, 999998), [], 9))
        elif k == 5:  # delete of a never-added in-range key
            base.insert(120, (1, 0, [add0[5][1] + 1], 0))
        if layout == "negative" and j % 2 == 0:
            base.insert(50, (0, -5, [0], 3))
        docs.append(base)
    rows = [r for d in docs for r in d]
    doc_off = np.zeros(len(docs) + 1, np.uint32)
    doc_off[1:] = np.cumsum([len(d) for d in docs])
    poff = np.zeros(len(rows) + 1, np.uint32)
    poff[1:] = np.cumsum([len(r[2]) for r in rows])
    s = dict(kind=np.array([r[0] for r in rows], np.uint8), ts=np.array([r[1] for r in rows], np.int64),
             path_off=poff, path=np.array([x for r in rows for x in r[2]] + [0], np.int64),
             val=np.array([r[3] for r in rows], np.uint32))
    out = forest_apply(s, doc_off)
    L = olib()
    for d in range(len(docs)):
        a, b = int(doc_off[d]), int(doc_off[d + 1])
        sub = dict(kind=s["kind"][a:b].copy(), ts=s["ts"][a:b].copy(), val=s["val"][a:b].copy(),
                   path_off=(poff[a:b + 1] - poff[a]).astype(np.uint32), path=s["path"][poff[a]:poff[b]].copy())
        t, rc, err = oracle_apply_arrays(sub, b - a)
        assert out["code"][d] == rc, f"document {d}"
        if rc == 0:
            h = C.c_uint64()
            nw = L.orc_canonical(t, 1, None, 0, C.byref(h))
            assert (int(out["words"][d]), int(out["hash"][d])) == (nw, h.value), f"document {d}"
            assert int(out["timestamp"][d]) == L.orc_timestamp(t)
        L.orc_free(t)


def _flat_variant(s, edits):
    """Rebuild a flat stream (path length 1) with edits: ('ins', k, ts, anchor)
    inserts an Add at position k; ('empty', k) inserts an Add with path []."""
    n = len(s["kind"])
    rows = [(int(s["ts"][i]), [int(s["path"][s["path_off"][i]])], int(s["val"][i])) for i in range(n)]
    for e in sorted(edits, key=lambda e: -e[1]):
        if e[0] == "ins":
            rows.insert(e[1], (e[2], [e[3]], 7))
        else:
            rows.insert(e[1], (e[2], [], 7))
    m = len(rows)
    off = np.zeros(m + 1, np.uint32)
    off[1:] = np.cumsum([len(r[1]) for r in rows])
    path = np.array([x for r in rows for x in r[1]] + [0], np.int64)
    return dict(kind=np.zeros(m, np.uint8), ts=np.array([r[0] for r in rows], np.int64), path_off=off, path=path,
                val=np.array([r[2] for r in rows], np.uint32)), m


@pytest.mark.parametrize("case", ["dup_later", "dup_earlier", "ts_zero", "empty_path", "anchor_later",
                                  "anchor_missing", "anchor_cycle", "anchor_self", "anchor_gap", "clean"])
def test_flat_closed_form_edges(case):
    """The flat closed form's one-pass claim + per-slot anchor check, and its
    per-op fallback (duplicates, ts 0, errors), against the oracle."""
    s, n = synth_case(n_ops=20000, replicas=16, window=64, seed=0xC0FFEE03)
    ts, anc = s["ts"], s["path"]
    edits = {
        "clean": [],
        "dup_later": [("ins", 15000, int(ts[100]), int(anc[100])), ("ins", 18000, int(ts[9000]), 0)],
        "dup_earlier": [("ins", 12000, int(ts[15000]), int(ts[50]))],
        "ts_zero": [("ins", 500, 0, 0)],
        "empty_path": [("empty", 7000, int(ts[3]))],
        "anchor_later": [("ins", 4000, (40 << 32) + 5, (41 << 32) + 5), ("ins", 9000, (41 << 32) + 5, 0)],
        "anchor_missing": [("ins", 11000, (42 << 32) + 1, (43 << 32) + 9)],
        # (the flat path speculates that every op applies; these fail and must not derail its walks)
        "anchor_cycle": [("ins", 6000, (44 << 32) + 1, (44 << 32) + 2), ("ins", 6001, (44 << 32) + 2, (44 << 32) + 1)],
        "anchor_self": [("ins", 8000, (45 << 32) + 1, (45 << 32) + 1)],
        "anchor_gap": [("ins", 3000, (46 << 32) + 1, 0), ("ins", 3001, (46 << 32) + 5, (46 << 32) + 3)],
    }[case]
    v, m = _flat_variant(s, edits)
    ot, rc, oerr = oracle_apply_arrays(v, m)
    et = CRDTree.init(0)
    res = et.apply_arrays(v, m)
    assert res.path_taken == N.PATH_CLOSED_FORM
    assert res.code == rc, (case, res.code, rc)
    if rc != 0:
        assert res.err_index == oerr
        return
    assert (res.n_applied, res.n_already) == (len(oracle_log(ot, 0)[0]), m - len(oracle_log(ot, 0)[0]))
    assert engine_summary(et) == oracle_summary(ot)
    assert engine_log(et, 0) == oracle_log(ot, 0)
    assert np.array_equal(et.document_handles(), oracle_visible_vals(ot))


@pytest.mark.gpu
def test_flat_sibling_fans():
    """Sibling-sort tiers (tiny 3..16, mid ..512, big ..4096, huge beyond):
    fans of concurrent inserts that all anchor after one node, children of
    each fan spread over 60 replicas and shuffled, against the oracle."""
    rng = np.random.default_rng(0xFA45)
    sizes = [3, 5, 16, 17, 300, 512, 513, 2000, 4096, 4097, 9000]
    heads = [((1 << 32) + k + 1, 0) for k in range(len(sizes))]
    ctr = {}
    kids = []
    for k, K in enumerate(sizes):
        for j in range(K):
            r = 2 + int(rng.integers(0, 60))
            ctr[r] = ctr.get(r, 0) + 1
            kids.append(((r << 32) + ctr[r], heads[k][0]))
    kids = [kids[i] for i in rng.permutation(len(kids))]
    rows = heads + kids
    m = len(rows)
    v = dict(kind=np.zeros(m, np.uint8), ts=np.array([a for a, _ in rows], np.int64),
             path_off=np.arange(m + 1, dtype=np.uint32), path=np.array([b for _, b in rows] + [0], np.int64),
             val=np.arange(m, dtype=np.uint32))
    ot, rc, _ = oracle_apply_arrays(v, m)
    assert rc == 0
    et = CRDTree.init(0)
    res = et.apply_arrays(v, m)
    assert res.code == 0 and res.path_taken == N.PATH_CLOSED_FORM
    assert engine_summary(et) == oracle_summary(ot)
    assert np.array_equal(et.document_handles(), oracle_visible_vals(ot))


@pytest.mark.parametrize("depth", [3, 62, 63, 64, 65, 150])
def test_flat_run_tree_depth(depth):
    """The flat order by ep-run decomposition walks the tree of runs (a run
    hangs from the slot of its head's effective parent); chains of runs up
    to RUN_MAXD deep take it, deeper ones the generic Euler-tour list
    ranking. Replica k's first node anchors after replica k-1's first node
    (one run deeper each), its second after the sentinel, plus a typing
    stream around them; against the oracle."""
    rows = []
    for k in range(1, depth + 1):
        a = ((k - 1) << 32) + 1 if k > 1 else 0
        rows.append(((k << 32) + 1, a))
        rows.append(((k << 32) + 2, 0))
    rng = np.random.default_rng(depth)
    last = {}
    for j in range(3000):
        r = depth + 1 + int(rng.integers(0, 8))
        c = last.get(r, 0) + 1
        anc = ((r << 32) + c - 1) if c > 1 and rng.random() < 0.9 else rows[int(rng.integers(0, len(rows)))][0]
        rows.append(((r << 32) + c, anc))
        last[r] = c
    m = len(rows)
    v = dict(kind=np.zeros(m, np.uint8), ts=np.array([a for a, _ in rows], np.int64),
             path_off=np.arange(m + 1, dtype=np.uint32), path=np.array([b for _, b in rows] + [0], np.int64),
             val=np.arange(m, dtype=np.uint32))
    ot, rc, _ = oracle_apply_arrays(v, m)
    assert rc == 0
    et = CRDTree.init(0)
    res = et.apply_arrays(v, m)
    assert res.code == 0 and res.path_taken == N.PATH_CLOSED_FORM
    assert engine_summary(et) == oracle_summary(ot)
    assert np.array_equal(et.document_handles(), oracle_visible_vals(ot))


@pytest.mark.parametrize("log_min,spare", [("512", "0"), ("1", "0"), ("512", "2")])
def test_blocked_chain_order_forced(monkeypatch, log_min, spare):
    """Every dict through the blocked chain-order replay (pdr.hip pdr_blocked,
    normally only dicts of more than 4096 slots): the adversarial quirk streams
    (copies, orphans, orphan anchors re-entering the chain, trailing
    tombstones), config 1 and config 2 shapes, with and without change-log
    snapshots, against the oracle."""
    from adversarial import adversarial
    monkeypatch.setenv("CRDTM_PDR_BLK_MIN", "1")
    monkeypatch.setenv("CRDTM_PDR_LOG_MIN", log_min)
    monkeypatch.setenv("CRDTM_PDR_BLK_SPARE", spare)  # 2: compactions (repacking the chain) all the time
    paths = {}
    for seed in range(0, 128):
        n = [40, 120, 400, 1500][seed % 4]
        ops = adversarial(seed, n, replicas=2 + seed % 3, max_depth=1 + seed % 4)
        arrs = pack(ops)
        ot, rc, oerr = oracle_apply_arrays(arrs, n)
        et = CRDTree.init(0)
        res = et.apply_arrays(arrs, n)
        paths[res.path_taken] = paths.get(res.path_taken, 0) + 1
        assert res.code == rc, seed
        if rc != 0:
            assert res.err_index == oerr, seed
            continue
        assert engine_summary(et) == oracle_summary(ot), seed
        assert engine_log(et, 0) == oracle_log(ot, 0), seed
    assert paths.get(N.PATH_DICT_REPLAY, 0) > 32, paths
    for name in ("cfg1", "cfg2_small"):
        s, n = synth_case(**CASES[name])
        ot, rc, _ = oracle_apply_arrays(s, n)
        et = CRDTree.init(0)
        res = et.apply_arrays(s, n)
        assert res.code == rc == 0 and res.path_taken == N.PATH_DICT_REPLAY, name
        assert engine_summary(et) == oracle_summary(ot), name
        assert np.array_equal(et.document_handles(), oracle_visible_vals(ot)), name


def _nested_rows(shape, rng):
    """Add rows (ts, path) of a nested batch: path = the ancestors' keys, then
    the anchor key (0 = the dict's head)."""
    rows = []  # (ts, path)
    ctr = [0]

    def new_ts(rep=1):
        ctr[0] += 1
        return (rep << 32) + ctr[0]

    if shape == "single":
        a = new_ts()
        rows += [(a, [0]), (new_ts(), [a, 0])]
    elif shape == "chain":  # every node the only child of the one before: one leaf at the bottom
        anc = []
        for _ in range(40):
            t = new_ts()
            rows.append((t, anc + [0]))
            anc = anc + [t]
    elif shape == "star":  # one node with 300 leaf children, siblings anchored at random earlier ones
        r = new_ts()
        rows.append((r, [0]))
        kids = []
        for _ in range(300):
            t = new_ts(2 + int(rng.integers(0, 8)))
            a = kids[int(rng.integers(0, len(kids)))] if kids and rng.random() < 0.7 else 0
            rows.append((t, [r, a]))
            kids.append(t)
    else:  # "random": 3000 nodes up to depth 5, anchors among existing siblings
        nodes = [([], [])]  # (path to the dict, children keys of that dict)
        for _ in range(3000):
            k = int(rng.integers(0, len(nodes)))
            path, sib = nodes[k]
            if len(path) >= 5:
                continue
            t = new_ts(1 + int(rng.integers(0, 4)))
            a = sib[int(rng.integers(0, len(sib)))] if sib and rng.random() < 0.8 else 0
            rows.append((t, path + [a]))
            sib.append(t)
            nodes.append((path + [t], []))
    return rows


@pytest.mark.gpu
@pytest.mark.parametrize("shape", ["single", "chain", "star", "random"])
def test_nested_tour_shapes(shape):
    """The nested closed form's document order (Euler tour whose leaves have
    no leave entry: a chain with one leaf, a star of leaves, a single child,
    a random tree) against the oracle's literal replay."""
    rng = np.random.default_rng(0x70E5)
    rows = _nested_rows(shape, rng)
    m = len(rows)
    off = np.zeros(m + 1, np.uint32)
    off[1:] = np.cumsum([len(p) for _, p in rows])
    v = dict(kind=np.zeros(m, np.uint8), ts=np.array([t for t, _ in rows], np.int64), path_off=off,
             path=np.array([x for _, p in rows for x in p] + [0], np.int64), val=np.arange(m, dtype=np.uint32))
    ot, rc, _ = oracle_apply_arrays(v, m)
    assert rc == 0
    et = CRDTree.init(0)
    res = et.apply_arrays(v, m)
    assert res.code == 0
    assert engine_summary(et) == oracle_summary(ot)
    assert engine_log(et, 0) == oracle_log(ot, 0)
    assert np.array_equal(et.document_handles(), oracle_visible_vals(ot))
