"""GPU parity of incremental merges: successive applies into a tree that
already holds state (src/CRDTree.elm:265-269 on a non-fresh tree — a replica
applying remote batches), chained against `orc_apply` on one oracle tree.

Every incremental path is pinned: the re-merge of log ++ batch on the
parallel fresh-tree paths (merge.hip apply_batch, CRDTM_FLAG_REMERGE), the
one-lane sequential replay on the existing state (CRDTM_INCREMENTAL=replay)
and the per-dict level replay on the state (ilr.hip, CRDTM_FLAG_DICT_INCR,
forced by CRDTM_INCREMENTAL=ilr; what it cannot decide falls back to the
re-merge).
Every step compares the dict structure, the visible document, timestamp,
replicas, lastOperation and the applied count; a failing batch in the middle
must leave everything unchanged (transactional, src/CRDTree.elm:224-232).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from crdtm import _native as N  # noqa: E402
from crdtm.tree import CRDTree  # noqa: E402
from parity_util import (engine_log, engine_summary, oracle_apply_arrays, oracle_log, oracle_summary,  # noqa: E402
                         oracle_visible_vals)

STREAMS = {
    # adds only, flat, 16 typing replicas: every re-merge is the flat closed form
    "flat_adds": dict(n_ops=60000, replicas=16, window=64, seed=31),
    # config-2 shape: interleaved deletes, branches -> per-dict replay / replay
    "nested_interleaved": dict(n_ops=30000, replicas=8, window=16, p_delete=0.2, p_branch=0.1, max_depth=3, seed=5),
    # config-2 shape itself (16 replicas, window 64, depth 4): busy dicts, long walks
    "config2_shape": dict(n_ops=60000, replicas=16, window=64, p_delete=0.2, p_branch=0.1, max_depth=4, seed=0xC0FFEE02),
    # config-4 shape: depth 12, deletes after adds -> nested closed form
    "deep_deletes_last": dict(n_ops=40000, replicas=16, p_delete=1 / 3, max_depth=12, max_children=8,
                              deletes_last=1, seed=9),
}


def sub(s, a, b):
    off = s["path_off"]
    return dict(kind=s["kind"][a:b].copy(), ts=s["ts"][a:b].copy(), val=s["val"][a:b].copy(),
                path_off=(off[a:b + 1] - off[a]).astype(np.uint32), path=s["path"][off[a]:off[b]].copy())


def failing_batch(s, a):
    """[the next op of the stream, an Add anchored at a key that does not exist]."""
    one = sub(s, a, a + 1)
    bad = dict(kind=np.zeros(1, np.uint8), ts=np.array([(63 << 32) + 7], np.int64), val=np.zeros(1, np.uint32),
               path_off=np.array([0, 1], np.uint32), path=np.array([(62 << 32) + 99991], np.int64))
    return dict(kind=np.concatenate([one["kind"], bad["kind"]]), ts=np.concatenate([one["ts"], bad["ts"]]),
                val=np.concatenate([one["val"], bad["val"]]),
                path_off=np.concatenate([one["path_off"], one["path_off"][-1] + bad["path_off"][1:]]).astype(np.uint32),
                path=np.concatenate([one["path"], bad["path"]]))


@pytest.mark.parametrize("mode", ["auto", "remerge", "replay", "ilr"])
@pytest.mark.parametrize("name", sorted(STREAMS))
def test_incremental_chain(name, mode, monkeypatch):
    if mode == "auto":  # the default: the incremental flat closed form where it applies
        monkeypatch.delenv("CRDTM_INCREMENTAL", raising=False)
    else:
        monkeypatch.setenv("CRDTM_INCREMENTAL", mode)
    s = N.synth(**STREAMS[name])
    n = len(s["kind"])
    rng = np.random.default_rng(len(name))
    # a large first batch, then batches of varied size (1 op .. a few thousand)
    cuts = [0, n // 2]
    while cuts[-1] < n:
        cuts.append(min(n, cuts[-1] + int(rng.choice([1, 7, 300, 2500, 6000]))))
    from oracle.oracle import lib as olib
    ot = olib().orc_init(0)
    et = CRDTree.init(0)
    remerged = incr = dict_incr = 0
    for k, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
        if k == 3:  # a failing batch in the middle: Err, nothing changes
            before = engine_summary(et)
            fb = failing_batch(s, a)
            _, rc, oerr = oracle_apply_arrays(fb, 2, tree=ot)
            st = np.full(2, 9, np.uint8)
            res = et.apply_arrays(fb, 2, status=st)
            assert (res.code, res.err_index) == (rc, oerr) == (3, 1)  # OperationFailed
            assert st[1] == 2  # CRDTM_ST_ERROR
            assert engine_summary(et) == before == oracle_summary(ot)
        chunk = sub(s, a, b)
        n_log0 = len(oracle_log(ot, 0)[0])
        _, rc, _ = oracle_apply_arrays(chunk, b - a, tree=ot)
        st = np.full(b - a, 9, np.uint8)
        res = et.apply_arrays(chunk, b - a, status=st)
        assert res.code == rc == 0, (k, res.code, rc)
        if k and mode == "remerge" and res.flags & N.FLAG_REMERGE:
            remerged += 1
        if k and mode == "replay":
            assert res.path_taken == N.PATH_REPLAY and not res.flags & N.FLAG_REMERGE
        if k and res.flags & N.FLAG_DICT_INCR:
            dict_incr += 1
            assert mode in ("auto", "ilr")
        if mode not in ("auto", "ilr"):
            assert not res.flags & N.FLAG_INCREMENTAL
        elif res.flags & N.FLAG_INCREMENTAL:
            incr += 1
        assert res.n_applied == len(oracle_log(ot, 0)[0]) - n_log0 == int(np.sum(st == 0)), k
        assert engine_summary(et) == oracle_summary(ot), (k, a, b)
        assert engine_log(et, 1) == oracle_log(ot, 1), k
    assert engine_log(et, 0) == oracle_log(ot, 0)
    assert np.array_equal(et.document_handles(), oracle_visible_vals(ot))
    if mode == "remerge" and name != "nested_interleaved":
        assert remerged == len(cuts) - 2  # every incremental step took the parallel paths
    if mode == "auto":
        # adds-only flat batches into a flat document: the incremental closed form
        assert (incr == len(cuts) - 2) if name == "flat_adds" else incr == 0
    if mode == "ilr" and name != "flat_adds":
        assert dict_incr >= (len(cuts) - 2) // 2, (dict_incr, len(cuts))
    olib().orc_free(ot)


@pytest.mark.parametrize("snapshot", ["1", "default"])
@pytest.mark.parametrize("seed", range(24))
def test_dict_incremental_adversarial(seed, snapshot, monkeypatch):
    """The per-dict level replay (ilr.hip) on the reference-test-shaped
    adversarial streams (copy quirks, nested copies, orphans, duplicates,
    deletes under deleted branches, errors): each stream applied as a base
    and then in chunks of varied size, every step against one oracle tree
    (structure, visible document, timestamp, replicas, log); batches it
    cannot decide fall back to the re-merge, failing ones leave the state
    unchanged."""
    monkeypatch.setenv("CRDTM_INCREMENTAL", "ilr")
    if snapshot == "1":  # every batch walks over the chain snapshot (by default only batches with a big group)
        monkeypatch.setenv("CRDTM_ILR_SNAPSHOT", "1")
    from adversarial import adversarial
    from crdtm.tree import pack
    from oracle.oracle import lib as olib
    s = pack(adversarial(seed, [600, 1500][seed % 2], replicas=2 + seed % 3, max_depth=1 + seed % 4))
    n = len(s["path_off"]) - 1
    rng = np.random.default_rng(seed)
    cuts = [0, max(1, n // 3)]
    while cuts[-1] < n:
        cuts.append(min(n, cuts[-1] + int(rng.choice([1, 3, 17, 60, 200]))))
    ot = olib().orc_init(0)
    et = CRDTree.init(0)
    used = 0
    for a, b in zip(cuts[:-1], cuts[1:]):
        chunk = sub(s, a, b)
        _, rc, oerr = oracle_apply_arrays(chunk, b - a, tree=ot)
        res = et.apply_arrays(chunk, b - a)
        assert (res.code, res.err_index if rc else -1) == (rc, oerr if rc else -1), (a, b)
        used += bool(res.flags & N.FLAG_DICT_INCR)  # (quirk-heavy chunks may all fall back)
        assert engine_summary(et) == oracle_summary(ot), (a, b)
    assert engine_log(et, 0) == oracle_log(ot, 0)
    assert np.array_equal(et.document_handles(), oracle_visible_vals(ot))
    olib().orc_free(ot)


# flat typing streams for the incremental closed form (incr.hip): many
# replicas typing at once (new runs landing in the same gaps, new anchors in
# other gaps, non-Lamport anchors), few replicas with long lags, and the
# sentinel as anchor
FINC_STREAMS = {
    "r64_w256": dict(n_ops=120000, replicas=64, window=256, seed=41),
    "r4_w2000": dict(n_ops=60000, replicas=4, window=2000, seed=42),
    "r16_w16": dict(n_ops=60000, replicas=16, window=16, seed=43),
    "r2_w1": dict(n_ops=30000, replicas=2, window=1, seed=44),
    # one cursor typing on: every batch lands in one gap at the document's
    # end (rebalance windows over the last blocks, a gap too large for any
    # window: the dense merge)
    "r1_cursor": dict(n_ops=60000, replicas=1, window=1, p_continue=1.0, seed=45),
    # three cursors that rarely jump: a few hot gaps per batch
    "r3_hot": dict(n_ops=60000, replicas=3, window=4, p_continue=0.995, seed=46),
}


@pytest.mark.parametrize("name", sorted(FINC_STREAMS))
def test_incremental_flat_closed_form(name, monkeypatch):
    """Adds-only flat batches merged into a flat document in place
    (CRDTM_FLAG_INCREMENTAL): batches of 1 .. 16,000 ops chained against the
    oracle tree (structure, visible order, log, lastOperation, replicas,
    timestamp); then one Delete, after which the document is no longer clean
    and later batches take the general paths."""
    monkeypatch.delenv("CRDTM_INCREMENTAL", raising=False)
    from oracle.oracle import lib as olib
    s = N.synth(**FINC_STREAMS[name])
    n = len(s["kind"])
    rng = np.random.default_rng(7)
    cuts = [0, n // 5]
    while cuts[-1] < n:
        cuts.append(min(n, cuts[-1] + int(rng.choice([1, 2, 64, 1000, 5000, 16000]))))
    ot = olib().orc_init(0)
    et = CRDTree.init(0)
    used = windows = dense = tour = 0
    for k, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
        chunk = sub(s, a, b)
        _, rc, _ = oracle_apply_arrays(chunk, b - a, tree=ot)
        res = et.apply_arrays(chunk, b - a)
        assert res.code == rc == 0, (k, res.code, rc)
        used += bool(res.flags & N.FLAG_INCREMENTAL)
        windows += bool(res.flags & N.FLAG_INCR_WINDOWS)
        dense += bool(res.flags & N.FLAG_INCR_DENSE)
        tour += bool(res.flags & N.FLAG_INCR_TOUR)
        if k % 7 == 0 or b == n:
            assert engine_summary(et) == oracle_summary(ot), (k, a, b)
            assert engine_log(et, 1) == oracle_log(ot, 1), k
        if k % 5 == 2:  # the order is kept gapped between batches: read it back mid-chain
            assert np.array_equal(et.document_handles(), oracle_visible_vals(ot)), k
        if k == 3:  # a version taken from a gapped order sees the same document
            v = et.clone()
            assert np.array_equal(v.document_handles(), oracle_visible_vals(ot))
            del v
    assert used == len(cuts) - 2
    if name == "r1_cursor":  # one hot gap: the windows and the dense merge both ran
        assert windows and dense, (windows, dense)
    if name in ("r2_w1", "r3_hot"):  # (typing runs: gaps in key order, ordered by their tree's DFS)
        assert tour, name
    assert engine_log(et, 0) == oracle_log(ot, 0)
    assert np.array_equal(et.document_handles(), oracle_visible_vals(ot))
    # a Delete makes the document unclean: no incremental closed form afterwards
    key = int(s["ts"][n // 3])
    dl = dict(kind=np.ones(1, np.uint8), ts=np.zeros(1, np.int64), val=np.zeros(1, np.uint32),
              path_off=np.array([0, 1], np.uint32), path=np.array([key], np.int64))
    _, rc, _ = oracle_apply_arrays(dl, 1, tree=ot)
    res = et.apply_arrays(dl, 1)
    assert res.code == rc == 0 and not res.flags & N.FLAG_INCREMENTAL
    more = N.synth(**dict(FINC_STREAMS[name], n_ops=n + 3000))
    chunk = sub(more, n, n + 3000)
    _, rc, _ = oracle_apply_arrays(chunk, 3000, tree=ot)
    res = et.apply_arrays(chunk, 3000)
    assert res.code == rc and not res.flags & N.FLAG_INCREMENTAL
    assert engine_summary(et) == oracle_summary(ot)
    olib().orc_free(ot)


def test_versions_copy_on_write():
    """Persistent versions (src/CRDTree.elm:228-232: `apply` returns a new
    tree and the old one stays valid): crdtm_tree_clone shares the device
    state, the first write to either handle copies it."""
    import gc
    from oracle.oracle import lib as olib
    s = N.synth(n_ops=20000, replicas=8, window=16, p_delete=0.2, p_branch=0.1, max_depth=3, seed=77)

    def oracle_upto(m):
        ot, rc, _ = oracle_apply_arrays(sub(s, 0, 10000), 10000)
        if m > 10000:
            _, rc2, _ = oracle_apply_arrays(sub(s, 10000, m), m - 10000, tree=ot)
            assert rc2 == 0
        return ot

    v0 = CRDTree.init(0)
    assert v0.apply_arrays(sub(s, 0, 10000), 10000).code == 0
    sum0, log0, doc0 = engine_summary(v0), engine_log(v0, 0), v0.document_handles()
    v1 = v0.clone()
    assert v1.apply_arrays(sub(s, 10000, 20000), 10000).code == 0
    v2 = v0.clone()
    assert v2.apply_arrays(sub(s, 10000, 15000), 5000).code == 0
    assert engine_summary(v0) == sum0 and engine_log(v0, 0) == log0
    assert np.array_equal(v0.document_handles(), doc0)
    o20, o15 = oracle_upto(20000), oracle_upto(15000)
    assert engine_summary(v1) == oracle_summary(o20)
    assert engine_summary(v2) == oracle_summary(o15)
    del v0
    gc.collect()
    assert engine_summary(v1) == oracle_summary(o20) and engine_log(v1, 0) == oracle_log(o20, 0)
    v3 = v1.clone()
    N.check(N.lib().crdtm_tree_reset(v3._h, 0))
    assert engine_summary(v1) == oracle_summary(o20)
    assert np.array_equal(v1.document_handles(), oracle_visible_vals(o20))
    assert v3.apply_arrays(sub(s, 0, 10000), 10000).code == 0
    assert engine_summary(v3) == oracle_summary(oracle_upto(10000))
    for t in (o20, o15):
        olib().orc_free(t)


@pytest.mark.parametrize("mode", ["auto", "ilr"])
def test_failed_fresh_batch_then_flat_op(mode, monkeypatch):
    """A fresh batch that fails after the nested merge handed it to the
    replay (which resets the device result block) must leave the context's
    replica range table clean: the next batch, one flat Add anchored at a key
    of that failed batch from another replica, is NotFound (adversarial seed
    14: ops [0, 200) fail at 192, op 200 anchors at op 185's key)."""
    monkeypatch.setenv("CRDTM_INCREMENTAL", mode)
    from adversarial import adversarial
    from crdtm.tree import pack
    from oracle.oracle import lib as olib
    s = pack(adversarial(14, 600, replicas=4, max_depth=3))
    ot = olib().orc_init(0)
    et = CRDTree.init(0)
    for a, b in ((0, 200), (200, 201), (201, 260)):
        _, rc, oerr = oracle_apply_arrays(sub(s, a, b), b - a, tree=ot)
        res = et.apply_arrays(sub(s, a, b), b - a)
        assert (res.code, res.err_index if rc else -1) == (rc, oerr if rc else -1), (a, b)
        assert engine_summary(et) == oracle_summary(ot), (a, b)
    olib().orc_free(ot)


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("n", [1000, 4000, 16000])
def test_level_replay_small_config2(n, seed, monkeypatch):
    """Small config-2-shaped streams (16 replicas typing into nested dicts
    with Deletes): half as a base, then chunks of varied size through the
    level replay, every chunk against one oracle tree. Their copy quirks make
    deferred copies whose source and destination dicts fall in one group
    (the lane copies, then lands its later ops in the copy)."""
    monkeypatch.setenv("CRDTM_INCREMENTAL", "ilr")
    from oracle.oracle import lib as olib
    s = N.synth(**dict(STREAMS["config2_shape"], n_ops=n, seed=seed))
    rng = np.random.default_rng(seed)
    cuts = [0, n // 2]
    while cuts[-1] < n:
        cuts.append(min(n, cuts[-1] + int(rng.choice([1, 7, 300, n // 8]))))
    ot = olib().orc_init(0)
    et = CRDTree.init(0)
    for k, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
        chunk = sub(s, a, b)
        _, rc, _ = oracle_apply_arrays(chunk, b - a, tree=ot)
        res = et.apply_arrays(chunk, b - a)
        assert res.code == rc == 0, (k, res.code, rc)
        assert engine_summary(et) == oracle_summary(ot), (k, a, b, res.flags)
    assert engine_log(et, 0) == oracle_log(ot, 0)
    olib().orc_free(ot)


SHAPES = [  # (replicas, window, p_delete, p_branch, max_depth, seed, chunking seed); the first re-fills
    # a slot whose children are a deferred copy still to run (its copy must not be taken in the batch)
    (16, 256, 0.4, 0.3, 3, 903783157, 14),
    (32, 64, 0.2, 0.3, 6, 11, 11), (8, 16, 0.4, 0.1, 8, 12, 12), (2, 4, 0.05, 0.3, 4, 13, 13),
    (16, 64, 0.4, 0.05, 2, 14, 14), (4, 256, 0.2, 0.1, 6, 15, 15),
]


@pytest.mark.parametrize("shape", SHAPES)
def test_level_replay_shapes(shape, monkeypatch):
    """Level replay chains over stream shapes beyond config 2 (depth 2-8,
    heavy branching and deleting), every chunk against the oracle."""
    monkeypatch.setenv("CRDTM_INCREMENTAL", "ilr")
    from oracle.oracle import lib as olib
    r, w, pd, pb, md, seed, cseed = shape
    s = N.synth(n_ops=6000, replicas=r, window=w, p_delete=pd, p_branch=pb, max_depth=md, seed=seed)
    n = len(s["kind"])
    rng = np.random.default_rng(cseed)
    cuts = [0, n // 2]
    while cuts[-1] < n:
        cuts.append(min(n, cuts[-1] + int(rng.choice([1, 7, 300, n // 8, n // 4]))))
    ot = olib().orc_init(0)
    et = CRDTree.init(0)
    for k, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
        chunk = sub(s, a, b)
        _, rc, _ = oracle_apply_arrays(chunk, b - a, tree=ot)
        res = et.apply_arrays(chunk, b - a)
        assert res.code == rc, (k, res.code, rc)
        assert engine_summary(et) == oracle_summary(ot), (k, a, b, res.flags)
    olib().orc_free(ot)


def test_level_replay_config2_shape(monkeypatch):
    """The level replay at the shape of `bench.py --workload incr_cfg2` (a
    config-2 document, nested typing with interleaved Deletes from 16
    replicas), scaled down: a 200k-op base, then five 10k-op batches. Every
    batch takes the level replay or, where its lanes cannot decide, the
    re-merge (its busy dicts walk over the chain snapshot), and must match the oracle after each batch (structure, document,
    timestamp, replicas), with the log checked at the end."""
    monkeypatch.delenv("CRDTM_INCREMENTAL", raising=False)
    monkeypatch.delenv("CRDTM_ILR_SNAPSHOT", raising=False)
    from oracle.oracle import lib as olib
    base, bsz, nb = 200_000, 10_000, 5
    s = N.synth(n_ops=base + bsz * nb, replicas=16, window=64, p_delete=0.2, p_branch=0.1, max_depth=4,
                seed=0xC0FFEE02)
    ot = olib().orc_init(0)
    et = CRDTree.init(0)
    cuts = [0, base] + [base + bsz * (j + 1) for j in range(nb)]
    dict_incr = 0
    for k, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
        chunk = sub(s, a, b)
        _, rc, _ = oracle_apply_arrays(chunk, b - a, tree=ot)
        res = et.apply_arrays(chunk, b - a)
        assert res.code == rc == 0, (k, res.code, rc)
        if k and res.flags & N.FLAG_DICT_INCR:
            assert res.path_taken == N.PATH_DICT_REPLAY
            dict_incr += 1
        assert engine_summary(et) == oracle_summary(ot), k
    # at most one batch of this smaller base falls back to the re-merge: its
    # fourth batch holds a copy quirk whose deferred copy would be needed two
    # levels down (IW_COPY_BELOW, an undecidable case of DESIGN.md §e); at the
    # bench's own shape no batch does (test_level_replay_incr_cfg2_bench_shape)
    assert dict_incr >= nb - 1, dict_incr
    assert np.array_equal(et.document_handles(), oracle_visible_vals(ot))
    assert engine_log(et, 0) == oracle_log(ot, 0)
    olib().orc_free(ot)


def _statuses_match_last_operation(st, chunk, m, ot):
    """Per-op statuses against the oracle: the ops with status Applied are
    exactly lastOperation (src/CRDTree.elm:298-325, :328-334), in order."""
    applied = np.nonzero(st[:m] == 0)[0]
    want, _ = oracle_log(ot, 1)
    off = chunk["path_off"]
    got = [(int(chunk["kind"][i]), int(chunk["ts"][i]) if chunk["kind"][i] == 0 else 0,
            tuple(int(x) for x in chunk["path"][off[i]:off[i + 1]]), int(chunk["val"][i]) if chunk["kind"][i] == 0 else 0)
           for i in applied]
    return got == want


def test_level_replay_incr_cfg2_bench_shape(monkeypatch):
    """`bench.py --workload incr_cfg2` at its own shape (INCR_CFG2: a 900k-op
    config-2 document, seed 0xC0FFEE02, then ten 10k-op batches), every batch
    against orc_apply on one oracle tree (src/CRDTree.elm:265-269): the dict
    structure, the visible document, timestamp, replicas, lastOperation and
    every op's status; each batch must be served by the level replay itself."""
    monkeypatch.delenv("CRDTM_INCREMENTAL", raising=False)
    monkeypatch.delenv("CRDTM_ILR_SNAPSHOT", raising=False)
    from oracle.oracle import lib as olib
    base, bsz, nb = 900_000, 10_000, 10
    s = N.synth(n_ops=base + bsz * nb, replicas=16, window=64, p_delete=0.2, p_branch=0.1, max_depth=4,
                seed=0xC0FFEE02)
    ot = olib().orc_init(0)
    et = CRDTree.init(0)
    first = sub(s, 0, base)
    _, rc, _ = oracle_apply_arrays(first, base, tree=ot)
    assert et.apply_arrays(first, base).code == rc == 0
    assert engine_summary(et) == oracle_summary(ot)
    for j in range(nb):
        a, b = base + j * bsz, base + (j + 1) * bsz
        chunk = sub(s, a, b)
        _, rc, _ = oracle_apply_arrays(chunk, bsz, tree=ot)
        st = np.full(bsz, 9, np.uint8)
        res = et.apply_arrays(chunk, bsz, status=st)
        assert res.code == rc == 0, (j, res.code, rc)
        assert res.flags & N.FLAG_DICT_INCR and res.path_taken == N.PATH_DICT_REPLAY, (j, res.flags)
        assert engine_summary(et) == oracle_summary(ot), j
        assert engine_log(et, 1) == oracle_log(ot, 1), j
        assert _statuses_match_last_operation(st, chunk, bsz, ot), j
        assert res.n_applied == int(np.sum(st == 0)), j
    assert np.array_equal(et.document_handles(), oracle_visible_vals(ot))
    assert engine_log(et, 0) == oracle_log(ot, 0)
    olib().orc_free(ot)


def _sweep_shapes(cases=40, rseed=1234):
    """Stream shapes drawn once with a fixed seed: 2-32 replicas, window 4-256,
    depth 2-8, branching and deleting up to 0.3 / 0.4."""
    rng = np.random.default_rng(rseed)
    out = []
    for _ in range(cases):
        out.append(dict(n_ops=6000, replicas=int(rng.choice([2, 4, 8, 16, 32])),
                        window=int(rng.choice([4, 16, 64, 256])), p_delete=float(rng.choice([0.05, 0.2, 0.4])),
                        p_branch=float(rng.choice([0.05, 0.1, 0.3])), max_depth=int(rng.choice([2, 3, 4, 6, 8])),
                        seed=int(rng.integers(1 << 30))))
    return out


@pytest.mark.parametrize("case", range(40))
def test_level_replay_sweep(case, monkeypatch):
    """The level replay forced over 40 fixed stream shapes (the sweep that
    found round 4's pending-copy bug), each chained against the oracle in
    chunks of 1 .. n/4 ops."""
    monkeypatch.setenv("CRDTM_INCREMENTAL", "ilr")
    from oracle.oracle import lib as olib
    cfg = _sweep_shapes()[case]
    s = N.synth(**cfg)
    n = len(s["kind"])
    rng = np.random.default_rng(case)
    cuts = [0, n // 2]
    while cuts[-1] < n:
        cuts.append(min(n, cuts[-1] + int(rng.choice([1, 7, 300, n // 8, n // 4]))))
    ot = olib().orc_init(0)
    et = CRDTree.init(0)
    for k, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
        chunk = sub(s, a, b)
        _, rc, _ = oracle_apply_arrays(chunk, b - a, tree=ot)
        res = et.apply_arrays(chunk, b - a)
        assert res.code == rc, (cfg, k, res.code, rc)
        assert engine_summary(et) == oracle_summary(ot), (cfg, k, a, b, res.flags)
    assert engine_log(et, 0) == oracle_log(ot, 0)
    olib().orc_free(ot)


def test_level_replay_commit_failure_rolls_back(monkeypatch):
    """A level replay whose commit fails after the levels changed the state in
    place (CRDTM_ILR_FAIL_COMMIT: an arena overflow injected at the commit's
    first scan) rolls the levels back; crdtm_apply then retries with a larger
    arena on the restored state, and the result matches the oracle."""
    monkeypatch.delenv("CRDTM_INCREMENTAL", raising=False)
    from oracle.oracle import lib as olib
    s = N.synth(n_ops=80_000, replicas=16, window=64, p_delete=0.2, p_branch=0.1, max_depth=4, seed=0xC0FFEE02)
    ot = olib().orc_init(0)
    et = CRDTree.init(0)
    cuts = [0, 60_000, 65_000, 70_000, 80_000]
    for k, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
        chunk = sub(s, a, b)
        _, rc, _ = oracle_apply_arrays(chunk, b - a, tree=ot)
        if k in (1, 3):
            monkeypatch.setenv("CRDTM_ILR_FAIL_COMMIT", f"fail{k}")
        res = et.apply_arrays(chunk, b - a)
        monkeypatch.delenv("CRDTM_ILR_FAIL_COMMIT", raising=False)
        assert res.code == rc == 0, (k, res.code)
        if k:
            assert res.flags & N.FLAG_DICT_INCR, (k, res.flags)
        assert engine_summary(et) == oracle_summary(ot), k
        assert engine_log(et, 1) == oracle_log(ot, 1), k
    assert engine_log(et, 0) == oracle_log(ot, 0)
    olib().orc_free(ot)
