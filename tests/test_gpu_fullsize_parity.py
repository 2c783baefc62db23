"""Full-size parity at BASELINE.json's configurations, against the C++ oracle
(oracle/crdtree_oracle.cpp, the line-by-line restatement of
src/CRDTree.elm:224-350 and src/Internal/Node.elm:51-163).

* config 2: one tree, 1M ops (80/20 interleaved, 16 replicas, branches, depth
  <= 4) — the interleaved-delete path;
* config 4: the deep tree at 10M ops (depth <= 12, <= 8 children, half the
  nodes deleted after the adds);
* config 5: all 12,500 documents of one GPU's share, through the op-log
  records of 8 simulated replicas (crdtm/shard.py local_log), the native
  record assembly of every one of 8 ranks (crdtm_shard_assemble) and
  crdtm_forest_apply;
* a nested adds-only batch large enough for many scan tiles (the closed
  form's "every op applied" log shortcut), its log and operationsSince.

Compared bit for bit: canonical structure digest (every dict entry incl.
tombstones, sentinels, copy-quirk slots), visible-order digest, timestamp,
replicas table, the operation log and lastOperation, the device document
order.
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from crdtm import _native as N  # noqa: E402
from crdtm.tree import CRDTree  # noqa: E402
from oracle.oracle import _ptr, lib as olib  # noqa: E402
from parity_util import engine_summary, oracle_apply_arrays, oracle_summary, oracle_visible_vals  # noqa: E402

CFG2 = dict(n_ops=1_000_000, replicas=16, window=64, p_delete=0.2, p_branch=0.1, max_depth=4, seed=0xC0FFEE02)
CFG4 = dict(n_ops=10_000_000, replicas=16, p_delete=1 / 3, max_depth=12, max_children=8, deletes_last=1,
            seed=0xC0FFEE04)
TREES = dict(per_doc=1000, n_docs=12_500, replicas=8, window=16, p_delete=0.2, seed=0xC0FFEE05)


def oracle_log_np(t, which):
    L = olib()
    pt = C.c_uint64(0)
    isb = C.c_int(0)
    n = L.orc_ops(t, which, None, None, None, None, None, C.byref(pt), C.byref(isb))
    a = dict(kind=np.zeros(n + 1, np.uint8), ts=np.zeros(n + 1, np.int64), off=np.zeros(n + 1, np.uint32),
             path=np.zeros(pt.value + 1, np.int64), val=np.zeros(n + 1, np.uint32))
    L.orc_ops(t, which, _ptr(a["kind"]), _ptr(a["ts"]), _ptr(a["off"]), _ptr(a["path"]), _ptr(a["val"]), None, None)
    return n, a, bool(isb.value)


def engine_log_np(tree, which, since=None):
    from crdtm.tree import _ptr as eptr
    o = N.Ops()
    isb = C.c_int(1)

    def fetch(ops):
        if since is None:
            N.check(N.lib().crdtm_tree_ops(tree._h, which, C.byref(ops), C.byref(isb)))
        else:
            N.check(N.lib().crdtm_tree_ops_since(tree._h, since, C.byref(ops)))

    fetch(o)
    n, npth = o.n_ops, o.n_path
    a = dict(kind=np.zeros(n + 1, np.uint8), ts=np.zeros(n + 1, np.int64), off=np.zeros(n + 1, np.uint32),
             path=np.zeros(npth + 1, np.int64), val=np.zeros(n + 1, np.uint32))
    fetch(N.Ops(n, npth, eptr(a["kind"]), eptr(a["ts"]), eptr(a["off"]), eptr(a["path"]), eptr(a["val"]), None))
    return n, a, bool(isb.value)


def assert_logs_equal(et, ot):
    for which in (0, 1):
        en, ea, eb = engine_log_np(et, which)
        on, oa, ob = oracle_log_np(ot, which)
        assert (en, eb) == (on, ob), which
        for k in ("kind", "ts", "off", "val"):
            assert np.array_equal(ea[k][:en + (k == "off")], oa[k][:on + (k == "off")]), (which, k)
        assert np.array_equal(ea["path"][:ea["off"][en]], oa["path"][:oa["off"][on]]), which


def full_parity(spec, want_path=None):
    s = N.synth(**spec)
    n = len(s["kind"])
    ot, rc, _ = oracle_apply_arrays(s, n)
    assert rc == 0
    et = CRDTree.init(0)
    res = et.apply_arrays(s, n)
    assert res.code == 0, (res.code, res.err_index)
    if want_path is not None:
        assert res.path_taken in want_path, (res.path_taken, res.guard)
    n_logged = oracle_log_np(ot, 0)[0]
    assert (res.n_applied, res.n_already) == (n_logged, n - n_logged)
    assert engine_summary(et) == oracle_summary(ot)
    assert_logs_equal(et, ot)
    assert np.array_equal(et.document_handles(), oracle_visible_vals(ot))
    return s, et, ot, res


def test_cfg2_1m_interleaved():
    """BASELINE config 2 at its full 1M ops (guard G fails: Deletes before
    later Adds in the same dicts; the exact GPU paths)."""
    _, et, ot, res = full_parity(CFG2)
    assert res.path_taken != N.PATH_CLOSED_FORM, "config 2 interleaves deletes: the guard must fail somewhere"
    olib().orc_free(ot)


def test_deep10m():
    """BASELINE config 4 at its full 10M ops: closed form with tombstones."""
    _, et, ot, res = full_parity(CFG4, want_path=(N.PATH_CLOSED_FORM,))
    olib().orc_free(ot)


def test_deep10m_interleaved():
    """Config 4's second variant at its full 10M ops: the same
    deep tree shape with its Deletes interleaved among the Adds (live leaves,
    synth.cpp genDeep), so dicts hold tombstones before later inserts — the
    regime of src/Internal/Node.elm:93-122 — through the exact per-dict replay
    (bench workload deep10m_il)."""
    spec = dict(CFG4, deletes_last=0)
    _, et, ot, res = full_parity(spec)
    assert res.path_taken != N.PATH_CLOSED_FORM and res.guard & 2, (res.path_taken, res.guard)
    olib().orc_free(ot)


def test_incremental_flat_1m(monkeypatch):
    """The bench's incremental workload shape at scale: a 1M-node flat
    document (config 3's stream, closed form), then successive 10k-op batches
    of the same stream merged in place (CRDTM_FLAG_INCREMENTAL); the final
    structure and visible digests against the fast flat restatement
    (`orc_flat_replay`, pinned against the general one) over the whole
    stream, and the device document order against the host walk."""
    import ctypes as C
    monkeypatch.delenv("CRDTM_INCREMENTAL", raising=False)
    base, bsz, nb = 1_000_000, 10_000, 4
    n = base + bsz * nb
    s = N.synth(n_ops=n, replicas=64, window=256, seed=0xC0FFEE03)
    off = s["path_off"]

    def sub(a, b):
        return dict(kind=s["kind"][a:b], ts=s["ts"][a:b], val=s["val"][a:b],
                    path_off=(off[a:b + 1] - off[a]).astype(np.uint32), path=s["path"][off[a]:off[b]])

    et = CRDTree.init(0)
    assert et.apply_arrays(sub(0, base), base).code == 0
    for k in range(nb):
        a = base + k * bsz
        res = et.apply_arrays(sub(a, a + bsz), bsz)
        assert res.code == 0 and res.flags & N.FLAG_INCREMENTAL, (k, res.code, res.flags)
        assert res.n_applied == bsz
    h = np.zeros(2, np.uint64)
    w = np.zeros(2, np.uint64)
    err = C.c_int64(-1)
    na = C.c_uint64()
    rc = olib().orc_flat_replay(n, _ptr(s["kind"]), _ptr(s["ts"]), _ptr(s["path_off"]), _ptr(s["path"]),
                                _ptr(s["val"]), C.byref(err), _ptr(h), _ptr(w), C.byref(na))
    assert rc == 0 and na.value == n
    for which in (0, 1):
        _, enw, eh = et.canonical(which, full=False)
        assert (enw, eh) == (int(w[which]), int(h[which])), which
    words, nw, _ = et.canonical(1, full=True)
    assert np.array_equal(et.document_handles().astype(np.int64), words[1::4])
    en, ea, _ = engine_log_np(et, 0)  # the log: every op, in order
    assert en == n and np.array_equal(ea["ts"][:n], s["ts"]) and np.array_equal(ea["path"][:n], s["path"])


def test_forced_sequential_replay(monkeypatch):
    """CRDTM_FORCE_REPLAY=1 sends a batch the parallel paths serve to the
    one-lane sequential replay (how bench.py --force-replay measures that
    fallback); its result must be the same."""
    monkeypatch.setenv("CRDTM_FORCE_REPLAY", "1")
    spec = dict(CFG2, n_ops=200_000)
    _, et, ot, res = full_parity(spec, want_path=(N.PATH_REPLAY,))
    assert res.guard & 32
    olib().orc_free(ot)


def test_nested_adds_every_applied_2m():
    """A nested adds-only batch (every op applies: the log is the batch, no
    log scans) over many scan tiles; log, lastOperation and operationsSince
    against the oracle (src/Internal/Operation.elm:25-53)."""
    s, et, ot, res = full_parity(dict(n_ops=2_000_000, replicas=8, window=16, p_branch=0.2, max_depth=6, seed=11),
                                 want_path=(N.PATH_CLOSED_FORM,))
    assert res.n_applied == len(s["kind"])
    on, oa, _ = oracle_log_np(ot, 0)
    rng = np.random.default_rng(17)
    adds = s["ts"][s["kind"] == 0]
    for want in list(rng.choice(adds, 6)) + [int(adds[-1]), 0, 12345]:
        want = int(want)
        en, ea, _ = engine_log_np(et, 0, since=want)
        if want == 0:
            j = 0
        else:
            hit = np.nonzero((oa["kind"][:on] == 0) & (oa["ts"][:on] == want))[0]
            j = int(hit[-1]) if len(hit) else on
        assert en == on - j, want
        assert np.array_equal(ea["ts"][:en], oa["ts"][j:on]), want
        assert np.array_equal(ea["path"][:ea["off"][en]], oa["path"][oa["off"][j]:oa["off"][on]]), want
    olib().orc_free(ot)


def test_trees_12500_documents_sharded():
    """BASELINE config 5: 12,500 documents x 1,000 ops. The 8 simulated
    replicas' op logs (records, as the RCCL all-gather delivers them) are
    assembled natively for each of 8 ranks and every owned document is merged
    by crdtm_forest_apply; every document is checked against the oracle."""
    import torch
    from crdtm import shard
    from crdtm.tree import forest_apply
    per, n_docs, world = TREES["per_doc"], TREES["n_docs"], 8
    parts, recs = [], [[] for _ in range(world)]
    for d0 in range(0, n_docs, 2000):  # the chunking bench.py uses (same streams)
        nd = min(2000, n_docs - d0)
        s = N.synth(n_ops=per, n_docs=nd, replicas=TREES["replicas"], window=TREES["window"],
                    p_delete=TREES["p_delete"], seed=TREES["seed"], doc_base=d0)
        parts.append(s)
        doc_off = np.arange(nd + 1, dtype=np.uint32) * per
        for k in range(world):
            r = shard.local_log(s, doc_off, k, world, TREES["replicas"])
            r[:, 0] += np.int64(d0) << 32
            recs[k].append(r)
    full = {k: np.concatenate([p[k] for p in parts]) for k in ("kind", "ts", "val")}
    full["path"] = np.concatenate([p["path"] for p in parts])
    assert len(full["path"]) == n_docs * per  # flat documents: one path element per op
    full["path_off"] = np.arange(n_docs * per + 1, dtype=np.uint32)
    doc_all = np.arange(n_docs + 1, dtype=np.uint32) * per
    L = olib()
    want = dict(code=np.zeros(n_docs, np.int32), err=np.zeros(n_docs, np.int64), hash=np.zeros(n_docs, np.uint64),
                words=np.zeros(n_docs, np.uint64), timestamp=np.zeros(n_docs, np.int64))
    L.orc_forest_apply(n_docs, _ptr(doc_all), 0, _ptr(full["kind"]), _ptr(full["ts"]), _ptr(full["path_off"]),
                       _ptr(full["path"]), _ptr(full["val"]), _ptr(want["code"]), _ptr(want["err"]),
                       _ptr(want["hash"]), _ptr(want["words"]), _ptr(want["timestamp"]))
    dev = torch.device("cuda", 0)
    records = torch.from_numpy(np.concatenate([np.concatenate(r) for r in recs])).to(dev)
    assert records.shape[0] == n_docs * per
    ctx = C.c_void_p()
    N.check(N.lib().crdtm_ctx_create(0, C.c_void_p(torch.cuda.current_stream().cuda_stream), C.byref(ctx)))
    checked = 0
    for rank in range(world):
        ops_t, doc_off, _ = shard.assemble(records, rank, world, n_docs, per, ctx=ctx)
        torch.cuda.synchronize()
        n = int(doc_off[-1])
        ops = N.Ops(n, n, ops_t["kind"].data_ptr(), ops_t["ts"].data_ptr(), ops_t["path_off"].data_ptr(),
                    ops_t["path"].data_ptr(), ops_t["val"].data_ptr(), None)
        out = forest_apply(ops, doc_off, on_device=True)
        assert out["rc"] == 0
        mine = np.arange(rank, n_docs, world)
        assert len(mine) == len(doc_off) - 1
        assert np.array_equal(out["code"], want["code"][mine]), rank
        ok = want["code"][mine] == 0
        assert np.array_equal(out["err"][~ok], want["err"][mine][~ok]), rank
        assert np.array_equal(out["hash"], want["hash"][mine]), rank
        assert np.array_equal(out["words"], want["words"][mine]), rank
        assert np.array_equal(out["timestamp"][ok], want["timestamp"][mine][ok]), rank
        checked += len(mine)
    N.lib().crdtm_ctx_destroy(ctx)
    assert checked == n_docs
