"""Traversal API (CRDTree.get/parent/next/prev/walk, CRDTree.Node.children/head;
src/CRDTree.elm:421-625, src/CRDTree/Node.elm:96-174) served from the device
state, against the oracle's literal restatement — on trees with tombstones,
copy-quirk slots, orphans and implicit sentinels (tests/adversarial.py)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from crdtm.operation import flatten  # noqa: E402
from crdtm.tree import CRDTree, pack  # noqa: E402
from kat_cases import SCENARIOS  # noqa: E402
from parity_util import oracle_apply_arrays  # noqa: E402


def _oracle(handle):
    from oracle.oracle import OTree
    t = OTree(_h=handle)
    t.raw_values = True
    return t


def _key(v):
    return None if v is None else (v.kind, v.value, tuple(v.path), v.next)


def check_tree(et, ot, paths):
    import crdtm.tree as T
    orig = T.VALUES.value
    T.VALUES.value = lambda h: h
    try:
        assert [_key(v) for v in et.walk_nodes()] == ot.node_query("walk_start")
        assert [_key(v) for v in et.children(et.root())] == ot.node_query("children", [])
        for p in paths:
            v = et.get(p)
            assert _key(v) == ot.node(p), p
            if v is None:
                continue
            assert _key(et.parent(v)) == ot.node_query("parent", p), p
            assert _key(et.next(v)) == ot.node_query("next", p), p
            assert _key(et.prev(v)) == ot.node_query("prev", p), p
            assert [_key(c) for c in et.children(v)] == ot.node_query("children", p), p
            assert [_key(w) for w in et.walk_nodes(v)] == ot.node_query("walk", p), p
    finally:
        T.VALUES.value = orig


def query_paths(leaves, rng):
    paths = set()
    for o in leaves:
        if o.kind == "add":
            node = tuple(o.path[:-1]) + (o.ts,)
            paths.add(node)
            paths.add(node + (0,))            # its children's sentinel
            paths.add(tuple(o.path))          # its anchor
        else:
            paths.add(tuple(o.path))
    paths = sorted(paths)
    extra = [p + (int(rng.integers(1, 1 << 40)),) for p in paths[:20]] + [(0,), (12345,)]
    return [list(p) for p in paths + extra]


@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_traversal_scenarios(name):
    replica, calls = SCENARIOS[name]
    from oracle.oracle import lib as olib
    ot = olib().orc_init(replica)
    et = CRDTree.init(replica)
    leaves_all = []
    for op in calls:
        leaves = flatten(op) if op.kind == "batch" else [op]
        arrs = pack(leaves)
        oracle_apply_arrays(arrs, len(leaves), is_batch=op.kind == "batch", tree=ot)
        et.apply_arrays(arrs, len(leaves), is_batch=op.kind == "batch")
        leaves_all += leaves
    check_tree(et, _oracle(ot), query_paths(leaves_all, np.random.default_rng(1)))


@pytest.mark.parametrize("seed", range(0, 64, 4))
def test_traversal_adversarial(seed):
    from adversarial import adversarial
    n = [40, 120, 400, 1500][seed % 4]
    ops = adversarial(seed, n, replicas=2 + seed % 3, max_depth=1 + seed % 4)
    arrs = pack(ops)
    ot, rc, _ = oracle_apply_arrays(arrs, n)
    et = CRDTree.init(0)
    assert et.apply_arrays(arrs, n).code == rc
    if rc != 0:
        return
    paths = query_paths(ops, np.random.default_rng(seed))
    check_tree(et, _oracle(ot), paths[:400])


def test_traversal_device_queries_large_tree():
    """Point queries (get / parent / next / prev / children, all served by the
    device kernels over the per-version slot hash) on a 60k-op config-2-shaped
    tree (copy quirks, nested dicts), sampled nodes against the oracle."""
    import crdtm._native as N
    import crdtm.tree as T
    s = N.synth(n_ops=60000, replicas=16, window=64, p_delete=0.2, p_branch=0.1, max_depth=4, seed=0xC0FFEE02)
    n = len(s["kind"])
    ot, rc, _ = oracle_apply_arrays(s, n)
    et = CRDTree.init(0)
    assert et.apply_arrays(s, n).code == rc == 0
    o = _oracle(ot)
    rng = np.random.default_rng(5)
    off = s["path_off"]
    orig = T.VALUES.value
    T.VALUES.value = lambda h: h
    try:
        for i in rng.choice(n, 150, replace=False):
            p = [int(x) for x in s["path"][off[i]:off[i + 1]]]
            if s["kind"][i] == 0:
                p = p[:-1] + [int(s["ts"][i])]
            v = et.get(p)
            assert _key(v) == o.node(p), p
            if v is None:
                continue
            assert _key(et.parent(v)) == o.node_query("parent", p), p
            assert _key(et.next(v)) == o.node_query("next", p), p
            assert _key(et.prev(v)) == o.node_query("prev", p), p
            assert [_key(c) for c in et.children(v)] == o.node_query("children", p), p
        assert [_key(c) for c in et.children(et.root())] == o.node_query("children", [])
    finally:
        T.VALUES.value = orig


@pytest.mark.parametrize("poke", ["next_out_of_range", "next_cycle", "child_out_of_range", "sentinel_elsewhere",
                                  "dict_out_of_range"])
def test_host_readers_refuse_unsound_state(poke):
    """The host readers that follow the state's indices on a host copy
    (crdtm_tree_canonical, and crdtm_tree_walk = CRDTree.walk,
    src/CRDTree.elm:583-625) check it first: a corrupted device state
    (crdtm_debug_poke) is CRDTM_E_STATE (-7), never a wild read, and the
    readers recover once the state is sound again (a reset and a merge)."""
    import ctypes as C
    from crdtm import _native as N
    s = N.synth(n_ops=3000, replicas=4, window=16, p_delete=0.2, p_branch=0.1, max_depth=3, seed=3)
    n = len(s["kind"])
    et = CRDTree.init(0)
    assert et.apply_arrays(s, n).code == 0
    L = N.lib()
    cnt = C.c_uint64()
    assert L.crdtm_tree_walk(et._h, N.REF_NONE, None, 0, C.byref(cnt)) == 0 and cnt.value > 0
    field, index, value = {"next_out_of_range": (0, 5, 0x7FFFFFF0), "next_cycle": (0, 0, 0),
                           "child_out_of_range": (1, 3, 0x7FFFFFF0), "sentinel_elsewhere": (3, 0, 7),
                           "dict_out_of_range": (2, 9, 0x7FFFFFF0)}[poke]
    assert L.crdtm_debug_poke(et._h, field, index, value) == 0
    h = C.c_uint64()
    assert L.crdtm_tree_canonical(et._h, 0, None, 0, C.byref(cnt), C.byref(h)) == -7
    assert L.crdtm_tree_canonical(et._h, 1, None, 0, C.byref(cnt), C.byref(h)) == -7
    assert L.crdtm_tree_walk(et._h, N.REF_NONE, None, 0, C.byref(cnt)) == -7
    assert L.crdtm_debug_poke(et._h, 0, 1 << 40, 0) == -1  # (out of range: E_ARG)
    N.check(L.crdtm_tree_reset(et._h, 0))
    assert et.apply_arrays(s, n).code == 0
    ot, rc, _ = oracle_apply_arrays(s, n)
    from parity_util import engine_summary, oracle_summary
    assert engine_summary(et) == oracle_summary(ot)
    assert L.crdtm_tree_walk(et._h, N.REF_NONE, None, 0, C.byref(cnt)) == 0


def test_traversal_timestamp_boundaries():
    """The device queries over keys at the timestamp boundaries (the largest
    timestamp, a counter of 2^32 - 1, counter 0, a children dict under the
    largest key: tests/test_gpu_parity_gaps.py _boundary_ops) in a nested
    tree, against the oracle."""
    from oracle.oracle import lib as olib
    from test_gpu_parity_gaps import TS_MAX, _arrays, _boundary_ops, _nested_ops
    base = _nested_ops(2000, 61)
    extra = _boundary_ops(base)
    s = _arrays(base + extra)
    ot = olib().orc_init(0)
    _, rc, _ = oracle_apply_arrays(s, len(base) + len(extra), tree=ot)
    et = CRDTree.init(0)
    assert et.apply_arrays(s, len(base) + len(extra)).code == rc
    paths = [[TS_MAX], [TS_MAX, 0], [TS_MAX, (5 << 32) + 999_999], [TS_MAX, (5 << 32) + 1_000_000],
             [(3 << 32) + 0xFFFFFFFF], [77 << 32], [TS_MAX, TS_MAX], [0]]
    paths += [[k for k in o[2][:-1]] + [o[1]] for o in base[:200] if o[0] == 0]
    check_tree(et, _oracle(ot), paths)
