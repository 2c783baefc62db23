"""Pin the CPU oracle against the reference's own known answers.

Transcribes tests/CRDTreeTest.elm (65 cases), tests/NodeTest.elm (15) and the
round-trip intent of tests/JsonTest.elm (see test_json_codec.py), plus the
hand-traced vectors of SURVEY.md Appendix C. CPU only.
"""
import pytest

from crdtm.operation import Add, Batch, Delete
from kat_cases import SCENARIOS, T32
from oracle.oracle import OTree


def ok(r):
    assert r[0] == "Ok", r
    return r[1]


def A(ts, path, v):
    return ("add", ts, list(path), v)


def D(path):
    return ("del", list(path))


def run(name):
    replica, ops = SCENARIOS[name]
    t = OTree(replica)
    for op in ops:
        r = t.apply(op)
        if r[0] != "Ok":
            return r
        t = r[1]
    return "Ok", t


# ---------------- tests/CRDTreeTest.elm ----------------

class TestCRDTree:
    def test_add(self):  # :56-82
        t = ok(OTree(0).add("a"))
        assert t.get_value([1]) == "a"
        assert t.operations() == [A(1, [0], "a")]
        assert t.last_operation() == A(1, [0], "a")

    def test_add_after(self):  # :85-122
        t = ok(OTree(0).add("a"))
        t = ok(t.add("b"))
        t = ok(t.add_after([1], "c"))
        assert [t.get_value([i]) for i in (1, 2, 3)] == ["a", "b", "c"]
        assert t.operations() == [A(1, [0], "a"), A(2, [1], "b"), A(3, [1], "c")]
        assert t.last_operation() == A(3, [1], "c")

    def test_add_after2(self):  # :125-160
        t = OTree(0)
        for v in "abc":
            t = ok(t.add(v))
        t = ok(t.add_after([1], "z"))
        assert t.visible_values() == ["a", "z", "b", "c"]
        assert t.operations() == [A(1, [0], "a"), A(2, [1], "b"), A(3, [2], "c"), A(4, [1], "z")]
        assert t.last_operation() == A(4, [1], "z")

    def test_batch(self):  # :163-199
        t = ok(OTree(0).batch([lambda t: t.add("a"), lambda t: t.add("b")]))
        assert t.get_value([1]) == "a" and t.get_value([2]) == "b"
        assert t.operations() == [A(1, [0], "a"), A(2, [1], "b")]
        assert t.last_operation() == ("batch", [A(1, [0], "a"), A(2, [1], "b")])

    def test_add_branch(self):  # :202-258
        t = ok(OTree(0).batch([lambda t: t.add_branch("a"), lambda t: t.add_branch("b"),
                               lambda t: t.add_branch("c"), lambda t: t.add_branch("d"),
                               lambda t: t.add("e"), lambda t: t.add("f")]))
        expected = [A(1, [0], "a"), A(2, [1, 0], "b"), A(3, [1, 2, 0], "c"), A(4, [1, 2, 3, 0], "d"),
                    A(5, [1, 2, 3, 4, 0], "e"), A(6, [1, 2, 3, 4, 5], "f")]
        assert t.get_value([1]) == "a"
        assert t.get_value([1, 2]) == "b"
        assert t.get_value([1, 2, 3]) == "c"
        assert t.get_value([1, 2, 3, 4]) == "d"
        assert t.get_value([1, 2, 3, 4, 5]) == "e"
        assert t.get_value([1, 2, 3, 4, 6]) == "f"
        assert t.operations() == expected
        assert t.last_operation() == ("batch", expected)
        # the same ops applied remotely build the same tree
        r = ok(run("add_branch"))
        assert r.canonical(0)[2] == t.canonical(0)[2]

    def test_delete(self):  # :261-278
        t = ok(OTree(0).add("a"))
        t = ok(t.delete([1]))
        assert t.get_value([1]) is None
        assert t.last_operation() == D([1])

    def test_add_to_deleted_branch(self):  # :281-321
        t = ok(run("add_to_deleted_branch"))
        assert t.get_value([1]) is None
        assert t.operations() == [A(1, [0], "a"), D([1])]
        assert t.last_operation() == ("batch", [A(1, [0], "a"), D([1])])

    def test_apply_batch(self):  # :324-358
        t = ok(run("apply_batch"))
        assert t.get_value([1]) == "a" and t.get_value([2]) == "b"
        assert t.operations() == [A(1, [0], "a"), A(2, [1], "b")]
        assert t.last_operation() == ("batch", [A(1, [0], "a"), A(2, [1], "b")])

    def test_batch_atomicity(self):  # :482-498
        r = run("atomicity")
        assert r[0] == "OperationFailed"
        assert r[1].kind == "add" and r[1].ts == 2

    def test_add_is_idempotent(self):  # :361-398
        t = ok(run("add_idempotent"))
        assert t.get_value([1]) == "a"
        assert t.operations() == [A(1, [0], "a")]
        assert t.last_operation() == ("batch", [A(1, [0], "a")])

    def test_insertion_between_nodes(self):  # :401-440
        t = ok(run("insertion_between"))
        assert [t.get_value([i]) for i in (1, 2, 3)] == ["a", "c", "b"]
        assert t.operations() == [A(1, [0], "a"), A(2, [1], "c"), A(3, [1], "b")]
        assert t.last_operation() == ("batch", t.operations())

    def test_add_leaf(self):  # :443-479
        t = ok(run("add_leaf"))
        assert t.get_value([1, 2]) == "b" and t.get_value([1, 3]) == "c"
        assert t.operations() == [A(1, [0], "a"), A(2, [1, 0], "b"), A(3, [1, 2], "c")]
        assert t.last_operation() == ("batch", t.operations())

    def test_delete_is_idempotent(self):  # :501-544
        t = ok(run("delete_idempotent"))
        assert t.get_value([1]) is None
        assert t.operations() == [A(1, [0], "a"), D([1])]
        assert t.last_operation() == ("batch", [A(1, [0], "a"), D([1])])

    @pytest.mark.parametrize("rid", [0, 1])
    def test_timestamps(self, rid):  # :547-589
        t = ok(OTree(rid).batch([lambda t: t.add("a"), lambda t: t.add("b"), lambda t: t.add("c")]))
        o = rid * T32
        assert t.operations() == [A(o + 1, [0], "a"), A(o + 2, [o + 1], "b"), A(o + 3, [o + 2], "c")]

    def test_operations_since(self):  # :592-658
        t = ok(run("operations_since"))
        full = [A(1, [0], "a"), A(2, [1], "b"), A(3, [2], "c"), A(4, [3], "d"), D([3]), A(5, [4], "e"),
                A(6, [5], "f")]
        assert t.operations_since(0) == full
        assert t.operations_since(2) == full[1:]
        assert t.operations_since(6) == [A(6, [5], "f")]
        assert t.operations_since(10) == []


# ---------------- tests/NodeTest.elm ----------------

class TestNode:
    @pytest.mark.parametrize("name", ["append_smaller_first", "append_bigger_first"])
    def test_append(self, name):  # :24-35
        assert ok(run(name)).visible_values() == ["b", "a"]

    @pytest.mark.parametrize("name", ["insert_smaller_first", "insert_bigger_first"])
    def test_insert(self, name):  # :36-59
        assert ok(run(name)).visible_values() == [1, 6, 5, 4, 2, 3]

    def test_flat_map(self):  # :85-134 (map/filterMap/foldl/foldr/head/last/find skip tombstone x)
        vals = ok(run("flat_example")).visible_values()
        assert vals == ["a", "b", "c", "d"]
        assert vals[0] == "a" and vals[-1] == "d"  # head / last
        assert vals[:vals.index("c")] == ["a", "b"]  # loop ... Done at 'c'

    def test_descendant_path_timestamp(self):  # :67-84
        t = ok(run("nested_example"))
        assert t.get_value([1, 2, 3, 4]) == "d"
        assert t.get_path([1, 2, 3, 4]) == [1, 2, 3, 4]
        assert t.get_path([1, 2, 3, 4])[-1] == 4


# ---------------- SURVEY.md Appendix C (hand-traced from src/Internal/Node.elm:56-122) ----------------

class TestAppendixC:
    def test_copy_quirk(self):  # C.1
        t = ok(run("quirk_copy"))
        # raw chain 10 -> 20(copy of 30, path [30]) -> 15; key 30 orphaned
        words, n, _ = t.canonical(0)
        recs = parse_structure(words)
        top = {r["key"]: r for r in recs if r["depth"] == 0}
        assert top[10]["next"] == 20
        assert top[20]["kind"] == 1 and top[20]["path"] == [30] and top[20]["next"] == 15
        assert top[30]["kind"] == 2  # the later Delete [30] tombstoned the orphan
        assert t.visible_values() == ["p", "r", "s"]

    def test_deletes_last(self):  # C.2
        t = ok(run("quirk_deletes_last"))
        assert t.visible_values() == ["p", "s"]

    def test_non_lamport(self):  # C.3
        assert ok(run("non_lamport")).visible_values() == [1, 5, 3, 2]

    def test_delete_sentinel(self):  # C.4
        t = ok(run("delete_sentinel"))
        assert t.operations() == [] and t.last_operation() == ("batch", [])

    def test_add_under_sentinel(self):  # C.5
        t = ok(run("add_under_sentinel"))
        assert t.operations() == [] and t.last_operation() == ("batch", [])

    def test_replica_accounting(self):  # C.6
        t = ok(run("replica_accounting"))
        assert t.timestamp() == T32 + 2  # the AlreadyApplied duplicate still bumps
        assert t.replicas() == {1: T32 + 1, 2: 2 * T32 + 1}

    def test_errors(self):
        assert run("invalid_path_empty")[0] == "InvalidPath"
        assert run("invalid_path_missing_parent")[0] == "InvalidPath"
        r = run("delete_missing")
        assert r[0] == "OperationFailed" and r[1].kind == "del"

    def test_quirk_copy_branch(self):
        t = ok(run("quirk_copy_branch"))
        recs = parse_structure(t.canonical(0)[0])
        # slot 20 holds a copy of 30 carrying its own children dict (persistent copy)
        kids20 = children_of(recs, 20)
        kids30 = children_of(recs, 30)
        assert 31 in kids20 and 31 in kids30
        assert 32 in kids20 and 32 not in kids30
        assert 33 in kids30 and 33 not in kids20


def parse_structure(words):
    out = []
    i = 0
    n = len(words)
    while i < n:
        d, k, kind, hn, nx, v, pl = (int(x) for x in words[i:i + 7])
        path = [int(x) for x in words[i + 7:i + 7 + pl]]
        out.append(dict(depth=d, key=k, kind=kind, next=nx if hn else None, val=v, path=path))
        i += 7 + pl
    return out


def children_of(recs, key):
    """keys of the depth-1 dict under the depth-0 entry `key` (DFS order dump)."""
    kids = []
    inside = False
    for r in recs:
        if r["depth"] == 0:
            inside = r["key"] == key
        elif inside and r["depth"] == 1:
            kids.append(r["key"])
    return kids


# ---------------- traversal: the reference's documented examples ----------------
# (src/CRDTree.elm:447-466: get / getValue on treeA = batch [addBranch "a",
# addBranch "b", add "c"] with replica 1; the walk order follows A.8)

class TestTraversal:
    def tree_a(self):
        return ok(OTree(1).batch([lambda t: t.add_branch("a"), lambda t: t.add_branch("b"), lambda t: t.add("c")]))

    def test_get_doc_examples(self):  # src/CRDTree.elm:447-466
        t = self.tree_a()
        o = T32
        assert t.node([o + 1])[:3] == ("node", "a", (o + 1,))
        assert t.node([o + 1, o + 2])[:3] == ("node", "b", (o + 1, o + 2))
        assert t.node([o + 1, o + 2, o + 3])[:3] == ("node", "c", (o + 1, o + 2, o + 3))
        assert t.node([4]) is None
        assert t.node([]) is None
        # a dict sentinel exists: Tombstone [] Nothing, whose parent is the root (path [])
        assert t.node([o + 1, 0]) == ("tombstone", None, (), o + 2)
        assert t.node_query("parent", [o + 1, 0])[0] == "root"

    def test_next_prev_children_walk(self):
        t = ok(OTree(1).batch([lambda t: t.add("a"), lambda t: t.add("b"), lambda t: t.add("c")]))
        o = T32
        ch = t.node_query("children", [])  # the root's children: a, b, c in chain order
        assert [c[1] for c in ch] == ["a", "b", "c"]
        assert t.node_query("next", [o + 1])[1] == "b"
        assert t.node_query("prev", [o + 3])[1] == "b"
        assert t.node_query("prev", [o + 1]) is None
        assert t.node_query("next", [o + 3]) is None
        # walk ... Nothing starts after the root's head: b, c
        assert [n[1] for n in t.node_query("walk_start")] == ["b", "c"]
        t2 = ok(t.delete([o + 2]))
        assert t2.node_query("next", [o + 1])[1] == "c"  # skips the Tombstone
        assert t2.node_query("prev", [o + 3])[1] == "a"

    def test_walk_skips_each_head(self):  # A.8
        t = ok(OTree(1).batch([lambda t: t.add("a"), lambda t: t.add_branch("b"), lambda t: t.add("b1"),
                               lambda t: t.add("b2")]))
        # root: a, b; b's children: b1, b2. walk Nothing: after head a -> b, then b's children after b1 -> b2
        assert [n[1] for n in t.node_query("walk_start")] == ["b", "b2"]


@pytest.mark.parametrize("seed", [0xC0FFEE03, 5, 6])
def test_flat_fast_restatement_matches_general(seed):
    """orc_flat_replay (the flat, Adds-only specialisation) gives the general
    restatement's canonical dumps; orc_flat_check accepts that order and
    rejects a perturbed one."""
    import ctypes as C
    import numpy as np
    from crdtm import _native as N
    from oracle.oracle import lib, _ptr
    L = lib()
    m = 30000
    s = N.synth(n_ops=m, replicas=8 + seed % 64, window=64, seed=seed)
    h = np.zeros(2, np.uint64)
    w = np.zeros(2, np.uint64)
    err = C.c_int64(-1)
    na = C.c_uint64()
    args = (_ptr(s["kind"]), _ptr(s["ts"]), _ptr(s["path_off"]), _ptr(s["path"]), _ptr(s["val"]))
    assert L.orc_flat_replay(m, *args, C.byref(err), _ptr(h), _ptr(w), C.byref(na)) == 0
    t = L.orc_init(0)
    e2 = C.c_int64(-1)
    assert L.orc_apply(t, 1, 0, m, *args, C.byref(e2)) == 0
    for which in (0, 1):
        hh = C.c_uint64()
        assert (L.orc_canonical(t, which, None, 0, C.byref(hh)), hh.value) == (int(w[which]), int(h[which]))
    nw = L.orc_canonical(t, 1, None, 0, None)
    buf = np.zeros(nw, np.int64)
    L.orc_canonical(t, 1, _ptr(buf), nw, None)
    L.orc_free(t)
    keys = buf[3::4].copy()
    chk = (_ptr(s["ts"]), _ptr(s["path_off"]), _ptr(s["path"]))
    assert L.orc_flat_check(len(keys), _ptr(keys), m, *chk) == 0
    keys[100], keys[101] = keys[101], keys[100]
    assert L.orc_flat_check(len(keys), _ptr(keys), m, *chk) > 0


def test_guard_g_statistics_hand_traced():
    """Guard G as the oracle counts it: an Add fails when
    its findInsertion walk meets a Tombstone above its timestamp as a raw
    `next` key. Appendix C.1: Add 15 after 10 meets Tombstone 20 > 15 (the
    copy quirk fires); C.2 (the Deletes last): no Add fails; a Tombstone below
    the Add's timestamp stops the walk without failing it."""
    import ctypes as C
    import numpy as np
    from oracle.oracle import lib

    def stats(ops):
        t = OTree(0)
        assert t.apply(Batch(ops))[0] == "Ok"
        out = np.zeros(3, np.uint64)
        lib().orc_guard_stats(out.ctypes.data_as(C.c_void_p))
        return tuple(int(x) for x in out)

    adds = [Add(10, [0], "a"), Add(20, [10], "b"), Add(30, [20], "c")]
    assert stats(adds + [Delete([20]), Add(15, [10], "d")]) == (4, 1, 5)
    assert stats(adds + [Add(15, [10], "d"), Delete([20]), Delete([30])]) == (4, 0, 6)
    # a Tombstone below the Add: 40 after 10 stops at Tombstone 20 < 40
    assert stats(adds + [Delete([20]), Add(40, [10], "d")]) == (4, 0, 5)
    # out[2], ops that reached their dict: not one whose path meets a Tombstone
    # (src/Internal/Node.elm:140-141: AlreadyApplied) — Add under deleted 20
    assert stats(adds + [Delete([20]), Add(50, [20, 0], "e")]) == (3, 0, 4)
