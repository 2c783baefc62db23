"""Merges after a tree reset, through the C ABI (crdtm_tree_reset / crdtm_apply).

The reset's launch also initialises the context's result block, and the flat
speculation that follows skips its own init (crdtm_ctx::dres_ready,
csrc/api.hip crdtm_tree_reset, csrc/merge.hip apply_core). The block belongs
to the context, not the tree, so these sequences check that every other use
of it in between leaves the next merge exact: a merge on another tree of the
same context, operationsSince (its search writes the block), a failing merge,
and a reset whose merge takes the general path. Each merge is compared with
the oracle's literal replay of the same batch (src/CRDTree.elm:298-325).
Also: device-resident ops at any alignment (the bench's and the ports' path).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from crdtm import _native as N  # noqa: E402
from crdtm.tree import CRDTree  # noqa: E402
from parity_util import (engine_summary, oracle_apply_arrays, oracle_summary,  # noqa: E402
                         oracle_visible_vals)


DELETE = 1  # (include/crdtm.h CRDTM_DELETE)


def _flat(n, seed):
    return N.synth(n_ops=n, replicas=8, window=32, seed=seed)


def _nested(n, seed):
    return N.synth(n_ops=n, replicas=4, window=16, p_delete=0.2, p_branch=0.1, max_depth=3, seed=seed)


def _reset(t):
    N.check(N.lib().crdtm_tree_reset(t._h, 0), "crdtm_tree_reset")


def _check(t, v, m, path=None):
    ot, rc, _ = oracle_apply_arrays(v, m)
    assert rc == 0
    res = t.apply_arrays(v, m)
    assert res.code == 0
    if path is not None:
        assert res.path_taken == path
    assert engine_summary(t) == oracle_summary(ot)
    assert np.array_equal(t.document_handles(), oracle_visible_vals(ot))


def test_reset_then_merges_sharing_the_context():
    a, b = CRDTree.init(0), CRDTree.init(0)
    f1, f2 = _flat(20_000, 11), _flat(30_000, 12)
    _check(a, f1, 20_000, N.PATH_CLOSED_FORM)
    _reset(a)  # initialises the shared block
    _check(b, f2, 30_000, N.PATH_CLOSED_FORM)  # another tree's merge takes it
    _reset(a)
    _check(a, f1, 20_000, N.PATH_CLOSED_FORM)
    _reset(b)
    _reset(a)  # (two resets in a row, then a merge on the other tree)
    _check(b, f1, 20_000, N.PATH_CLOSED_FORM)
    _check(a, f2, 30_000, N.PATH_CLOSED_FORM)


def test_reset_then_operations_since_then_merge():
    a = CRDTree.init(0)
    f = _flat(25_000, 21)
    _check(a, f, 25_000, N.PATH_CLOSED_FORM)
    _reset(a)
    a.operations_since(int(f["ts"][100]))  # (its search writes the result block)
    _check(a, f, 25_000, N.PATH_CLOSED_FORM)
    _reset(a)
    a.operations_since(12345)
    _check(a, _flat(5_000, 22), 5_000, N.PATH_CLOSED_FORM)


def test_reset_then_failing_and_general_merges():
    a = CRDTree.init(0)
    f = _flat(10_000, 31)
    # the batch plus a Delete of an earlier Add's node: the speculation's shape
    # check fails after the reset, and the general path merges the batch
    n = 10_000
    mixed = dict(kind=np.append(f["kind"], np.uint8(DELETE)), ts=np.append(f["ts"], np.int64(0)),
                 path_off=np.append(f["path_off"], np.uint32(n + 1)), path=np.append(f["path"][:n], f["ts"][100]),
                 val=np.append(f["val"], np.uint32(0)))
    _reset(a)
    _check(a, mixed, n + 1)
    # a batch the reference rejects (an Add under a missing parent): no commit
    bad = {k: v.copy() for k, v in f.items() if v is not None}
    bad["path"][7000] = (99 << 32) | 12345
    _reset(a)
    ot, rc, _ = oracle_apply_arrays(bad, 10_000)
    res = a.apply_arrays(bad, 10_000)
    assert (res.code == 0) == (rc == 0)
    _reset(a)
    _check(a, f, 10_000, N.PATH_CLOSED_FORM)
    _reset(a)
    _check(a, _nested(8_000, 32), 8_000)  # the general nested path after a reset
    _reset(a)
    _check(a, f, 10_000, N.PATH_CLOSED_FORM)


def test_reset_of_a_tree_whose_version_is_shared():
    """A clone shares the merged state (copy on write); resetting the original
    then merging into it must leave the clone's version untouched, and the
    clone merges on from its own state."""
    a = CRDTree.init(0)
    f1, f2 = _flat(15_000, 41), _flat(12_000, 42)
    _check(a, f1, 15_000, N.PATH_CLOSED_FORM)
    b = a.clone()
    _reset(a)
    _check(a, f2, 12_000, N.PATH_CLOSED_FORM)
    ot1, rc, _ = oracle_apply_arrays(f1, 15_000)
    assert rc == 0
    assert engine_summary(b) == oracle_summary(ot1)
    assert np.array_equal(b.document_handles(), oracle_visible_vals(ot1))
    extra = dict(kind=np.zeros(2, np.uint8), ts=np.array([(9 << 32) + 1, (9 << 32) + 2], np.int64),
                 path_off=np.array([0, 1, 2], np.uint32), path=np.array([int(f1["ts"][5]), (9 << 32) + 1], np.int64),
                 val=np.array([1, 2], np.uint32))
    _, rc2, _ = oracle_apply_arrays(extra, 2, tree=ot1)
    assert rc2 == 0 and b.apply_arrays(extra, 2).code == 0
    assert engine_summary(b) == oracle_summary(ot1)
    assert np.array_equal(b.document_handles(), oracle_visible_vals(ot1))


@pytest.mark.parametrize("pad", [0, 1, 3])
@pytest.mark.parametrize("kind", ["flat", "nested"])
def test_device_resident_ops_any_alignment(pad, kind):
    """crdtm_apply on device-resident ops (ops_on_device = 1, the bench's and
    the Elm ports' path) whose arrays start `pad` elements into their
    allocations: misaligned columns are copied to aligned scratch
    (csrc/api.hip align_ops) and the merge equals the oracle's."""
    import torch
    n = 12_000
    s = _flat(n, 91) if kind == "flat" else _nested(n, 92)
    dev = torch.device("cuda", 0)
    keep = []

    def on_dev(a):
        t = torch.zeros(len(a) + pad, dtype=torch.from_numpy(a[:1]).dtype, device=dev)
        t[pad:] = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        keep.append(t)
        return t[pad:].data_ptr()

    npath = int(s["path_off"][n])
    ops = N.Ops(n, npath, on_dev(s["kind"]), on_dev(s["ts"]), on_dev(s["path_off"]), on_dev(s["path"][:npath]),
                on_dev(s["val"]), None)
    torch.cuda.synchronize()
    ot, rc, _ = oracle_apply_arrays(s, n)
    et = CRDTree.init(0)
    res = et.apply_arrays(ops, n, on_device=True)
    assert res.code == rc
    assert engine_summary(et) == oracle_summary(ot)
    assert np.array_equal(et.document_handles(), oracle_visible_vals(ot))


def test_two_contexts_interleaved():
    """Two engine contexts on one device (each its own stream, result block,
    pinned staging and scratch arena), their merges interleaved: each tree
    equals the oracle's."""
    import ctypes as C
    L = N.lib()
    ctx2 = C.c_void_p()
    N.check(L.crdtm_ctx_create(0, None, C.byref(ctx2)), "crdtm_ctx_create")
    h = C.c_void_p()
    N.check(L.crdtm_tree_create(ctx2, 0, C.byref(h)), "crdtm_tree_create")
    b = CRDTree(h)
    a = CRDTree.init(0)
    try:
        f1, f2 = _flat(20_000, 51), _nested(9_000, 52)
        _check(a, f1, 20_000, N.PATH_CLOSED_FORM)
        _check(b, f2, 9_000)
        _reset(a)
        _reset(b)
        _check(b, f1, 20_000, N.PATH_CLOSED_FORM)
        _check(a, f2, 9_000)
    finally:
        del b
        import gc
        gc.collect()
        L.crdtm_ctx_destroy(ctx2)
