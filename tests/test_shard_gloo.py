"""Multi-process (world_size 2, gloo on CPU) checks of the document sharding
and op-log exchange used by bench.py --workload trees (RCCL on the GPU node):
the op-log exchange by document owner (shard.Exchange: all_to_all_single,
and the padded all-gather fallback), the assembly of each
rank's documents, and the merge of the assembled documents on the oracle
(orc_forest_apply, oracle/crdtree_oracle.cpp) against the single-process
stream's documents."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle_forest(ops, n_docs, per_doc):
    import numpy as np
    from oracle.oracle import _ptr, lib as olib
    n = n_docs * per_doc
    a = dict(kind=np.ascontiguousarray(ops["kind"][:n], np.uint8), ts=np.ascontiguousarray(ops["ts"][:n], np.int64),
             path=np.ascontiguousarray(ops["path"][:n], np.int64), val=np.ascontiguousarray(ops["val"][:n], np.uint32))
    off = np.arange(n_docs + 1, dtype=np.uint32) * per_doc
    path_off = np.arange(n + 1, dtype=np.uint32)
    out = dict(code=np.zeros(n_docs, np.int32), err=np.zeros(n_docs, np.int64), hash=np.zeros(n_docs, np.uint64),
               words=np.zeros(n_docs, np.uint64), ts=np.zeros(n_docs, np.int64))
    olib().orc_forest_apply(n_docs, _ptr(off), 0, _ptr(a["kind"]), _ptr(a["ts"]), _ptr(path_off), _ptr(a["path"]),
                            _ptr(a["val"]), _ptr(out["code"]), _ptr(out["err"]), _ptr(out["hash"]),
                            _ptr(out["words"]), _ptr(out["ts"]))
    return out


def _worker(rank, world, port, n_docs, per_doc, q, mode="auto"):
    sys.path.insert(0, os.path.join(ROOT, "crdt-graph_amd"))
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from crdtm import _native as N
    from crdtm import shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s = N.synth(n_ops=per_doc, n_docs=n_docs, replicas=8, window=16, p_delete=0.2, seed=0xC0FFEE05)
    doc_off = np.arange(n_docs + 1, dtype=np.uint32) * per_doc
    local = torch.from_numpy(shard.local_log(s, doc_off, rank, world, replicas=8))
    ex = shard.Exchange(local, mode=mode)
    for _ in range(2):  # the buffers are reused step after step
        allrec = ex.gather()
    if ex.mode == "all_gather":
        assert allrec.shape[0] == world * ex.block and ex.counts[rank] == local.shape[0]
    else:  # exactly this rank's documents' records, from every rank
        assert ex.mode == "all_to_all" and mode in ("auto", "all_to_all")
        assert allrec.shape[0] == sum(ex.recv_splits) and sum(ex.send_splits) == local.shape[0]
        assert bool(((allrec[:, 0] >> 32) % world == rank).all())
    ops, my_off, keep = shard.assemble(allrec, rank, world, n_docs, per_doc)
    n_kept = int(keep.sum())
    # expected: the owned documents' streams, sliced directly from the generator output
    mine = [t for t in range(n_docs) if t % world == rank]
    idx = np.concatenate([np.arange(t * per_doc, (t + 1) * per_doc) for t in mine])
    m = len(idx)  # arrays carry one spill slot at the end
    ok = (np.array_equal(ops["kind"].numpy()[:m], s["kind"][idx]) and np.array_equal(ops["ts"].numpy()[:m], s["ts"][idx])
          and np.array_equal(ops["path"].numpy()[:m], s["path"][idx])
          and np.array_equal(ops["val"].numpy()[:m].astype(np.uint32), s["val"][idx]) and n_kept == m
          and int(my_off[-1]) == m)
    # the assembled documents merge exactly as the generator's own streams do
    got = _oracle_forest({k: v.numpy() for k, v in ops.items()}, len(mine), per_doc)
    want = _oracle_forest({k: s[k][idx] for k in ("kind", "ts", "path", "val")}, len(mine), per_doc)
    merged = all(np.array_equal(got[k], want[k]) for k in got) and bool(np.all(got["code"] == 0))
    q.put((rank, bool(ok and merged), int(local.shape[0]), int(n_kept), ex.mode))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["all_to_all", "all_gather"])
def test_oplog_exchange_world2(mode):
    world, n_docs, per_doc = 2, 12, 300
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_docs, per_doc, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    assert all(r[1] for r in res) and all(r[4] == mode for r in res), res
    # every op travels in exactly one rank's log; every op is kept by exactly one rank
    assert sum(r[2] for r in res) == n_docs * per_doc
    assert sum(r[3] for r in res) == n_docs * per_doc
