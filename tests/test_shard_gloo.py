"""Multi-process (world_size 2, gloo on CPU) checks of the document sharding
and op-log exchange used by bench.py --workload trees (RCCL on the GPU node)."""
import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_docs, per_doc, q):
    sys.path.insert(0, os.path.join(ROOT, "crdt-graph_amd"))
    import torch
    import torch.distributed as dist
    from crdtm import _native as N
    from crdtm import shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s = N.synth(n_ops=per_doc, n_docs=n_docs, replicas=8, window=16, p_delete=0.2, seed=0xC0FFEE05)
    doc_off = np.arange(n_docs + 1, dtype=np.uint32) * per_doc
    local = torch.from_numpy(shard.local_log(s, doc_off, rank, world, replicas=8))
    allrec = shard.all_gather_records(local)
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
    q.put((rank, bool(ok), int(local.shape[0]), int(allrec.shape[0])))
    dist.barrier()
    dist.destroy_process_group()


def test_oplog_exchange_world2():
    world, n_docs, per_doc = 2, 12, 300
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_docs, per_doc, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    assert all(ok for _, ok, _, _ in res), res
    # every op travels in exactly one rank's log; everyone receives all of them
    assert sum(r[2] for r in res) == n_docs * per_doc
    assert all(r[3] == n_docs * per_doc for r in res)
