"""Multi-GPU sharding of many independent documents.

One process per GPU. Every rank hosts some of the R simulated replicas and
holds, for every document, the ops those replicas authored (their op logs).
A step is: exchange the op logs by document owner (document t -> rank
t mod world) with one all-to-all (RCCL over xGMI with backend "nccl"; gloo in
CPU tests) — or, in `all_gather` mode (north_star's named collective), an
all-gather of every rank's whole log, of which each rank keeps its documents —
put each document's ops back in causal order, and merge every owned document
with `crdtm_forest_apply`. There is no second exchange: the documents are
independent CRDTrees.

Op record (4 x int64, flat documents): [doc << 32 | seq, kind << 32 | val, ts, anchor]
where seq is the op's position in its document's causal stream.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

REC_W = 4


def owner(doc, world):
    return doc % world


def hosted_replicas(rank, world, replicas):
    """Replica ids 1..R hosted by `rank` (round-robin)."""
    return [r for r in range(1, replicas + 1) if (r - 1) % world == rank]


def pack_records(s, doc_off, mask):
    """Host op arrays (flat documents) -> records of the ops selected by mask."""
    n = len(s["kind"])
    doc = np.repeat(np.arange(len(doc_off) - 1, dtype=np.int64), np.diff(doc_off.astype(np.int64)))
    seq = np.arange(n, dtype=np.int64) - doc_off.astype(np.int64)[doc]
    rec = np.empty((n, REC_W), np.int64)
    rec[:, 0] = (doc << 32) | seq
    rec[:, 1] = (s["kind"].astype(np.int64) << 32) | s["val"].astype(np.int64)
    rec[:, 2] = s["ts"]
    rec[:, 3] = s["path"][s["path_off"][:-1].astype(np.int64)]
    return rec[mask]


def local_log(s, doc_off, rank, world, replicas):
    """This rank's share of every document's stream: the ops its replicas authored.
    Deletes carry no timestamp; they are attributed to the replica of the node
    they delete (its key's replica id), which spreads them over the ranks."""
    key = np.where(s["kind"] == 0, s["ts"], s["path"][s["path_off"][:-1].astype(np.int64)])
    rid = key >> 32
    mine = np.isin(rid, hosted_replicas(rank, world, replicas))
    if rank == 0:
        mine |= (rid < 1) | (rid > replicas)  # anything unattributed stays with rank 0
    return pack_records(s, doc_off, mine)


class Exchange:
    """The op-log exchange of one step, with its buffers kept across steps.

    Every record goes to the rank that owns its document (t mod world) with
    one all-to-all (RCCL `all_to_all_single`): a rank receives exactly the
    records of the documents it merges, (world - 1) / world of its own
    documents' ops, instead of every rank's whole log (the all-gather sent
    world x as many bytes: 2.8 GB per rank per step at 8 ranks for 0.35 GB
    used). The local records are sorted by destination once; the per-pair
    counts are static, so they are exchanged once at setup (no host sync in
    the step). `gather()` is one all_to_all_single into a persistent receive
    buffer that the assembly reads as it is. Where the backend has no
    all-to-all, the padded all-gather of every log is the fallback
    (`mode` says which)."""

    def __init__(self, local: torch.Tensor, group=None, mode: str = "auto"):
        self.group = group
        self.dist = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
        self.world = dist.get_world_size(group) if self.dist else 1
        self.mode = "local"
        if not self.dist:
            self.recv = local
            self.block = local.shape[0]
            return
        if mode not in ("auto", "all_to_all", "all_gather"):
            raise ValueError(f"exchange mode {mode!r}")
        if mode in ("auto", "all_to_all"):
            ok = 1
            try:
                self._setup_all_to_all(local)
            except (RuntimeError, NotImplementedError):
                if mode == "all_to_all":
                    raise
                ok = 0
            if mode == "auto":
                # every rank takes the same mode: a rank whose setup raised (or
                # saw an asynchronous error) must not leave the others in the
                # all-to-all while it all-gathers
                flag = torch.tensor([ok], dtype=torch.int32, device=local.device)
                dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
                ok = int(flag.item())
            if ok:
                self.mode = "all_to_all"
                return
        self._setup_all_gather(local)
        self.mode = "all_gather"

    def _setup_all_to_all(self, local):
        dest = (local[:, 0] >> 32) % self.world
        order = torch.argsort(dest, stable=True)
        self.send = local[order].contiguous()
        send_counts = torch.bincount(dest, minlength=self.world).to(torch.int64)
        recv_counts = torch.empty_like(send_counts)
        dist.all_to_all_single(recv_counts, send_counts, group=self.group)  # once, at setup
        self.send_splits = [int(c) for c in send_counts.cpu()]
        self.recv_splits = [int(c) for c in recv_counts.cpu()]
        self.block = max(self.recv_splits)
        self.recv = torch.empty((sum(self.recv_splits), REC_W), dtype=torch.int64, device=local.device)
        self._all_to_all()  # (fails here, at setup, where the backend has none)

    def _setup_all_gather(self, local):
        cnt = torch.tensor([local.shape[0]], dtype=torch.int64, device=local.device)
        cnts = torch.zeros(self.world, dtype=torch.int64, device=local.device)
        dist.all_gather_into_tensor(cnts, cnt, group=self.group)
        self.counts = [int(c) for c in cnts.cpu()]  # once, at setup
        self.block = max(self.counts)
        self.send = torch.full((self.block, REC_W), -1, dtype=torch.int64, device=local.device)
        self.send[:local.shape[0]] = local
        self.recv = torch.empty((self.world * self.block, REC_W), dtype=torch.int64, device=local.device)

    def _all_to_all(self):
        dist.all_to_all_single(self.recv, self.send, self.recv_splits, self.send_splits, group=self.group)

    @property
    def recv_bytes(self) -> int:
        """Bytes this rank receives per step (its own block included)."""
        return int(self.recv.numel() * self.recv.element_size())

    def gather(self) -> torch.Tensor:
        """The records this rank merges (all_gather mode: every rank's, padding rows included)."""
        if self.dist:
            if self.mode == "all_to_all":
                self._all_to_all()
            else:
                dist.all_gather_into_tensor(self.recv, self.send, group=self.group)
        return self.recv


def all_gather_records(local: torch.Tensor, group=None) -> torch.Tensor:
    """All-gather variable-length record blocks: counts first, then padded blocks."""
    if not (dist.is_available() and dist.is_initialized()):
        return local
    world = dist.get_world_size(group)
    if world == 1:
        return local
    cnt = torch.tensor([local.shape[0]], dtype=torch.int64, device=local.device)
    cnts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(cnts, cnt, group=group)
    cnts = [int(c.item()) for c in cnts]
    m = max(cnts)
    pad = torch.zeros((m, REC_W), dtype=torch.int64, device=local.device)
    pad[:local.shape[0]] = local
    if local.device.type == "cuda":
        out = torch.empty((world * m, REC_W), dtype=torch.int64, device=local.device)
        dist.all_gather_into_tensor(out, pad, group=group)
        parts = [out[k * m:k * m + cnts[k]] for k in range(world)]
    else:
        bufs = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(bufs, pad, group=group)
        parts = [bufs[k][:cnts[k]] for k in range(world)]
    return torch.cat(parts, 0)


_ARANGE = {}
_SOA = {}


def assemble(records: torch.Tensor, rank, world, n_docs, per_doc, ctx=None):
    """Records of every replica -> SoA ops of this rank's documents in causal order.
    Documents owned: t = rank, rank + world, ... (local index t // world);
    every document holds exactly per_doc ops. Sync-free: records of other
    ranks' documents are scattered into a spill slot at index n."""
    n_mine = (n_docs - rank + world - 1) // world
    n = n_mine * per_doc
    doc_off = np.arange(n_mine + 1, dtype=np.uint32) * per_doc
    if ctx is not None and records.device.type == "cuda":
        # one HIP pass (crdtm_shard_assemble) on the engine's stream
        import ctypes as C
        from . import _native as N
        dev = records.device
        key = ("soa", str(dev), n, ctx.value if hasattr(ctx, "value") else id(ctx))
        out = _SOA.get(key)
        if out is None:  # every slot is rewritten each step: kept across steps
            out = dict(kind=torch.zeros(n + 1, dtype=torch.uint8, device=dev),
                       ts=torch.zeros(n + 1, dtype=torch.int64, device=dev),
                       path_off=torch.empty(n + 1, dtype=torch.int32, device=dev),
                       path=torch.zeros(n + 1, dtype=torch.int64, device=dev),
                       val=torch.zeros(n + 1, dtype=torch.int32, device=dev))
            _SOA.clear()
            _SOA[key] = out
        records = records.contiguous()
        ops = N.Ops(n, n, out["kind"].data_ptr(), out["ts"].data_ptr(), out["path_off"].data_ptr(),
                    out["path"].data_ptr(), out["val"].data_ptr(), None)
        N.check(N.lib().crdtm_shard_assemble(ctx, C.c_void_p(records.data_ptr()), records.shape[0], rank, world,
                                             per_doc, C.byref(ops)), "crdtm_shard_assemble")
        return out, doc_off, None
    doc = records[:, 0] >> 32
    seq = records[:, 0] & 0xFFFFFFFF
    keep = (doc >= 0) & ((doc % world) == rank) & (seq < per_doc)  # padding rows carry -1
    dst = torch.where(keep, (doc // world) * per_doc + seq, torch.full_like(doc, n))
    dev = records.device
    kind = torch.zeros(n + 1, dtype=torch.uint8, device=dev)
    val = torch.zeros(n + 1, dtype=torch.int32, device=dev)
    ts = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    path = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    kind[dst] = (records[:, 1] >> 32).to(torch.uint8)
    val[dst] = (records[:, 1] & 0xFFFFFFFF).to(torch.int32)
    ts[dst] = records[:, 2]
    path[dst] = records[:, 3]
    key = (str(dev), n)
    if key not in _ARANGE:
        _ARANGE[key] = torch.arange(n + 1, dtype=torch.int32, device=dev)
    return dict(kind=kind, ts=ts, path_off=_ARANGE[key], path=path, val=val), doc_off, keep
