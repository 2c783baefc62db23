#!/usr/bin/env python3
"""Benchmark: merged ops/sec of CRDTree batch merges on MI355X.

Metric (BASELINE.json): merged ops/sec (whole node) on a 10M-op batch, % of
HBM peak, 1/2/4/8 GPU. One step = one `apply (Batch ops)` of the whole
synthetic batch onto a fresh tree (crdtm_tree_reset + crdtm_apply through the
C ABI), inputs already resident in HBM.

Default workload = SURVEY.md config 3: one flat RGA text document, 10M char
inserts from 64 replicas (window 256, seed 0xC0FFEE03). With N ranks (one
process per GPU: an external torchrun, or bench.py starts the N ranks itself
when launched without one), every rank merges its own independent document
(seed + rank): documents shard by id with no data-path collective, so the
scaling is weak; the only collectives are the timing barrier and max. With
N > 1 the config-5 line (RCCL all-gather of op logs + sharded merge) rides
along under "exchange".

    python bench.py --gpus N --steps K --warmup W [--workload flat10m|deep10m|deep10m_il|cfg2|trees|incr|incr_cfg2]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "crdt-graph_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md)

WORKLOADS = {
    # SURVEY.md §8d config 3
    "flat10m": dict(n_ops=10_000_000, replicas=64, window=256, seed=0xC0FFEE03),
    # depth <= 12, <= 8 children, 6.67M adds then deletes of half the nodes
    "deep10m": dict(n_ops=10_000_000, replicas=16, p_delete=1 / 3, max_depth=12, max_children=8, deletes_last=1,
                    seed=0xC0FFEE04),
    # config 4's second variant: the same deep tree shape with its Deletes interleaved
    # among the Adds (live leaves; synth.cpp genDeep), so dicts hold tombstones before later inserts:
    # measures the exact per-dict replay
    "deep10m_il": dict(n_ops=10_000_000, replicas=16, p_delete=1 / 3, max_depth=12, max_children=8, deletes_last=0,
                       seed=0xC0FFEE04),
    # one tree, 1M ops (80/20 interleaved), 16 replicas, branches, depth <= 4
    # (Deletes interleaved before later inserts: the exact sequential replay)
    "cfg2": dict(n_ops=1_000_000, replicas=16, window=64, p_delete=0.2, p_branch=0.1, max_depth=4,
                 seed=0xC0FFEE02),
    # SURVEY.md §8d config 1 shape: 2 replicas, 10k ops, 70/30 interleaved, depth <= 3
    "cfg1": dict(n_ops=10_000, replicas=2, window=8, p_delete=0.3, p_branch=0.05, max_depth=3, seed=0xC0FFEE01),
}
# CPU baseline samples (ops): config 2 and config 1 whole; the 10M-op batches as large a prefix as a bounded
# run allows (their per-op CPU cost grows with the document, so a prefix flatters the CPU)
# (about 10-30 s of CPU work each on the GPU box's host: `apply op` costs
# grow with the document -- flat10m's 1M-op sample ran over 3 minutes)
CPU_SAMPLE = {"flat10m": 200_000, "deep10m": 500_000, "deep10m_il": 500_000, "trees": 2_000_000,
              "cfg2": 1_000_000, "cfg1": 10_000}
# 100k documents x 1k ops (80/20), 8 replicas, sharded by
# document id; 12.5k documents per GPU (100k at 8 GPUs), weak scaling.
# Incremental merges: a 10M-node document, then successive 10k-op batches of the same stream
INCR = dict(base=10_000_000, batch=10_000, batches=100)
# config-2-shaped incremental merges: a 900k-op nested document with deletes,
# then 10 successive 10k-op batches of the same stream
INCR_CFG2 = dict(base=900_000, batch=10_000, batches=10)
TREES = dict(per_doc=1000, docs_per_gpu=12_500, replicas=8, window=16, p_delete=0.2, seed=0xC0FFEE05)


def alg_bytes(s):
    """Add = 49 + 8L bytes, Delete = 9 + 8L bytes (read op once, write result once)."""
    L = np.diff(s["path_off"].astype(np.int64))
    add = s["kind"] == 0
    return int(np.sum(np.where(add, 49 + 8 * L, 9 + 8 * L)))


def stream_copy_gbs(dev, nbytes=1 << 30, reps=5):
    """Measured device-copy ceiling (read + write bytes / time), SURVEY.md §8d."""
    import torch
    a = torch.empty(nbytes // 4, dtype=torch.int32, device=dev)
    b = torch.empty_like(a)
    b.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    gbs = 2 * nbytes * reps / (e0.elapsed_time(e1) / 1e3) / 1e9
    del a, b
    return gbs


def head(s, m):
    off = s["path_off"]
    return dict(kind=s["kind"][:m].copy(), ts=s["ts"][:m].copy(), val=s["val"][:m].copy(),
                path_off=off[:m + 1].copy(), path=s["path"][:off[m]].copy())


def pmc_table(workload):
    """Per-kernel HBM bytes per dispatch from the newest committed rocprofv3
    --pmc summary of this workload (profiles/r<N>_<workload>_pmc.json, written
    by tools/pmc_summary.py from separate FETCH_SIZE and WRITE_SIZE passes of
    this bench). `hbm_bytes` applies the gfx950 FETCH_SIZE x2 correction only to
    the kernels whose reads are calibrated wide streams (MI355X_MICROARCH.md,
    HBM); the others carry the raw counter bytes."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{workload}_pmc.json")),
                   key=lambda f: int(os.path.basename(f)[1:].split("_")[0]))
    for f in reversed(files):
        try:
            return json.load(open(f)), os.path.basename(f)
        except (OSError, ValueError):
            continue
    return {}, None


def pmc_live(args, counters=("FETCH_SIZE", "WRITE_SIZE")):
    """HBM traffic per step measured on this box, now: one `rocprofv3 --pmc`
    pass per counter (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE do not
    fit one pass) over a child run of this bench (--pmc-child) that performs
    exactly one step of the workload (incremental workloads: the base document
    alone is a second child, subtracted). Counts the engine's own kernels
    (crdtm::*) in KB per dispatch. Returns {kernel base name: [F, W] bytes per
    step}, or None when rocprofv3 is missing or a pass fails."""
    import csv
    import shutil
    import subprocess
    import tempfile
    from collections import defaultdict
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None
    modes = ["step", "base"] if args.workload in ("incr", "incr_cfg2") else ["step"]
    tot = {m: defaultdict(lambda: [0.0, 0.0]) for m in modes}
    env = dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp"))
    with tempfile.TemporaryDirectory() as td:
        for m in modes:
            for ci, ctr in enumerate(counters):
                d = os.path.join(td, f"{m}_{ctr}")
                cmd = ["timeout", "-s", "KILL", "150", prof, "--pmc", ctr, "-d", d, "-o", "run",
                       "--output-format", "csv", "--", sys.executable, os.path.abspath(__file__), "--workload",
                       args.workload, "--pmc-child", m]
                if args.n_ops:
                    cmd += ["--n-ops", str(args.n_ops)]
                if args.docs_per_gpu:
                    cmd += ["--docs-per-gpu", str(args.docs_per_gpu)]
                r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, env=env)
                f = os.path.join(d, "run_counter_collection.csv")
                if r.returncode != 0 or not os.path.exists(f):
                    return None
                for row in csv.DictReader(open(f)):
                    k = row["Kernel_Name"]
                    if "crdtm::" not in k:
                        continue
                    b = k.split("(")[0].replace("void ", "").split("<")[0].split("::")[-1]
                    tot[m][b][ci] += float(row["Counter_Value"]) * 1024.0
    out = dict(tot["step"])
    if "base" in tot:
        for b, v in tot["base"].items():
            e = out.setdefault(b, [0.0, 0.0])
            e[0] = max(0.0, e[0] - v[0])
            e[1] = max(0.0, e[1] - v[1])
        out = {b: v for b, v in out.items() if v[0] + v[1] > 0}
    return out


def roofline(workload, per_step, launches, B_alg, ms_step, steps_profiled, live=None):
    """SURVEY.md §8d roofline of the whole merge (one crdtm_apply / forest
    step): achieved = algorithmic bytes / merge time, against the 8 TB/s HBM
    peak; traffic = the merge's HBM bytes summed over its kernels' PMC counts
    (bytes per dispatch x dispatches per step). The dominant kernel (largest
    device-time share) is reported beside it with its own counter bandwidth."""
    pmc, src = pmc_table(workload)

    def kbytes(nm, key="hbm_bytes"):
        base = nm.strip("()").split("<")[0]
        # labelled scan phases (k_dscan_runs, k_dscan_xs, ...) are instances of
        # k_dscan, whose PMC entry is the dispatch-weighted mean over all of
        # them: summed over the step's dispatches it gives their exact total
        e = pmc.get(base) or (pmc.get("k_dscan") if base.startswith("k_dscan") else None)
        if e and key not in e and key == "hbm_bytes" and "hbm_bytes_corrected" in e:
            key = "hbm_bytes_corrected"  # (round-1 summaries)
        return None if not e or key not in e else e[key]

    merge_s = ms_step / 1e3
    achieved = B_alg / merge_s / 1e9
    if live:
        # measured in this run: [raw F + W, corrected 2F + W] per step (MI355X_MICROARCH.md: FETCH_SIZE
        # counts half the bytes of coalesced reads on gfx950; exact for streams, an upper bound for gathers)
        def step_bytes(nm, corrected=True):
            base = nm.strip("()").split("<")[0]
            if base.startswith("k_dscan"):
                return None  # (labelled scan phases share k_dscan's entry: reported in the total only)
            e = live.get(base)
            return None if e is None else (2 * e[0] + e[1] if corrected else e[0] + e[1])
        traffic = sum(2 * f + w for f, w in live.values())
        traffic_raw = sum(f + w for f, w in live.values())
        src = "live: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over one step of this workload (bench.py --pmc-child)"
        covered = True
        # the time share of the kernels whose counters the passes saw
        seen = sum(t for nm, t in per_step.items()
                   if nm.strip("()").split("<")[0] in live or nm.startswith("k_dscan"))
    else:
        def step_bytes(nm, corrected=True):
            b = kbytes(nm, "hbm_bytes" if corrected else "hbm_bytes_raw")
            return None if b is None else b * launches[nm] / steps_profiled
        traffic, traffic_raw, covered, seen = 0.0, 0.0, True, 0.0
        for nm, t in per_step.items():
            b, braw = step_bytes(nm), step_bytes(nm, False)
            if b is None or braw is None:
                covered = False
                continue
            traffic += b
            traffic_raw += braw
            seen += t
    kernels = []
    for nm, t in sorted(per_step.items(), key=lambda kv: -kv[1])[:8]:
        b = step_bytes(nm)
        per = launches[nm] / steps_profiled
        e = {"name": nm, "ms_per_step": t, "launches_per_step": per}
        if b is not None:
            e["hbm_bytes_per_step"] = b
            e["hbm_gbs"] = b / (t / 1e3) / 1e9
            e["hbm_frac"] = e["hbm_gbs"] / HBM_PEAK_GBS
        kernels.append(e)
    tot_ms = sum(per_step.values())
    have = bool(live) or bool(pmc)
    return {"bound": "hbm", "scope": "whole merge (every kernel of one step)", "achieved": achieved,
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
            "traffic": (traffic if have else None), "traffic_lower": (traffic_raw if have else None),
            "traffic_complete": covered, "traffic_time_share": (seen / tot_ms if tot_ms else None),
            "traffic_source": src, "traffic_over_alg": (traffic / B_alg if have else None),
            "alg_bytes": B_alg, "kernels_ms_per_step": tot_ms,
            "dominant_kernel": kernels[0] if kernels else None, "top_kernels": kernels}


def cpu_baseline(s, m, doc_off=None, workers=1, batch_cut=20_000, chunk_cut=200_000):
    """CPU baseline: the Elm-compiled-to-JS cost model —
    oracle/crdtree.js (persistent red-black Dicts, cons Lists; test
    infrastructure) run by `node` on this host, ops pre-decoded, timed around
    `apply` with process.hrtime. Value = `apply op` one op at a time over the
    first m ops (same final tree as one Batch, without the O(N^2)
    lastOperation accumulator); the reference's own `apply (Batch ops)` is
    timed beside it up to `batch_cut` ops. The C++ restatement
    (oracle/crdtree_oracle.cpp, mutable maps) is timed on the same sample."""
    import tempfile
    from oracle import jsoracle
    from oracle.oracle import lib as olib, _ptr
    sub = head(s, m) if doc_off is None else s
    out = {}
    with tempfile.TemporaryDirectory() as td:
        f = os.path.join(td, "batch.bin")
        jsoracle.write_batch(f, sub, m, doc_off=doc_off)
        # (progress on stderr: a silent minute reads as a hang to the GPU runner)
        print(f"[bench] cpu baseline: apply op over {m} ops", file=sys.stderr, flush=True)
        js = jsoracle.run(f, mode="op", workers=workers, timeout=900)
        out["js"] = js
        if doc_off is None and batch_cut:
            print(f"[bench] cpu baseline: apply (Batch ops) over {min(batch_cut, m)} ops", file=sys.stderr, flush=True)
            out["js_batch"] = jsoracle.run(f, mode="batch", limit=min(batch_cut, m), timeout=900)
        if doc_off is None:  # SURVEY.md 8d mode (ii): apply over 10k-op Batch chunks
            # (cut off at chunk_cut ops: ~9 s per 100k ops, each chunk's
            # lastOperation accumulator being quadratic in the chunk)
            print(f"[bench] cpu baseline: 10k-op Batch chunks over {min(chunk_cut, m)} ops", file=sys.stderr,
                  flush=True)
            out["js_chunk"] = jsoracle.run(f, mode="chunk", chunk=10_000, limit=min(chunk_cut, m), timeout=900)
    if doc_off is None:
        print(f"[bench] cpu baseline: C++ restatement over {m} ops", file=sys.stderr, flush=True)
        L = olib()
        t = L.orc_init(0)
        err = C.c_int64(-1)
        t0 = time.perf_counter()
        rc = L.orc_apply(t, 1, 0, m, _ptr(sub["kind"]), _ptr(sub["ts"]), _ptr(sub["path_off"]), _ptr(sub["path"]),
                         _ptr(sub["val"]), C.byref(err))
        out["cpp"] = (m / (time.perf_counter() - t0))
        L.orc_free(t)
        assert rc == 0
    return out


def cpu_flat_full(s, n):
    """The whole flat batch on one core: oracle/crdtree_oracle.cpp
    orc_flat_replay, the same findInsertion semantics with the stop node found
    through a treap over the list order instead of the literal walk (pinned
    against the literal walk and the general restatement by
    tests/test_oracle_flat.py), so all N ops finish in seconds."""
    from oracle.oracle import lib as olib, _ptr
    print(f"[bench] cpu baseline: C++ flat restatement over all {n} ops", file=sys.stderr, flush=True)
    h = np.zeros(2, np.uint64)
    w = np.zeros(2, np.uint64)
    err = C.c_int64(-1)
    na = C.c_uint64()
    t0 = time.perf_counter()
    rc = olib().orc_flat_replay(n, _ptr(s["kind"]), _ptr(s["ts"]), _ptr(s["path_off"]), _ptr(s["path"]),
                                _ptr(s["val"]), C.byref(err), _ptr(h), _ptr(w), C.byref(na))
    sec = time.perf_counter() - t0
    assert rc == 0 and na.value == n
    return {"value": n / sec, "unit": "ops/s", "cores": 1, "ops": n, "seconds": sec,
            "note": "oracle/crdtree_oracle.cpp orc_flat_replay over the whole batch: findInsertion's stop node "
                    "through a treap (O(log n) per op), one core"}


def cpu_line(cb, what):
    js = cb["js"]
    d = {"value": js["ops_per_s"], "unit": "ops/s", "cores": js["workers"], "kind": "port",
         "sample": f"{what}: oracle/crdtree.js (Elm-compiled-to-JS cost model: persistent RB Dicts, cons Lists), "
                   f"`apply op` per op, node {js['node']}, {js['workers']} worker(s) on {js['cpu_count']} x "
                   f"{js['cpu_model']}, --max-old-space-size {js['max_old_space_mb']} MB, {js['seconds']:.1f} s"}
    if "js_batch" in cb:
        b = cb["js_batch"]
        d["reference_batch_mode"] = {"value": b["ops_per_s"], "ops": b["ops"],
                                     "note": "apply (Batch ops) in one call: O(N^2) lastOperation accumulator "
                                             "(src/CRDTree.elm:224-232), cut off at this size"}
    if "js_chunk" in cb:
        c = cb["js_chunk"]
        d["chunked_batch_mode"] = {"value": c["ops_per_s"], "ops": c.get("ops"),
                                   "note": "apply (Batch chunk) over 10k-op chunks (same final tree; lastOperation "
                                           "= the last chunk), SURVEY.md 8d mode (ii)"}
    if "cpp" in cb:
        d["cpp_restatement"] = {"value": cb["cpp"], "note": "oracle/crdtree_oracle.cpp (mutable maps), same sample"}
    return d


def launch_ranks(n):
    """`bench.py --gpus N` without a launcher: start N ranks of this same
    command line under torch.distributed.run (one process per GPU, rendezvous
    on 127.0.0.1) as a child process and return its exit code. Runs before
    this process touches the GPU (no exec from a GPU-initialised process)."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def want_pmc(args, world):
    return args.pmc == "on" or (args.pmc == "auto" and world == 1 and not args.pmc_child)


def dry_run(args, rank, world):
    """--dry-run: the multi-rank plumbing of a real run on the CPU (gloo): the
    ranks the launcher started, the timing barrier and max over ranks, and the
    config-5 exchange (shard.Exchange all-to-all of the simulated replicas' op
    logs, then each rank's assembly of the documents it owns). No merge runs,
    so no throughput is claimed (`value` null)."""
    import torch
    import torch.distributed as dist
    from crdtm import _native as N
    from crdtm import shard
    if world > 1:
        dist.init_process_group("gloo")
    per, dpg = 100, 8
    n_docs = dpg * world
    s = N.synth(n_ops=per, n_docs=n_docs, replicas=TREES["replicas"], window=TREES["window"],
                p_delete=TREES["p_delete"], seed=TREES["seed"])
    doc_off = np.arange(n_docs + 1, dtype=np.uint32) * per
    local = torch.from_numpy(shard.local_log(s, doc_off, rank, world, TREES["replicas"]))
    modes = ["all_to_all", "all_gather"] if args.exchange_mode == "both" else [args.exchange_mode]
    n_mine = (n_docs - rank + world - 1) // world
    res = {}
    for md in modes:  # every mode must assemble exactly this rank's documents
        ex = shard.Exchange(local, mode=md if world > 1 else "auto")
        kept = 0
        for _ in range(args.warmup):
            ex.gather()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            _, my_off, keep = shard.assemble(ex.gather(), rank, world, n_docs, per)
            kept = int(keep.sum())
        if world > 1:
            dist.barrier()
        ok = kept == n_mine * per and int(my_off[-1]) == kept
        res[md] = (time.perf_counter() - t0, ok, ex)
    ex = res[modes[0]][2]
    t = torch.tensor([res[modes[0]][0], 0.0 if all(v[1] for v in res.values()) else 1.0], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        line = {"metric": "merged ops/sec (whole node) on 10M-op batch", "value": None, "unit": "ops/s",
                "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": float(t[0]) / max(1, args.steps) * 1e3, "higher_is_better": True, "scaling": "weak",
                "vs_baseline": None, "dtype": "int64", "data": "synthetic", "dry_run": True,
                "config": {"workload": "dry run (launcher and exchange plumbing, no merge)",
                           "parallelism": f"documents sharded by id over {world} rank(s) (gloo)"},
                "exchange": {"documents": n_docs, "records_per_rank_block": int(getattr(ex, "block", kept)),
                             "mode": ex.mode, "recv_bytes_per_rank": ex.recv_bytes,
                             "modes": {md: {"mode": v[2].mode, "recv_bytes_per_rank": v[2].recv_bytes,
                                            "assembled_ok": bool(v[1])} for md, v in res.items()},
                             "assembled_ok": bool(t[1] == 0)}}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if t[1] != 0:
        sys.exit(1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="flat10m", choices=sorted(WORKLOADS) + ["trees", "incr", "incr_cfg2"])
    ap.add_argument("--docs-per-gpu", type=int, default=0, help="trees workload: override documents per GPU")
    ap.add_argument("--n-ops", type=int, default=0, help="override the batch size (parity/debug only)")
    ap.add_argument("--cpu-sample", type=int, default=-1, help="oracle sample ops (0 = skip)")
    ap.add_argument("--profile-steps", type=int, default=3)
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--exchange", choices=("auto", "on", "off"), default="auto",
                    help="also run config 5 (op-log all-gather + sharded merge) after a single-document "
                         "workload and attach its line as 'exchange' (auto: when N > 1)")
    ap.add_argument("--exchange-mode", choices=("both", "all_to_all", "all_gather"), default="both",
                    help="config 5's op-log exchange at N > 1: all_to_all by document owner, north_star's "
                         "all_gather of every log, or both (the step timed with each; all_to_all is `value`)")
    ap.add_argument("--force-replay", action="store_true",
                    help="every merge takes the one-lane sequential replay (env CRDTM_FORCE_REPLAY=1): "
                         "measures the fallback cliff on the same batch")
    ap.add_argument("--pmc", choices=("auto", "on", "off"), default="auto",
                    help="measure HBM traffic per step live with rocprofv3 --pmc child passes (auto: 1 GPU)")
    ap.add_argument("--pmc-child", choices=("step", "base"), default=None, help=argparse.SUPPRESS)
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher plumbing only, no GPU: ranks (gloo), timing barrier, max over ranks and the "
                         "config-5 op-log exchange + assembly run; no merge is timed and `value` is null")
    args = ap.parse_args()
    if args.pmc_child:  # (a profiled child: one GPU, no launcher, no PMC of its own)
        args.gpus, args.pmc, args.exchange = 1, "off", "off"
    if args.force_replay:
        os.environ["CRDTM_FORCE_REPLAY"] = "1"  # (read by every merge)

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # self-launch: one child rank per GPU (before anything touches the GPU)
        sys.exit(launch_ranks(args.gpus))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but {world} rank(s) were launched", file=sys.stderr)
        sys.exit(2)
    import torch
    import torch.distributed as dist
    if args.dry_run:
        return dry_run(args, rank, world)
    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    # One explicit stream shared by torch and the engine (crdtm_ctx_create on
    # its handle): the default stream's handle is 0, which the C ABI reads as
    # "engine-owned stream" and which would not be ordered with torch's work.
    torch.cuda.set_stream(torch.cuda.Stream(device=local_rank))

    from crdtm import _native as N
    L = N.lib()
    if args.workload in ("trees", "incr", "incr_cfg2"):
        line = (run_trees if args.workload == "trees" else run_incr)(args, rank, world, local_rank)
        if rank == 0 and line is not None:
            print(json.dumps(line), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    spec = dict(WORKLOADS[args.workload])
    if args.n_ops:
        spec["n_ops"] = args.n_ops
    spec["seed"] = spec["seed"] + rank  # an independent document per rank
    s = N.synth(**spec)
    n = len(s["kind"])
    B_alg = alg_bytes(s)

    dev = torch.device("cuda", local_rank)
    tens = {k: torch.from_numpy(s[k]).to(dev) for k in ("kind", "ts", "path_off", "path", "val")}
    ops = N.Ops(n, int(s["path_off"][n]), tens["kind"].data_ptr(), tens["ts"].data_ptr(),
                tens["path_off"].data_ptr(), tens["path"].data_ptr(), tens["val"].data_ptr(), None)
    stream = torch.cuda.current_stream()
    ctx = C.c_void_p()
    N.check(L.crdtm_ctx_create(local_rank, C.c_void_p(stream.cuda_stream), C.byref(ctx)), "ctx")
    tree = C.c_void_p()
    N.check(L.crdtm_tree_create(ctx, 0, C.byref(tree)), "tree")
    res = N.Result()

    def step():
        N.check(L.crdtm_tree_reset(tree, 0), "reset")
        N.check(L.crdtm_apply(tree, C.byref(ops), 1, 1, None, C.byref(res)), "apply")
        if res.code != 0:
            raise RuntimeError(f"merge failed: code {res.code} at op {res.err_index}")

    if args.pmc_child:  # exactly one step under rocprofv3 --pmc (pmc_live)
        step()
        torch.cuda.synchronize()
        L.crdtm_tree_destroy(tree)
        L.crdtm_ctx_destroy(ctx)
        return

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    path_taken = res.path_taken
    guard = res.guard
    serial = {"ops": int(res.serial_ops), "dicts": int(res.serial_dicts), "largest": int(res.serial_max)}

    # Per-kernel device time (HIP events recorded on the launch stream) over a
    # few extra, untimed steps.
    L.crdtm_ctx_profile(ctx, 1)
    acc = {}
    for _ in range(max(1, args.profile_steps)):
        step()
        names = C.create_string_buffer(1 << 16)
        ms = (C.c_double * 512)()
        k = L.crdtm_ctx_phase_times(ctx, names, len(names), ms, 512)
        labels = names.raw.split(b"\0")
        for j in range(min(k, 512)):
            nm = labels[j].decode()
            acc.setdefault(nm, []).append(ms[j])
    L.crdtm_ctx_profile(ctx, 0)
    # guard G, measured by the per-dict
    # replay in one more untimed step: Adds whose walk met a Tombstone above
    # their timestamp, and the ops before each dict's first such Add (what a
    # closed-form prefix per dict could serve)
    guard_g = None
    if path_taken == 3:
        os.environ["CRDTM_GUARD_STATS"] = "1"
        step()
        del os.environ["CRDTM_GUARD_STATS"]
        gs = np.zeros(4, np.uint64)
        if L.crdtm_ctx_guard_stats(ctx, gs.ctypes.data_as(C.c_void_p)) == 1:
            walked, fail, prefix, nrep = (int(x) for x in gs)
            guard_g = {"adds_walked": walked, "adds_failing": fail, "failure_rate": fail / max(1, walked),
                       "ops_replayed": nrep, "closed_form_prefix_ops": prefix,
                       "closed_form_prefix_fraction": prefix / max(1, nrep),
                       "note": "an Add fails guard G when its findInsertion walk meets a Tombstone above its "
                               "timestamp; a dict's ops before its first failing Add are what a closed-form "
                               "prefix could serve (the rest needs the in-order replay)"}
    # a kernel launched several times per step is summed within the step
    ps = max(1, args.profile_steps)
    per_step = {nm: sum(v) / ps for nm, v in acc.items()}
    launches = {nm: len(v) for nm, v in acc.items()}

    ms_step = elapsed / args.steps * 1e3
    value = world * n * args.steps / elapsed
    # SURVEY.md 8d (config 2): how much of the merge ran as in-order replay, and its device-time share
    serial_ms = sum(v for nm, v in per_step.items() if nm.startswith(("k_pdr_small", "k_pdr_big", "k_pdr_huge",
                                                                        "k_pdr_blk", "k_replay")))
    serial_ms -= per_step.get("k_replay_index", 0.0)
    serial["time_share"] = serial_ms / max(1e-9, sum(per_step.values()))
    serial["fraction_of_ops"] = serial["ops"] / n
    line = {
        "metric": "merged ops/sec (whole node) on 10M-op batch",
        "value": value,
        "unit": "ops/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic (deterministic generator, SURVEY.md §8d)",
        "config": {"workload": f"{args.workload}: {n} ops per GPU, one document per GPU",
                   "replicas": spec.get("replicas"), "window": spec.get("window", 0),
                   "path": {1: "closed-form", 2: "replay", 3: "per-dict replay"}.get(path_taken, "?"),
                   "guard": guard, "serial_replay": serial, "guard_g": guard_g,
                   "parallelism": f"documents sharded by id over {world} GPU(s)"},
        "roofline": roofline(args.workload, per_step, launches, B_alg, ms_step, ps,
                             live=pmc_live(args) if (rank == 0 and want_pmc(args, world)) else None),
    }
    if rank == 0:
        sc = stream_copy_gbs(dev)
        line["roofline"]["stream_copy_gbs"] = sc
        line["roofline"]["frac_of_stream"] = line["roofline"]["achieved"] / sc
    if args.verbose and rank == 0:
        for nm, v in sorted(per_step.items(), key=lambda kv: -kv[1]):
            print(f"  {nm:28s} {v:9.3f} ms/step ({len(acc[nm]) // max(1, args.profile_steps)} launches)",
                  file=sys.stderr)
    if rank == 0 and world == 1:
        m = args.cpu_sample if args.cpu_sample >= 0 else CPU_SAMPLE[args.workload]
        if m > 0:
            m = min(m, n)
            line["cpu_baseline"] = cpu_line(cpu_baseline(s, m),
                                            f"first {m} ops of the same batch (cost grows with the batch)")
            if args.workload == "flat10m":
                line["cpu_baseline"]["cpp_flat_full_batch"] = cpu_flat_full(s, n)
    L.crdtm_tree_destroy(tree)
    L.crdtm_ctx_destroy(ctx)
    del tens
    # The single-document workloads exchange nothing between ranks; config 5 is
    # the path with the RCCL all-gather, so a multi-GPU run measures it too and
    # carries its line (same clocks, same contract) under "exchange".
    if args.exchange == "on" or (args.exchange == "auto" and world > 1):
        ex = run_trees(args, rank, world, local_rank, cpu=False)
        line["exchange"] = {k: ex[k] for k in ("metric", "value", "unit", "ms_per_step", "config")}
        line["exchange"]["roofline_frac"] = ex["roofline"]["frac"]
        line["exchange"]["all_gather_ms"] = ex["all_gather_ms"]  # (the exchange alone: all_to_all or all_gather)
        line["exchange"]["modes"] = ex["exchange_modes"]  # (each mode's whole step and exchange alone)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def run_incr(args, rank, world, local_rank):
    """Incremental merges (src/CRDTree.elm:265-269 on a tree that holds state):
    a 10M-node flat document (config 3's stream, merged untimed), then one
    step = 100 successive 10k-op batches of the same stream applied to it
    (incr_cfg2: a 900k-op config-2 document, nested with deletes, then 10
    successive 10k-op batches).
    Each step is bracketed by its own synchronisations; the base is rebuilt
    (reset + merge, untimed) between steps so every step sees the same
    document. Single document per rank (replicas only)."""
    import torch
    from crdtm import _native as N
    L = N.lib()
    nested = args.workload == "incr_cfg2"
    cfg = INCR_CFG2 if nested else INCR
    base, bsz, nb = cfg["base"], cfg["batch"], cfg["batches"]
    if args.n_ops:
        base = args.n_ops
    spec = dict(WORKLOADS["cfg2" if nested else "flat10m"])
    spec["n_ops"] = base + bsz * nb
    spec["seed"] = spec["seed"] + rank
    s = N.synth(**spec)
    n = len(s["kind"])
    assert n == base + bsz * nb and (nested or int(s["path_off"][n]) == n)  # flat: one path element per op
    dev = torch.device("cuda", local_rank)
    tens = {k: torch.from_numpy(s[k]).to(dev) for k in ("kind", "ts", "path", "val")}
    po = s["path_off"].astype(np.int64)
    offs = {}  # per (start, size): the path offsets rebased to 0 (device)

    def ops_at(a, m):
        if (a, m) not in offs:
            offs[a, m] = torch.from_numpy((po[a:a + m + 1] - po[a]).astype(np.uint32).view(np.int32)).to(dev)
        return N.Ops(m, int(po[a + m] - po[a]), tens["kind"].data_ptr() + a, tens["ts"].data_ptr() + 8 * a,
                     offs[a, m].data_ptr(), tens["path"].data_ptr() + 8 * int(po[a]), tens["val"].data_ptr() + 4 * a,
                     None)

    base_ops = ops_at(0, base)
    batches = [ops_at(base + j * bsz, bsz) for j in range(nb)]
    stream = torch.cuda.current_stream()
    ctx = C.c_void_p()
    N.check(L.crdtm_ctx_create(local_rank, C.c_void_p(stream.cuda_stream), C.byref(ctx)), "ctx")
    tree = C.c_void_p()
    N.check(L.crdtm_tree_create(ctx, 0, C.byref(tree)), "tree")
    res = N.Result()
    acct = {"remerge": 0, "incremental": 0, "dict_incr": 0, "paths": {}}

    def apply(o):
        N.check(L.crdtm_apply(tree, C.byref(o), 1, 1, None, C.byref(res)), "apply")
        if res.code != 0:
            raise RuntimeError(f"merge failed: code {res.code} at op {res.err_index}")

    def rebuild():
        N.check(L.crdtm_tree_reset(tree, 0), "reset")
        apply(base_ops)

    def step():
        for o in batches:
            apply(o)
            acct["remerge"] += bool(res.flags & N.FLAG_REMERGE)
            acct["incremental"] += bool(res.flags & N.FLAG_INCREMENTAL)
            acct["dict_incr"] += bool(res.flags & N.FLAG_DICT_INCR)
            acct["paths"][res.path_taken] = acct["paths"].get(res.path_taken, 0) + 1

    def canon(t_):
        out = []
        for which in (0, 1):
            nw, hh = C.c_uint64(), C.c_uint64()
            N.check(L.crdtm_tree_canonical(t_, which, None, 0, C.byref(nw), C.byref(hh)), "canonical")
            out.append((nw.value, hh.value))
        return out

    want = None
    if not args.pmc_child:  # the expected state: one fresh merge of base ++ batches
        fresh = C.c_void_p()
        N.check(L.crdtm_tree_create(ctx, 0, C.byref(fresh)), "tree")
        N.check(L.crdtm_apply(fresh, C.byref(ops_at(0, n)), 1, 1, None, C.byref(res)), "apply")
        if res.code != 0:
            raise RuntimeError(f"fresh merge failed: code {res.code} at op {res.err_index}")
        want = canon(fresh)
        L.crdtm_tree_destroy(fresh)
    check_each = os.environ.get("CRDTM_BENCH_CHECK_EACH") is not None  # (debug: every step's state)

    if args.pmc_child:  # the base document alone, or the base and one step (pmc_live subtracts)
        rebuild()
        if args.pmc_child == "step":
            step()
        torch.cuda.synchronize()
        L.crdtm_tree_destroy(tree)
        L.crdtm_ctx_destroy(ctx)
        return None
    for _ in range(args.warmup):
        rebuild()
        if check_each:
            print("base state", canon(tree), file=sys.stderr, flush=True)
        step()
        if check_each:
            print("warmup state", canon(tree) == want, canon(tree), want, file=sys.stderr, flush=True)
    elapsed = 0.0
    for _ in range(args.steps):
        rebuild()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step()
        torch.cuda.synchronize()
        elapsed += time.perf_counter() - t0
        if check_each:
            print("step state", canon(tree) == want, canon(tree), want, file=sys.stderr, flush=True)
    # per-kernel device time of one incremental batch (the last one of a step)
    rebuild()
    for o in batches[:-1]:
        apply(o)
    L.crdtm_ctx_profile(ctx, 1)
    apply(batches[-1])
    names = C.create_string_buffer(1 << 16)
    ms = (C.c_double * 512)()
    k = L.crdtm_ctx_phase_times(ctx, names, len(names), ms, 512)
    labels = names.raw.split(b"\0")
    L.crdtm_ctx_profile(ctx, 0)
    per_k, launches = {}, {}
    for j in range(min(k, 512)):
        nm = labels[j].decode()
        per_k[nm] = per_k.get(nm, 0.0) + ms[j]
        launches[nm] = launches.get(nm, 0) + 1
    # the state the batches built, against one fresh merge of base ++ batches
    # (the re-merge path): structure and visible document, hash and size
    verified = canon(tree) == want
    if not verified:
        raise RuntimeError(f"incremental state differs from the fresh merge of the same ops: {canon(tree)} {want}")
    ms_step = elapsed / args.steps * 1e3
    # SURVEY.md 8d algorithmic bytes of the step's nb batches (Add 49 + 8L, Delete 9 + 8L)
    a0 = base
    B_alg = alg_bytes({"kind": s["kind"][a0:], "path_off": s["path_off"][a0:]})
    # the kernels of the profiled batch (the step's last), times the batches of a step
    per_k = {k: v * nb for k, v in per_k.items()}
    launches = {k: v * nb for k, v in launches.items()}
    line = {
        "metric": "merged ops/sec (whole node) on 10M-op batch",
        "value": world * bsz * nb * args.steps / elapsed, "unit": "ops/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms_step, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "int64", "data": "synthetic (deterministic generator, SURVEY.md §8d)",
        "config": {"workload": (f"incr_cfg2: {nb} successive {bsz}-op batches into a {base}-op nested document "
                                f"with deletes (config 2 stream), per GPU") if nested else
                               (f"incr: {nb} successive {bsz}-op batches into a {base}-op flat document "
                                f"(config 3 stream), per GPU"),
                   "replicas": spec["replicas"], "window": spec["window"],
                   "batches_remerged": acct["remerge"], "batches_incremental": acct["incremental"],
                   "batches_level_replay": acct["dict_incr"],
                   "batches": nb * (args.steps + args.warmup),
                   "paths": {({1: "closed-form", 2: "replay", 3: "per-dict replay"}).get(p_, "?"): c_
                             for p_, c_ in acct["paths"].items()},
                   "ms_per_batch": ms_step / nb,
                   "verified": "final state == fresh merge of base ++ batches (structure + document hashes)",
                   "parallelism": f"one document per GPU ({world} GPU(s)), replicas only"},
        "roofline": roofline(args.workload, per_k, launches, B_alg, ms_step, 1,
                             live=pmc_live(args) if (rank == 0 and want_pmc(args, world)) else None),
    }
    line["roofline"]["note"] = ("per step (all its batches): achieved = the batches' algorithmic bytes / step "
                                "time; kernel times are the profiled last batch x batches per step")
    if rank == 0 and world == 1:
        m = args.cpu_sample if args.cpu_sample >= 0 else CPU_SAMPLE["cfg2" if nested else "flat10m"]
        if m > 0:
            line["cpu_baseline"] = cpu_line(cpu_baseline(s, min(m, n)),
                                            f"first {min(m, n)} ops of the same stream, one op at a time (a CPU "
                                            f"replica merges incrementally at this per-op cost or worse)")
    L.crdtm_tree_destroy(tree)
    L.crdtm_ctx_destroy(ctx)
    return line


def run_trees(args, rank, world, local_rank, cpu=True):
    """Config 5: the simulated replicas' op logs exchanged by document owner
    (RCCL all_to_all_single; document t -> rank t mod world), then every rank
    merges the documents it owns."""
    import torch
    import torch.distributed as dist
    from crdtm import _native as N
    from crdtm import shard
    L = N.lib()
    per = TREES["per_doc"]
    dpg = args.docs_per_gpu or TREES["docs_per_gpu"]
    n_docs = dpg * world
    dev = torch.device("cuda", local_rank)
    # this rank's replicas' op logs for every document (generated in chunks)
    logs = []
    chunk = 2000
    for d0 in range(0, n_docs, chunk):
        nd = min(chunk, n_docs - d0)
        s = N.synth(n_ops=per, n_docs=nd, replicas=TREES["replicas"], window=TREES["window"],
                    p_delete=TREES["p_delete"], seed=TREES["seed"], doc_base=d0)
        doc_off = np.arange(nd + 1, dtype=np.uint32) * per
        rec = shard.local_log(s, doc_off, rank, world, TREES["replicas"])
        rec[:, 0] += (np.int64(d0) << 32)  # global document id
        logs.append(rec)
    local = torch.from_numpy(np.concatenate(logs)).to(dev)
    del logs
    # records by owner rank (all_to_all; counts exchanged once; persistent buffers), or the all-gather
    primary = "all_gather" if args.exchange_mode == "all_gather" else ("auto" if world == 1 else "all_to_all")
    ex = shard.Exchange(local, mode=primary)
    ctx = C.c_void_p()
    stream = torch.cuda.current_stream()
    N.check(L.crdtm_ctx_create(local_rank, C.c_void_p(stream.cuda_stream), C.byref(ctx)), "ctx")
    n_mine = (n_docs - rank + world - 1) // world
    code = np.zeros(n_mine, np.int32)
    applied = np.zeros(n_mine, np.uint32)
    state = {}

    def step(ex=ex):
        allrec = ex.gather()
        ops_t, doc_off, _ = shard.assemble(allrec, rank, world, n_docs, per, ctx=ctx)
        n = int(doc_off[-1])
        ops = N.Ops(n, n, ops_t["kind"].data_ptr(), ops_t["ts"].data_ptr(), ops_t["path_off"].data_ptr(),
                    ops_t["path"].data_ptr(), ops_t["val"].data_ptr(), None)
        rc = L.crdtm_forest_apply(ctx, 0, C.byref(ops), doc_off.ctypes.data_as(C.c_void_p), n_mine, 1,
                                  code.ctypes.data_as(C.c_void_p), None, applied.ctypes.data_as(C.c_void_p),
                                  None, None, None)
        N.check(rc, "forest")
        state["ops_t"] = ops_t
        state["n"] = n

    if args.pmc_child:  # exactly one step under rocprofv3 --pmc (pmc_live)
        step()
        torch.cuda.synchronize()
        L.crdtm_ctx_destroy(ctx)
        return None
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    n = state["n"]
    ok_docs = int(np.sum(code == 0))
    if ok_docs != n_mine:  # every generated document merges; anything else is a regression
        raise RuntimeError(f"forest merge: {n_mine - ok_docs} of {n_mine} documents returned an error")
    # dominant kernel time (HIP events on the launch stream)
    L.crdtm_ctx_profile(ctx, 1)
    step()
    names = C.create_string_buffer(1 << 14)
    ms = (C.c_double * 64)()
    k = L.crdtm_ctx_phase_times(ctx, names, len(names), ms, 64)
    labels = names.raw.split(b"\0")
    L.crdtm_ctx_profile(ctx, 0)
    per_k, launches = {}, {}
    for j in range(min(k, 64)):
        nm = labels[j].decode()
        per_k[nm] = per_k.get(nm, 0.0) + ms[j]
        launches[nm] = launches.get(nm, 0) + 1
    # the all-gather alone (RCCL over xGMI), timed the same way
    ag_ms = 0.0
    if world > 1:
        torch.cuda.synchronize()
        dist.barrier()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            ex.gather()
        torch.cuda.synchronize()
        t = torch.tensor([time.perf_counter() - t1], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ag_ms = float(t.item()) / args.steps * 1e3
    # north_star's all-gather beside it: the whole step and the exchange alone, same clocks
    modes = {ex.mode: {"ms_per_step": elapsed / args.steps * 1e3, "exchange_ms": ag_ms,
                       "recv_bytes_per_rank": ex.recv_bytes}}
    if world > 1 and args.exchange_mode == "both":
        ex2 = shard.Exchange(local, mode="all_gather" if ex.mode == "all_to_all" else "all_to_all")
        for _ in range(args.warmup):
            step(ex2)
        torch.cuda.synchronize()
        dist.barrier()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            step(ex2)
        torch.cuda.synchronize()
        dist.barrier()
        e_step = time.perf_counter() - t1
        t1 = time.perf_counter()
        for _ in range(args.steps):
            ex2.gather()
        torch.cuda.synchronize()
        t = torch.tensor([e_step, time.perf_counter() - t1], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if int(np.sum(code == 0)) != n_mine:
            raise RuntimeError(f"forest merge ({ex2.mode} exchange): documents returned an error")
        modes[ex2.mode] = {"ms_per_step": float(t[0]) / args.steps * 1e3,
                           "exchange_ms": float(t[1]) / args.steps * 1e3, "recv_bytes_per_rank": ex2.recv_bytes}
        del ex2
    ot = state["ops_t"]
    kinds = ot["kind"][:n].cpu().numpy()
    B_alg = int(np.sum(np.where(kinds == 0, 57, 17)))  # flat documents: L = 1
    ms_step = elapsed / args.steps * 1e3
    line = {
        "metric": "merged ops/sec (whole node) on 10M-op batch",
        "value": world * n * args.steps / elapsed, "unit": "ops/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms_step, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "int64", "data": "synthetic (deterministic generator, SURVEY.md §8d)",
        "config": {"workload": f"trees: {n_mine} documents x {per} ops per GPU ({n} ops), {n_docs} documents total",
                   "replicas": TREES["replicas"], "documents_ok": ok_docs,
                   "parallelism": f"documents sharded by id over {world} GPU(s); op logs exchanged by owner "
                                  f"({ex.mode}, RCCL)",
                   "exchange_mode": ex.mode, "recv_bytes_per_rank": ex.recv_bytes,
                   "used_bytes_per_rank": int(n * shard.REC_W * 8)},
        "roofline": roofline("trees", per_k, launches, B_alg, ms_step, 1,
                             live=pmc_live(args) if (cpu and rank == 0 and want_pmc(args, world)) else None),
        "all_gather_ms": ag_ms,
        "exchange_modes": modes,
    }
    if args.verbose and rank == 0:
        for nm, v in sorted(per_k.items(), key=lambda kv: -kv[1])[:12]:
            print(f"  {nm:28s} {v:9.3f} ms", file=sys.stderr)
    if cpu and rank == 0 and world == 1:
        m = args.cpu_sample if args.cpu_sample >= 0 else CPU_SAMPLE["trees"]
        if m > 0:
            host = {k: v.cpu().numpy() for k, v in ot.items()}
            ndoc = max(1, min(n_mine, m // per))
            sub = dict(kind=host["kind"][:ndoc * per], ts=host["ts"][:ndoc * per],
                       val=host["val"][:ndoc * per].astype(np.uint32),
                       path_off=np.arange(ndoc * per + 1, dtype=np.uint32), path=host["path"][:ndoc * per])
            # (SURVEY.md 8d asks for os.cpus().length workers: on the GPU box
            # that reports the whole host, while a one-GPU job is given 16
            # cores; more threads than cores would time the same 16 cores)
            workers = min(16, os.cpu_count() or 1)
            cb = cpu_baseline(sub, ndoc * per, doc_off=np.arange(ndoc + 1, dtype=np.uint32) * per, workers=workers)
            line["cpu_baseline"] = cpu_line(cb, f"{ndoc} documents x {per} ops, documents round-robin over "
                                                f"worker_threads")
            line["cpu_baseline"]["workers_note"] = (
                f"{workers} worker_threads = the CPU share of a one-GPU job on this pool; os.cpus().length "
                f"reports the host's {os.cpu_count()} CPUs")
    L.crdtm_ctx_destroy(ctx)
    return line


if __name__ == "__main__":
    main()
