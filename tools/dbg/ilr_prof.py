"""Debug: per-launch device times of incremental batches into a config-2 document (incr_cfg2 shape)."""
import ctypes as C
import os
import sys
sys.path.insert(0, "crdt-graph_amd")
sys.path.insert(0, ".")
import numpy as np
import torch
from crdtm import _native as N
import bench

L = N.lib()
spec = dict(bench.WORKLOADS["cfg2"])
base, bsz, nb = 900_000, 10_000, int(os.environ.get("NB", "4"))
spec["n_ops"] = base + bsz * nb
s = N.synth(**spec)
dev = torch.device("cuda", 0)
tens = {k: torch.from_numpy(s[k]).to(dev) for k in ("kind", "ts", "path", "val")}
po = s["path_off"].astype(np.int64)
keep = []


def ops_at(a, m):
    off = torch.from_numpy((po[a:a + m + 1] - po[a]).astype(np.uint32).view(np.int32)).to(dev)
    keep.append(off)
    return N.Ops(m, int(po[a + m] - po[a]), tens["kind"].data_ptr() + a, tens["ts"].data_ptr() + 8 * a,
                 off.data_ptr(), tens["path"].data_ptr() + 8 * int(po[a]), tens["val"].data_ptr() + 4 * a, None)


ctx = C.c_void_p()
N.check(L.crdtm_ctx_create(0, C.c_void_p(torch.cuda.current_stream().cuda_stream), C.byref(ctx)), "ctx")
tree = C.c_void_p()
N.check(L.crdtm_tree_create(ctx, 0, C.byref(tree)), "tree")
res = N.Result()
N.check(L.crdtm_apply(tree, C.byref(ops_at(0, base)), 1, 1, None, C.byref(res)), "base")
for j in range(nb):
    o = ops_at(base + j * bsz, bsz)
    L.crdtm_ctx_profile(ctx, 1)
    N.check(L.crdtm_apply(tree, C.byref(o), 1, 1, None, C.byref(res)), "apply")
    names = C.create_string_buffer(1 << 16)
    ms = (C.c_double * 1024)()
    k = L.crdtm_ctx_phase_times(ctx, names, len(names), ms, 1024)
    labels = names.raw.split(b"\0")
    L.crdtm_ctx_profile(ctx, 0)
    tot = sum(ms[q] for q in range(min(k, 1024)))
    print(f"batch {j}: path {res.path_taken} flags {res.flags} code {res.code} kernels {k} total {tot:.3f} ms", flush=True)
    agg = {}
    for q in range(min(k, 1024)):
        nm = labels[q].decode()
        if nm.startswith("k_ilr_level") or nm.startswith("k_ilr_prep") or ms[q] > 0.05:
            print(f"   {q:3d} {nm:28s} {ms[q]*1e3:9.1f} us")
        agg[nm] = agg.get(nm, 0.0) + ms[q]
    top = sorted(agg.items(), key=lambda x: -x[1])[:8]
    print("   top:", ", ".join(f"{a} {b*1e3:.0f}us" for a, b in top), flush=True)
