"""Scratch check of the incremental flat closed form (incr.hip) on the GPU:
chains small flat batches into one tree and compares with the oracle after
each one, printing progress (tools/, not a test)."""
import sys, time
sys.path[:0] = ["crdt-graph_amd", "tests", "."]
import numpy as np
from crdtm import _native as N
from crdtm.tree import CRDTree
from parity_util import engine_summary, oracle_apply_arrays, oracle_summary, oracle_visible_vals
import ctypes as C
from oracle.oracle import lib as olib


def sub(s, a, b):
    off = s["path_off"]
    return dict(kind=s["kind"][a:b].copy(), ts=s["ts"][a:b].copy(), val=s["val"][a:b].copy(),
                path_off=(off[a:b + 1] - off[a]).astype(np.uint32), path=s["path"][off[a]:off[b]].copy())


s = N.synth(n_ops=60000, replicas=16, window=64, seed=31)
n = len(s["kind"])
cuts = [0, 1000, 1001, 1003, 1010, 1100, 1500, 2000, 3000, 30000, 30001, 30008, 30308, 32808, 38808, 44808]
ot = olib().orc_init(0)
et = CRDTree.init(0)
for k, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
    chunk = sub(s, a, b)
    _, rc, _ = oracle_apply_arrays(chunk, b - a, tree=ot)
    t0 = time.time()
    res = et.apply_arrays(chunk, b - a)
    print(k, a, b, "code", res.code, rc, "flags", res.flags, "t %.3f" % (time.time() - t0), flush=True)
    dh = et.document_handles()
    ov = oracle_visible_vals(ot)
    print("   doc", len(dh), len(ov), np.array_equal(dh, ov), flush=True)
    L = olib()
    h = C.c_uint64()
    nw = L.orc_canonical(ot, 0, None, 0, C.byref(h))
    _, enw, eh = et.canonical(0, full=False)
    print("   dict dump", (enw, eh) == (nw, h.value), flush=True)
    nw1 = L.orc_canonical(ot, 1, None, 0, C.byref(h))
    _, enw1, eh1 = et.canonical(1, full=False)
    print("   visible dump", (enw1, eh1) == (nw1, h.value), flush=True)
    print("   summary", engine_summary(et) == oracle_summary(ot), flush=True)
    if not np.array_equal(dh, ov):
        i = int(np.argmax(dh[:min(len(dh), len(ov))] != ov[:min(len(dh), len(ov))]))
        print("   first diff at", i, dh[max(0, i - 3):i + 5], ov[max(0, i - 3):i + 5], flush=True)
        break
