"""Debug: the incremental bench's shape (bench.py INCR_CFG2 by default) on
three trees — the default paths (level replay), the re-merge and the
sequential replay — compared batch by batch (structure and document hashes),
then against one fresh merge of everything.

    python tools/dbg/bench_shape.py [--base 900000] [--batch 10000] [--batches 10] [--seed 0xC0FFEE02]
"""
import argparse
import os
import sys

sys.path.insert(0, "crdt-graph_amd")
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import numpy as np  # noqa: E402
from crdtm import _native as N  # noqa: E402
from crdtm.tree import CRDTree  # noqa: E402
from test_gpu_incremental import sub  # noqa: E402


def canon(t):
    return tuple(t.canonical(w, full=False)[1:] for w in (0, 1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--base", type=int, default=900_000)
    ap.add_argument("--batch", type=int, default=10_000)
    ap.add_argument("--batches", type=int, default=10)
    ap.add_argument("--seed", type=lambda x: int(x, 0), default=0xC0FFEE02)
    ap.add_argument("--modes", default="auto,remerge,replay")
    a = ap.parse_args()
    s = N.synth(n_ops=a.base + a.batch * a.batches, replicas=16, window=64, p_delete=0.2, p_branch=0.1, max_depth=4,
                seed=a.seed)
    modes = a.modes.split(",")
    trees = {m: CRDTree.init(0) for m in modes}
    cuts = [0, a.base] + [a.base + a.batch * (j + 1) for j in range(a.batches)]
    for k, (x, y) in enumerate(zip(cuts[:-1], cuts[1:])):
        chunk = sub(s, x, y)
        out = {}
        for m in modes:
            if m == "auto":
                os.environ.pop("CRDTM_INCREMENTAL", None)
            else:
                os.environ["CRDTM_INCREMENTAL"] = m
            res = trees[m].apply_arrays(chunk, y - x)
            try:
                c = canon(trees[m])
            except Exception as e:  # noqa: BLE001
                c = repr(e)
            out[m] = (res.code, res.flags, res.path_taken, c)
        same = len({v[3] for v in out.values()}) == 1
        print(f"k={k} [{x},{y}) same={same} " + " ".join(f"{m}:{v[:3]}" for m, v in out.items()), flush=True)
        if not same:
            for m, v in out.items():
                print(f"   {m} {v[3]}", flush=True)
    os.environ.pop("CRDTM_INCREMENTAL", None)
    fresh = CRDTree.init(0)
    res = fresh.apply_arrays(sub(s, 0, cuts[-1]), cuts[-1])
    cf = canon(fresh)
    print("fresh", res.code, res.flags, cf, {m: canon(t) == cf for m, t in trees.items()}, flush=True)


if __name__ == "__main__":
    main()
