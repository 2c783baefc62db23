"""Debug: the level replay over many stream shapes (depth, branching, deletes,
replicas, window), each chained against the oracle in chunks; prints the
shapes whose state differs.

    CRDTM_INCREMENTAL=ilr python tools/dbg/ilr_sweep.py [--n 6000] [--cases 48]
"""
import argparse
import sys

sys.path.insert(0, "crdt-graph_amd")
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import numpy as np  # noqa: E402
from crdtm import _native as N  # noqa: E402
from crdtm.tree import CRDTree  # noqa: E402
from parity_util import engine_summary, oracle_apply_arrays, oracle_summary  # noqa: E402
from test_gpu_incremental import sub  # noqa: E402


def chain(cfg, seed):
    from oracle.oracle import lib as olib
    s = N.synth(**cfg)
    n = len(s["kind"])
    rng = np.random.default_rng(seed)
    cuts = [0, n // 2]
    while cuts[-1] < n:
        cuts.append(min(n, cuts[-1] + int(rng.choice([1, 7, 300, n // 8, n // 4]))))
    ot = olib().orc_init(0)
    et = CRDTree.init(0)
    ilr = 0
    try:
        for k, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
            chunk = sub(s, a, b)
            _, rc, _ = oracle_apply_arrays(chunk, b - a, tree=ot)
            res = et.apply_arrays(chunk, b - a)
            ilr += bool(res.flags & N.FLAG_DICT_INCR)
            if res.code != rc:
                return f"k={k} code {res.code} vs {rc}", ilr
            try:
                es = engine_summary(et)
            except Exception as e:  # noqa: BLE001
                return f"k={k} {e!r}", ilr
            if es != oracle_summary(ot):
                return f"k={k} state differs", ilr
    finally:
        olib().orc_free(ot)
    return None, ilr


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=6000)
    ap.add_argument("--cases", type=int, default=48)
    ap.add_argument("--only", type=int, default=-1, help="run just this case")
    ap.add_argument("--rseed", type=int, default=1234, help="seed of the shape draws")
    a = ap.parse_args()
    rng = np.random.default_rng(a.rseed)
    bad = 0
    for c in range(a.cases):
        cfg = dict(n_ops=a.n, replicas=int(rng.choice([2, 4, 8, 16, 32])), window=int(rng.choice([4, 16, 64, 256])),
                   p_delete=float(rng.choice([0.05, 0.2, 0.4])), p_branch=float(rng.choice([0.05, 0.1, 0.3])),
                   max_depth=int(rng.choice([2, 3, 4, 6, 8])), seed=int(rng.integers(1 << 30)))
        if a.only >= 0 and c != a.only:
            continue
        why, ilr = chain(cfg, c)
        print(f"case {c} {cfg} ilr_batches={ilr} -> {why or 'ok'}", flush=True)
        bad += why is not None
    print(f"{bad} of {a.cases} cases differ", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
