"""Debug: the incremental chain test's config-2-shaped stream under the level
replay, checked against the oracle after every batch; with `--variants`,
one child process per switch setting (CRDTM_ILR_OFF bits, snapshot off), to
bisect which lane shortcut breaks the state.

    python tools/dbg/c2chain.py [--variants] [--n 60000] [--seed 0xC0FFEE02]
"""
import argparse
import os
import subprocess
import sys

sys.path.insert(0, "crdt-graph_amd")
sys.path.insert(0, "tests")
sys.path.insert(0, ".")


def run_chain(n_ops, seed, stop_first=True):
    import numpy as np
    from crdtm import _native as N
    from crdtm.tree import CRDTree
    from parity_util import engine_summary, oracle_apply_arrays, oracle_summary
    from test_gpu_incremental import STREAMS, sub
    from oracle.oracle import lib as olib
    cfg = dict(STREAMS["config2_shape"], n_ops=n_ops, seed=seed)
    s = N.synth(**cfg)
    n = len(s["kind"])
    rng = np.random.default_rng(len("config2_shape"))
    cuts = [0, n // 2]
    while cuts[-1] < n:
        cuts.append(min(n, cuts[-1] + int(rng.choice([1, 7, 300, 2500, 6000]))))
    ot = olib().orc_init(0)
    et = CRDTree.init(0)
    bad = 0
    for k, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
        chunk = sub(s, a, b)
        oracle_apply_arrays(chunk, b - a, tree=ot)
        res = et.apply_arrays(chunk, b - a)
        try:
            es = engine_summary(et)
        except Exception as e:  # noqa: BLE001  (a state the read API refuses)
            es = repr(e)
        osum = oracle_summary(ot)
        ok = es == osum
        print(f"k={k} [{a},{b}) code={res.code} flags={res.flags} path={res.path_taken} ok={ok}", flush=True)
        if not ok:
            print("   engine", es if isinstance(es, str) else (es[0], es[1]), flush=True)
            print("   oracle", osum[0], osum[1], flush=True)
            bad += 1
            if stop_first:
                return k
    return -1 if not bad else bad


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", action="store_true")
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--n", type=int, default=60000)
    ap.add_argument("--seed", type=lambda x: int(x, 0), default=0xC0FFEE02)
    args = ap.parse_args()
    if args.sweep:  # the smallest failing stream: sizes x seeds, one child each
        for n in (1000, 2000, 4000, 8000, 16000):
            for seed in range(6):
                e = dict(os.environ, CRDTM_INCREMENTAL="ilr", CRDTM_STATE_DEBUG="1", CRDTM_ILR_DEBUG="1")
                print(f"=== n={n} seed={seed}", flush=True)
                p = subprocess.run([sys.executable, "-u", __file__, "--n", str(n), "--seed", str(seed)], env=e,
                                   timeout=240)
                print(f"=== n={n} seed={seed} exit {p.returncode}", flush=True)
                if p.returncode < 0 or p.returncode > 1:
                    return
        return
    if not args.variants:
        k = run_chain(args.n, args.seed)
        sys.exit(0 if k < 0 else 1)
    variants = [("base", {}), ("snap0", {"CRDTM_ILR_SNAPSHOT": "0"})]
    variants += [(f"off{b}", {"CRDTM_ILR_OFF": str(b)}) for b in (1, 2, 4, 8, 16, 31)]
    variants += [("off31_snap0", {"CRDTM_ILR_OFF": "31", "CRDTM_ILR_SNAPSHOT": "0"})]
    for name, env in variants:
        e = dict(os.environ, CRDTM_INCREMENTAL="ilr", **env)
        print(f"=== {name}", flush=True)
        p = subprocess.run([sys.executable, "-u", __file__, "--n", str(args.n), "--seed", hex(args.seed)], env=e,
                           timeout=240)
        print(f"=== {name} exit {p.returncode}", flush=True)
        if p.returncode < 0 or p.returncode > 1:
            break  # (a crash: nothing more on the GPU)


if __name__ == "__main__":
    main()
