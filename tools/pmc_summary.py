#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 --pmc CSVs (one pass per directory).

    python tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_sq [--json out.json]

FETCH_SIZE / WRITE_SIZE are in KB per dispatch. Calibration on this box
(tools/pmc_calibrate.hip -> profiles/r2_pmc_calibration.txt): coalesced reads
of 4, 8 and 16 B per lane count exactly half their bytes in FETCH_SIZE;
WRITE_SIZE counts writes exactly; a random 4 B gather counts 64 B per access,
which is the true transfer (half-line request) or half of it (full line). So
every kernel gets two figures: `raw_MB` = F + W (a lower bound of its HBM
bytes) and `hbm_MB` = 2F + W (exact for streaming reads, an upper bound for
gather-heavy kernels).
"""
import csv
import os
import sys
from collections import defaultdict


def load(d):
    f = os.path.join(d, "run_counter_collection.csv")
    rows = list(csv.DictReader(open(f)))
    out = defaultdict(lambda: defaultdict(list))
    meta = {}
    for r in rows:
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        out[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        meta[k] = (r["VGPR_Count"], r["LDS_Block_Size"], r["Scratch_Size"])
    return out, meta


def base_name(k):
    """crdtm::k_lc_contract<crdtm::FlatEulerSrc> -> k_lc_contract (the name bench.py's HIP-event marks use)."""
    return k.split("<")[0].split("::")[-1]


def main(args):
    out_json = None
    if "--json" in args:
        i = args.index("--json")
        out_json = args[i + 1]
        args = args[:i] + args[i + 2:]
    dirs = args
    agg = defaultdict(dict)
    meta = {}
    for d in dirs:
        data, m = load(d)
        meta.update(m)
        for k, cs in data.items():
            for c, v in cs.items():
                agg[k][c] = (sum(v) / len(v), len(v))
    cols = sorted({c for k in agg for c in agg[k]})
    print("kernel".ljust(40), "vgpr lds scr", " ".join(c[:14].rjust(14) for c in cols), "raw_MB".rjust(9),
          "hbm_MB".rjust(9))
    for k in sorted(agg, key=lambda k: -agg[k].get("FETCH_SIZE", (0, 0))[0] - agg[k].get("WRITE_SIZE", (0, 0))[0]):
        vals = " ".join(f"{agg[k][c][0]:14.1f}" if c in agg[k] else " " * 14 for c in cols)
        f = agg[k].get("FETCH_SIZE", (0, 0))[0]
        w = agg[k].get("WRITE_SIZE", (0, 0))[0]
        print(k[:40].ljust(40), " ".join(meta.get(k, ("?", "?", "?"))).ljust(12), vals, f"{(f + w) / 1024:9.1f}",
              f"{(2 * f + w) / 1024:9.1f}")
    if out_json:
        import json
        # template instances share the base name bench.py's HIP-event marks
        # use (k_dscan has five): merge them into per-dispatch averages
        # weighted by dispatches, so average x dispatches = their total
        tot = defaultdict(lambda: defaultdict(float))
        for k, cs in agg.items():
            b = base_name(k)
            nd = max(v[1] for v in cs.values())
            tot[b]["dispatches"] += nd
            for c, v in cs.items():
                tot[b][c] += v[0] * nd
        res = {}
        for b, t in tot.items():
            nd = t.pop("dispatches")
            e = {c: v / nd for c, v in t.items()}
            e["dispatches"] = int(nd)
            if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
                # bytes per dispatch: [raw, corrected] = [F + W, 2F + W] (see the module docstring)
                e["hbm_bytes"] = (2 * e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024
                e["hbm_bytes_raw"] = (e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024
            res[b] = e
        json.dump(res, open(out_json, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1:])
