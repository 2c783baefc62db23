#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 --pmc CSVs (one pass per directory).

    python tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_sq [--json out.json]

FETCH_SIZE / WRITE_SIZE are in KB per dispatch. On gfx950 FETCH_SIZE counts
half the bytes of wide coalesced streaming reads (MI355X_MICROARCH.md, HBM);
the `hbm_MB` column applies that x2 correction to FETCH_SIZE, so it is an
upper bound for kernels whose reads are not wide streams.
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
    print("kernel".ljust(40), "vgpr lds scr", " ".join(c[:14].rjust(14) for c in cols), "hbm_MB".rjust(9))
    for k in sorted(agg, key=lambda k: -agg[k].get("FETCH_SIZE", (0, 0))[0] - agg[k].get("WRITE_SIZE", (0, 0))[0]):
        vals = " ".join(f"{agg[k][c][0]:14.1f}" if c in agg[k] else " " * 14 for c in cols)
        f = agg[k].get("FETCH_SIZE", (0, 0))[0]
        w = agg[k].get("WRITE_SIZE", (0, 0))[0]
        print(k[:40].ljust(40), " ".join(meta.get(k, ("?", "?", "?"))).ljust(12), vals, f"{(2 * f + w) / 1024:9.1f}")
    if out_json:
        import json
        res = {}
        for k, cs in agg.items():
            b = base_name(k)
            e = {c: v[0] for c, v in cs.items()}
            e["dispatches"] = max(v[1] for v in cs.values())
            if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
                # bytes per dispatch; FETCH_SIZE doubled (gfx950 counts half of wide streaming reads)
                e["hbm_bytes_corrected"] = (2 * e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024
                e["hbm_bytes_raw"] = (e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024
            res.setdefault(b, e)
        json.dump(res, open(out_json, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1:])
