#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 --pmc CSVs (one pass per directory).

    python tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_sq

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


def main(dirs):
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


if __name__ == "__main__":
    main(sys.argv[1:])
