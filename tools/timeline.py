#!/usr/bin/env python3
"""One merge step's kernel timeline from a rocprofv3 --kernel-trace CSV:
start, gap since the previous kernel ended, duration, name. Steps are
delimited by `marker` (the first kernel of a merge); the `which`-th from the
end is printed (-2 = the last complete step).

    python3 tools/timeline.py <run_kernel_trace.csv> [marker] [which]
"""
import csv
import sys


def main(path, marker="k_dres_init", which=-2):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    step = rows[idx[which]:idx[which + 1]] if which + 1 < 0 else rows[idx[which]:]
    t0 = prev = int(step[0]["Start_Timestamp"])
    busy = 0
    for r in step:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy += e - s
        print("%8.1f gap %7.1f dur %7.1f  %s" % ((s - t0) / 1e3, (s - prev) / 1e3, (e - s) / 1e3,
                                               r["Kernel_Name"].split("(")[0][:70]))
        prev = e
    print("step %.1f us, kernels busy %.1f us, %d kernels" % ((prev - t0) / 1e3, busy / 1e3, len(step)))


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], *(a[1:2]), *([int(a[2])] if len(a) > 2 else []))
