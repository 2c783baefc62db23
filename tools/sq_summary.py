#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counters per kernel (all dispatches) and print the
kernels whose name contains `pattern`.   python3 tools/sq_summary.py <dir> [pattern]"""
import csv
import os
import sys
from collections import defaultdict

d = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
agg = defaultdict(lambda: defaultdict(float))
for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(agg.items()):
    if pat in k:
        print(k, " ".join("%s=%.4g" % (c, x) for c, x in sorted(v.items())))
