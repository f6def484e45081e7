"""Summarise rocprofv3 counter CSVs (mean per dispatch, per kernel)."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(os.path.join(root, "*", "*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        agg[(r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-60:], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print(f"{k:60s} {c:26s} n={len(v):3d} mean={sum(v) / len(v):.5e}")
