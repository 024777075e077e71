#!/usr/bin/env python3
"""Summarise gpurun_out/pmcK_*/run_counter_collection.csv: mean counter value
per (kernel, counter) over dispatches."""
import collections
import csv
import glob
import sys

rows = collections.defaultdict(list)
for f in sorted(glob.glob((sys.argv[1] if len(sys.argv) > 1 else "gpurun_out") + "/pmcK_*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        short = name.replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1][:40]
        rows[(short, r["Counter_Name"])].append(float(r["Counter_Value"]))
kern = collections.defaultdict(dict)
for (k, c), v in rows.items():
    kern[k][c] = sum(v) / len(v)
for k, cs in sorted(kern.items()):
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {v:16.0f}")
