"""Summarise rocprofv3 --pmc CSVs (gpurun_out/pmc/*/run_counter_collection.csv): per kernel,
the mean of each counter over its dispatches (dispatches after the first two, i.e. warm)."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        vals[short][(r["Counter_Name"], r["Dispatch_Id"])].append(float(r["Counter_Value"]))
for k, d in sorted(vals.items()):
    agg = defaultdict(list)
    for (cn, did), v in d.items():
        agg[cn].append(sum(v))  # sum over dimensions (XCD / SE instances)
    print(k)
    for cn in sorted(agg):
        xs = agg[cn][2:] or agg[cn]
        print("   %-28s %16.1f  (n=%d)" % (cn, sum(xs) / len(xs), len(xs)))
