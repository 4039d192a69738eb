"""Summarise rocprofv3 PMC passes (gpurun_out/pmc/*) per kernel, per dispatch."""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
out = collections.defaultdict(dict)
for d in sorted(glob.glob(os.path.join(root, "*", "run_counter_collection.csv"))):
    rows = list(csv.DictReader(open(d)))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        k = r["Kernel_Name"].split("(")[0]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        for c, x in v.items():
            out[k][c] = sum(x) / len(x)
for k, v in out.items():
    if "wce::" in k:
        print(k, json.dumps({c: round(x, 1) for c, x in sorted(v.items())}))
if len(sys.argv) > 2:
    json.dump({k: v for k, v in out.items() if "wce::" in k}, open(sys.argv[2], "w"), indent=1)
