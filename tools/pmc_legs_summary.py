"""Summarise tools/pmc_legs.sh: for each leg, the per-dispatch average of
every counter of the leg's own kernel (tools/prof_leg.py LEGS), plus the
launch size, into one JSON (profiles/<round>_pmc_legs.json, read by bench.py)."""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_leg import LEGS  # noqa: E402

root, dst = sys.argv[1], sys.argv[2]
out = {}
for leg, (kernel, frames) in LEGS.items():
    counters = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(root, leg, "*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0]
            if name.endswith("wce::" + kernel) or name == "void wce::" + kernel:
                counters[r["Counter_Name"]].append(float(r["Counter_Value"]))
    if counters:
        out[leg] = {"kernel": kernel, "frames": frames, "dispatches": max(len(v) for v in counters.values()),
                    "counters": {c: sum(v) / len(v) for c, v in sorted(counters.items())}}
        print(leg, json.dumps({c: round(x, 1) for c, x in out[leg]["counters"].items()}))
json.dump(out, open(dst, "w"), indent=1)
