"""Merge freshly profiled PMC legs into a round's committed leg file.
tools/pmc_legs.sh <legs> writes only the legs it ran (gpurun_out/pmc_legs.json);
this folds them into profiles/<round>_pmc_legs.json (the bench reads the newest
such file) and writes the merged result back to gpurun_out/pmc_legs.json, which
tools/collect_profiles.sh copies into profiles/.
usage: python tools/pmc_merge.py profiles/r03_pmc_legs.json gpurun_out/pmc_legs.json"""
import json
import sys

base_path, new_path = sys.argv[1], sys.argv[2]
base = json.load(open(base_path))
new = json.load(open(new_path))
base.update(new)
for p in (base_path, new_path):
    with open(p, "w") as f:
        json.dump(base, f, indent=1)
print("merged legs:", ", ".join(sorted(new)))
