#!/usr/bin/env python3
"""Per-launch averages of every counter collected by tools/pmc.sh <tag>, for the
dominant kernel (name substring, default train_). usage: pmc_table.py <tag> [kernel_sub]"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
tag = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "train_"
vals = defaultdict(list)
for f in sorted((ROOT / "gpurun_out" / f"pmc_{tag}").glob("*/*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if sub in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {k: sum(v) / len(v) for k, v in sorted(vals.items())}
print(json.dumps(out, indent=1))
