#!/usr/bin/env python3
"""Summarise gpurun_out/pmc/<variant>_p*/run_counter_collection.csv for the trace kernels:
per-dispatch mean of each counter (summed over XCDs / instances)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
match = sys.argv[2] if len(sys.argv) > 2 else "trace_"
out = {}
for vdir in sorted(glob.glob(os.path.join(root, "v*_p*"))):
    tag = os.path.basename(vdir).split("_p")[0]
    f = os.path.join(vdir, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    per = defaultdict(lambda: defaultdict(float))
    for row in csv.DictReader(open(f)):
        if match not in row["Kernel_Name"]:
            continue
        per[row["Dispatch_Id"]][row["Counter_Name"]] += float(row["Counter_Value"])
    if not per:
        continue
    d = out.setdefault(tag, {})
    keys = set(k for v in per.values() for k in v)
    for k in keys:
        vals = [v[k] for v in per.values() if k in v]
        d[k] = sum(vals) / len(vals)
    d.setdefault("_dispatches", 0)
    d["_dispatches"] = max(d["_dispatches"], len(per))
print(json.dumps(out, indent=1, sort_keys=True))
