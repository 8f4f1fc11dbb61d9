#!/usr/bin/env python3
"""Summarise tools/pmc_passes.sh output: per counter, the mean over the trace kernel's dispatches
(the kernel the bench line's roofline.kernel names), plus derived per-bounce figures.
Usage: python tools/pmc_summary.py gpurun_out/<TAG>_pmc [OUT_JSON]"""
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
res, bpl, kname = {}, None, None
for d in sorted(glob.glob(os.path.join(root, "p*"))):
    log = open(os.path.join(d, "log.txt")).read().splitlines()
    lines = [l for l in log if l.startswith("{")]
    if not lines:
        continue
    line = json.loads(lines[-1])
    kname = line["roofline"]["kernel"]
    bpl = line["roofline"]["bounces_per_launch"]
    per = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if kname not in row["Kernel_Name"]:
                continue
            per.setdefault(row["Counter_Name"], {}).setdefault(row["Dispatch_Id"], 0.0)
            per[row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
    for c, v in per.items():
        res[c] = sum(v.values()) / len(v)
out = {"kernel": kname, "bounces_per_launch": bpl, "counters_per_dispatch": res}
g = res.get
if bpl:
    out["per_bounce"] = {k: g(k) / bpl for k in res if k.startswith("SQ_INSTS")}
if g("SQ_WAVE_CYCLES"):
    out["wait_any_frac"] = g("SQ_WAIT_ANY", 0) / g("SQ_WAVE_CYCLES")
    out["wait_inst_frac"] = g("SQ_WAIT_INST_ANY", 0) / g("SQ_WAVE_CYCLES")
    out["active_inst_frac"] = g("SQ_ACTIVE_INST_ANY", 0) / g("SQ_WAVE_CYCLES")
if g("SQ_ACTIVE_INST_VALU"):
    out["lanes_active_per_valu"] = g("SQ_THREAD_CYCLES_VALU", 0) / (64 * g("SQ_ACTIVE_INST_VALU"))
if g("TCC_HIT_sum") is not None and g("TCC_MISS_sum") is not None:
    out["l2_hit_rate"] = g("TCC_HIT_sum") / max(g("TCC_HIT_sum") + g("TCC_MISS_sum"), 1)
print(json.dumps(out, indent=1))
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)
