#!/usr/bin/env python3
"""Summarise tools/pmc_passes.sh output: per counter, the mean over the trace kernel's dispatches
(the kernel the bench line's roofline.kernel names), plus derived per-bounce figures.
With --merge PMC_JSON the issue-side roofline of this build is also recorded there under
"<config>:v<variant>" with the library hash, where bench.py reads it (roofline.valu):
  valu_busy_frac = SQ_ACTIVE_INST_VALU x 4 / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)   (quad-cycles;
                   GRBM_GUI_ACTIVE is summed over the 8 XCDs, MI355X_MICROARCH.md),
  lanes_active_per_valu = SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU),
  valu / salu / vmem wave-instructions per bounce.
Usage: python tools/pmc_summary.py gpurun_out/<TAG>_pmc [OUT_JSON] [--merge profiles/pmc.json]"""
import csv
import glob
import json
import os
import sys

args = [a for a in sys.argv[1:] if a != "--merge"]
merge = sys.argv[sys.argv.index("--merge") + 1] if "--merge" in sys.argv else None
if merge:
    args.remove(merge)
root = args[0]
res, bpl, kname, line, durs = {}, None, None, None, []
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
    # the trace kernel's own durations in this pass (kernel trace): the clock estimate's denominator
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if kname in row["Kernel_Name"]:
                durs.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
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
if g("SQ_ACTIVE_INST_VALU") and g("GRBM_GUI_ACTIVE"):
    out["valu_busy_frac"] = 4 * g("SQ_ACTIVE_INST_VALU") / (g("GRBM_GUI_ACTIVE") / 8 * 1024)
if durs:
    durs.sort()
    out["kernel_median_s_profiled"] = durs[len(durs) // 2]
    if g("GRBM_GUI_ACTIVE"):
        out["effective_clock_ghz"] = g("GRBM_GUI_ACTIVE") / 8 / out["kernel_median_s_profiled"] / 1e9
print(json.dumps(out, indent=1))
if len(args) > 1:
    json.dump(out, open(args[1], "w"), indent=1)
if merge and line:
    pb = out.get("per_bounce", {})
    key = f"{line['config']['workload'].split(':')[0]}:v{line['config']['kernel_variant']}"
    entry = {"lib_sha16": line["config"]["lib_sha16"], "kernel": kname,
             "valu_busy_frac": round(out.get("valu_busy_frac", float("nan")), 4),
             "lanes_active_per_valu": round(out.get("lanes_active_per_valu", float("nan")), 4),
             "valu_per_bounce": round(pb.get("SQ_INSTS_VALU", float("nan")), 3),
             "salu_per_bounce": round(pb.get("SQ_INSTS_SALU", float("nan")), 3),
             "vmem_per_bounce": round(pb.get("SQ_INSTS_VMEM_RD", 0.0) + pb.get("SQ_INSTS_VMEM_WR", 0.0), 3),
             "wait_any_frac": round(out.get("wait_any_frac", float("nan")), 4),
             "effective_clock_ghz": round(out.get("effective_clock_ghz", float("nan")), 3),
             "note": "rocprofv3 --pmc passes of the trace kernel on this build (tools/pmc_passes.sh); "
                     "valu_busy_frac = SQ_ACTIVE_INST_VALU x 4 / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs); "
                     "effective clock = GRBM_GUI_ACTIVE / 8 / the trace kernel's median duration in the profiled passes"}
    data = {}
    if os.path.exists(merge):
        try:
            data = json.load(open(merge))
        except ValueError:
            data = {}
    data[key] = entry
    json.dump(data, open(merge, "w"), indent=1)
    print(json.dumps({key: entry}))
