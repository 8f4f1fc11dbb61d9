#!/usr/bin/env python3
"""Fabric traffic of the trace kernel from rocprofv3 PMC passes over bench.py.

Two separate counter passes (FETCH_SIZE, then WRITE_SIZE; --kernel-trace only, one counter
group per run, as MI355X_MICROARCH.md's rocprofv3 section prescribes), each counter averaged
over the dispatches of the kernel the bench line names (roofline.kernel), written as bytes per
bounce under the key "<config>:v<variant>" together with the sha of the library measured, so
bench.py uses it only for that exact build.  FETCH_SIZE / WRITE_SIZE are KiB; they count L2 <->
fabric requests, Infinity-Cache hits included, so the figure bounds HBM bytes from above.  The
kernel's loads are 4- and 8-B gathers and 16-B ray-column reads, not the 16-B/lane streaming
reads the guide's x2 FETCH_SIZE correction is calibrated for: the raw value is reported, the
x2 figure alongside as an upper bound.
Usage: python tools/pmc_traffic.py OUT_JSON [bench args...]
"""
import csv
import glob
import json
import os
import subprocess
import sys
import tempfile

out_json = sys.argv[1]
bench_args = sys.argv[2:]
repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
res = {}
line = None
for counter in ("FETCH_SIZE", "WRITE_SIZE"):
    d = tempfile.mkdtemp(prefix="pmc_", dir="/tmp")
    cmd = ["rocprofv3", "--kernel-trace", "--output-format", "csv", "-d", d, "-o", "run", "--pmc", counter,
           "--", sys.executable, os.path.join(repo, "bench.py"), "--no-cpu-baseline", "--no-extras", "--steps", "5",
           "--warmup", "1", "--traffic-json", "/dev/null"] + bench_args
    r = subprocess.run(cmd, cwd="/tmp", capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        print(r.stdout[-2000:], r.stderr[-4000:])
        sys.exit(r.returncode)
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    kname = line["roofline"]["kernel"]
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if kname in row["Kernel_Name"] and row["Counter_Name"] == counter:
                vals[row["Dispatch_Id"]] = vals.get(row["Dispatch_Id"], 0.0) + float(row["Counter_Value"])
    res[counter] = sum(vals.values()) / max(len(vals), 1)
    res[counter + "_dispatches"] = len(vals)
fetch_b, write_b = res["FETCH_SIZE"] * 1024, res["WRITE_SIZE"] * 1024
bpl = line["roofline"]["bounces_per_launch"]
cname = line["config"]["workload"].split(":")[0]
key = f"{cname}:v{line['config']['kernel_variant']}"
entry = {"bytes_per_bounce": (fetch_b + write_b) / bpl, "kernel": line["roofline"]["kernel"],
         "lib_sha16": line["config"]["lib_sha16"], "bounces_per_launch": bpl,
         "fetch_bytes_per_launch": int(fetch_b), "write_bytes_per_launch": int(write_b),
         "fetch_x2_upper_bytes_per_launch": int(2 * fetch_b), "dispatches": res["FETCH_SIZE_dispatches"],
         "algo_bytes_per_launch": 72 * bpl,
         "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, mean over trace-kernel dispatches"}
data = {}
if os.path.exists(out_json):
    try:
        data = json.load(open(out_json))
    except ValueError:
        data = {}
data[key] = entry
json.dump(data, open(out_json, "w"), indent=1)
print(json.dumps({key: entry}))
