#!/usr/bin/env python3
"""HBM traffic of the bounce kernel from rocprofv3 PMC passes over bench.py.

Runs two separate counter passes (FETCH_SIZE, then WRITE_SIZE; --kernel-trace only, as
MI355X_MICROARCH.md's rocprofv3 section prescribes), averages each counter over the
dispatches of the kernel the bench line names (roofline.kernel) and writes {cfg_key: {...}}
JSON -- HBM bytes per bounce, which bench.py multiplies by its bounces per launch into
roofline.traffic (a fused launch covers several steps).  FETCH_SIZE / WRITE_SIZE are in KiB.  The gfx950 "x2" FETCH_SIZE
correction applies to 16-B/lane streaming reads; the kernel's reads are 4- and 8-B
per lane, for which the raw FETCH_SIZE matches the known input bytes (8 float32 columns +
uint32 RNG per ray), so the raw values are reported, with the x2 upper bound alongside.
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
for counter in ("FETCH_SIZE", "WRITE_SIZE"):
    d = tempfile.mkdtemp(prefix="pmc_", dir="/tmp")
    cmd = ["rocprofv3", "--kernel-trace", "--output-format", "csv", "-d", d, "-o", "run", "--pmc", counter,
           "--", sys.executable, os.path.join(repo, "bench.py"), "--no-cpu-baseline", "--steps", "3",
           "--warmup", "1", "--no-unfused", "--traffic-json", "/dev/null"] + bench_args
    r = subprocess.run(cmd, cwd="/tmp", capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        print(r.stdout[-2000:], r.stderr[-4000:])
        sys.exit(r.returncode)
    bench_line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    line = json.loads(bench_line[-1])
    res["cfg"] = line["config"]
    kname = line["roofline"]["kernel"]
    res["bounces_per_launch"] = line["roofline"]["bounces_per_launch"]
    res["kernel"] = kname
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if kname in row["Kernel_Name"] and row["Counter_Name"] == counter:
                vals[row["Dispatch_Id"]] = vals.get(row["Dispatch_Id"], 0.0) + float(row["Counter_Value"])
    res[counter] = sum(vals.values()) / max(len(vals), 1)
    res[counter + "_dispatches"] = len(vals)
fetch_b = res["FETCH_SIZE"] * 1024
write_b = res["WRITE_SIZE"] * 1024
cfg = res.get("cfg", {})
import argparse  # noqa: E402
ap = argparse.ArgumentParser()
ap.add_argument("--nx", type=int, default=21)
ap.add_argument("--ny", type=int, default=21)
ap.add_argument("--rays-per-fov", type=int, default=1024)
ap.add_argument("--lambdas", default="0,1,2")
ap.add_argument("--lut-profile", default="default")
ap.add_argument("--lut-seed", type=int, default=0)
ap.add_argument("--variant", type=int, default=0)
a, _ = ap.parse_known_args(bench_args)
key = f"{a.nx}x{a.ny}x{len(a.lambdas.split(','))}xR{a.rays_per_fov}:{a.lut_profile}:{a.lut_seed}:v{a.variant}"
entry = {"hbm_bytes_per_bounce": (fetch_b + write_b) / res["bounces_per_launch"], "kernel": res["kernel"],
         "bounces_per_launch": res["bounces_per_launch"],
         "hbm_bytes_per_launch": int(fetch_b + write_b), "fetch_bytes": int(fetch_b), "write_bytes": int(write_b),
         "fetch_bytes_x2_upper": int(2 * fetch_b + write_b), "dispatches": res["FETCH_SIZE_dispatches"],
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
