#!/usr/bin/env python3
"""Benchmark: ray-bounces/s of the full-colour waveguide bounce kernel on MI355X.

BASELINE.json metric: "ray-bounces/sec, full-color 21x21 FoV, num_rays_per_FoV=1024;
1/2/4/8 GPU".  A ray-bounce = 1 in-coupling event + 1 per executed iteration of the
reference's bounce loop (GRTF:860-905); counted on the device by the kernel itself.

One step = one trace of every ray of the batch = ONE launch of the reference's kernel
(gpu_ray_tracing_pro_fullColor.py:169-177 issues num_iter = 4 of them, each starting from
the RNG states the previous one left and adding its out-couplings to the eyebox grid).  The
headline ``value`` times K such steps as K separate launches (``num_iter = 1`` each, SURVEY.md
§8(d)), inputs already resident in HBM, plus the eyebox collective at N > 1.  More rates of the
same batch ride along: ``main_job`` -- the reference's job shape, 4 chained traces issued as one
call (the engine fuses them into one persistent launch, bit-identical to 4 launches) --,
``fused`` -- all K steps in one call -- and ``long_region`` -- the headline's single launches
over a timed region of at least LONG_STEPS steps (>= 50 ms; the driver's K = 20 gives a 5-ms region).

Workloads (``--config``, BASELINE.json configs, configs.py):
    C2  single-lambda 532 nm, 11x11 FoV, num_rays_per_FoV = 1024
    C3  full-colour 21x21 FoV x 3 lambda, num_rays_per_FoV = 1024 (the metric's workload)
    C4  full-colour 21x21 FoV x 3 lambda, num_rays_per_FoV = 4096
    C5  full-colour 41x41 FoV x 3 lambda, num_rays_per_FoV = 16384, deep-bounce stress (hops x 0.05)
    C5d the C5 batch on the design geometry (unscaled hops)
    auto (default) = C3: the metric's workload.
Multi-GPU: one process per GPU through distributed.py.
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
``--scaling strong`` (default): the metric's one batch split over the N ranks -- interleaved FoV x
wavelength blocks (BASELINE config 4's "FoV x lambda sharded"), each rank's eyebox slabs gathered to
rank 0 over RCCL -- so ``value`` is the batch's bounces over the slowest rank's time; at N = 8 a C3
batch is bound by its longest ray chains, not by the GPUs.  At N > 1 the line also
carries ``weak``: every rank tracing the whole batch as its own replica (global ray ids offset by
rank x batch) with one RCCL sum-reduce of the grid -- weak scaling, reported beside the metric's
curve, never as it.  ``--scaling weak`` makes the replicas the headline.  At N = 1 the line carries
``emulated_strong``: each of the N = 2 / 4 / 8 strong-scaling shards of C3 and C4 traced alone on
the one GPU (single launches, and the reference's 4-chained job per shard), i.e. the N-GPU step
time the curve should show before the collective.  ``--emulate-ranks N`` prints one such record.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

ALGO_BYTES_PER_BOUNCE = 72      # read + write of the minimal 36-B ray record
HBM_PEAK_GBPS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s
LIFETIME_BUCKETS = (1, 10, 30, 100, 300, 1000)   # bounce-count histogram edges (last bucket open)
LONG_STEPS = 200                # long_region: >= 50 ms of C3 single launches
EMULATE_STEPS = 20              # single launches per shard in the emulated_strong record
# emulated_strong: BASELINE configs 3 and 4, and config 5 on the design geometry (C5d) and as the
# short-hop stress batch (C5, fewer launches: 60 ms each on one GPU)
EMULATE_CONFIGS = (("C3", EMULATE_STEPS), ("C4", EMULATE_STEPS), ("C5d", EMULATE_STEPS), ("C5", 4))
FUSED_EMULATE = ("C3", "C4")    # emulated_strong also times the fused shape (the steps as one call) per shard
# the strong-scaling gather's transfer, modelled: every rank sends its payload (1/N of the eyebox grid) to
# rank 0 over its own xGMI link at the same time; one direction of a link carries half of the
# ~153.6 GB/s per-link figure of the node, and one RCCL gather call adds a fixed cost
XGMI_LINK_GBPS = 76.8
RCCL_CALL_MS = 0.03


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=LONG_STEPS)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="auto", choices=["auto", "C2", "C3", "C4", "C5", "C5d"])
    ap.add_argument("--lut-seed", type=int, default=0)
    ap.add_argument("--variant", type=int, default=0, help="kernel variant (include/wgrt.h); 0 auto")
    ap.add_argument("--scaling", default="strong", choices=["weak", "strong"],
                    help="N > 1: strong = the metric's batch split over the ranks (FoV x lambda blocks, eyebox "
                         "gather); weak = one replica of the batch per rank (global ids offset per rank), eyebox "
                         "sum-reduce")
    ap.add_argument("--assign", default="interleaved", choices=["interleaved", "contiguous"],
                    help="FoV x wavelength blocks per rank (distributed.rank_blocks)")
    ap.add_argument("--collective", default="gather", choices=["gather", "reduce"],
                    help="eyebox collection at N > 1: gather each rank's own slabs (1/N of the grid per rank) "
                         "or sum-reduce the whole grid")
    ap.add_argument("--emulate-ranks", type=int, default=0, metavar="N",
                    help="one GPU: time each of N ranks' shards in turn (predicted N-GPU step time)")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the main_job / fused / long_region / weak / emulated_strong records")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for N > 1 (nccl = RCCL over xGMI; gloo only to rehearse the "
                         "N > 1 path on a one-GPU box together with --one-device)")
    ap.add_argument("--one-device", action="store_true",
                    help="rehearsal: every rank uses cuda:0 (with --dist-backend gloo)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline sample length")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "traffic.json"),
                    help="PMC traffic per bounce (tools/pmc_traffic.py), used when its library hash matches")
    ap.add_argument("--pmc-json", default=os.path.join(REPO, "profiles", "pmc.json"),
                    help="PMC issue counters per bounce (tools/pmc_summary.py), used when its library hash matches")
    return ap.parse_args(argv)


def config_for(name: str, world: int):
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.configs import CONFIGS
    if name == "auto":
        name = "C3"
    return name, CONFIGS[name]


def lib_sha16() -> str:
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd._lib import loaded_path
    with open(loaded_path(), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def lifetime_histogram(per_ray) -> dict:
    """Per-ray bounce counts of one trace -> mean, max and counts per LIFETIME_BUCKETS bucket."""
    b = per_ray.cpu().numpy().view(np.uint32).astype(np.int64)
    edges = list(LIFETIME_BUCKETS) + [np.iinfo(np.int64).max]
    counts = {f"[{lo},{'inf' if hi == edges[-1] else hi})": int(((b >= lo) & (b < hi)).sum())
              for lo, hi in zip(edges[:-1], edges[1:])}
    return {"mean": round(float(b.mean()), 3) if b.size else 0.0, "max": int(b.max()) if b.size else 0,
            "rays": int(b.size), "by_bounces": counts}


def pmc_roofline(path: str, key: str, sha: str):
    """The issue-side (VALU) roofline of the trace kernel from a PMC summary of this build
    (tools/pmc_summary.py), or None when no summary matches the library hash."""
    try:
        with open(path) as f:
            ent = json.load(f).get(key)
    except (OSError, ValueError):
        return None
    if not ent or ent.get("lib_sha16") != sha:
        return None
    return {k: ent[k] for k in ("valu_busy_frac", "lanes_active_per_valu", "valu_per_bounce", "salu_per_bounce",
                                "vmem_per_bounce", "wait_any_frac", "effective_clock_ghz", "note") if k in ent}


def main(argv=None):
    a = parse(argv)
    import torch
    import torch.distributed as dist

    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.configs import build_inputs
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.distributed import (EyeboxGather, hip_shard_builder,
                                                                                hip_tracer, make_shard,
                                                                                reduce_eyebox, replica_shard,
                                                                                run_steps, split_calls, timed_run)
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.engine import (Scene, check_stats, new_stats, reserve,
                                                                           trace_fullcolor)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    if a.emulate_ranks and world != 1:
        raise SystemExit("--emulate-ranks runs on one GPU (WORLD_SIZE=1)")
    if a.one_device:
        if a.dist_backend != "gloo":
            raise SystemExit("--one-device needs --dist-backend gloo (RCCL refuses two ranks on one GPU)")
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    cname, w = config_for(a.config, world)
    nx, ny, lambdas, R = w.nx, w.ny, list(w.lambdas), w.R
    geom, luts, points = build_inputs(w, lut_seed=a.lut_seed)   # same on every rank (seeded)
    t_scene = time.perf_counter()
    scene = Scene.from_geometry(geom, luts, device=local)
    t_scene = time.perf_counter() - t_scene
    if a.emulate_ranks:
        rec = emulate_shards(scene, w, points, a.emulate_ranks, a.steps, a.warmup, dev, a.variant, a.assign)
        print(json.dumps({"emulated_ranks": a.emulate_ranks, "config": f"{cname}: {w.name}", "assign": a.assign,
                          **rec}), flush=True)
        scene.close()
        return
    weak = a.scaling == "weak"
    shard = (replica_shard(nx, ny, len(lambdas), R, world, rank) if weak else
             make_shard(nx, ny, len(lambdas), R, world, rank, a.assign))
    rays, rng = hip_shard_builder(points, nx, ny, lambdas, R, dev)(shard)
    eb = torch.zeros(scene.eb_shape(), dtype=torch.float32, device=dev)
    stats = new_stats(dev)
    tracer = hip_tracer(scene, a.variant, stats)
    reserve(scene, shard.n_rays, max(split_calls(max(a.steps, 4), 0)))
    if world > 1 and not weak and a.collective == "gather":
        all_blocks = [make_shard(nx, ny, len(lambdas), R, world, r, a.assign).blocks for r in range(world)]
        collect = EyeboxGather(all_blocks, nx, ny, lambdas, scene.num_lmd, device=dev)
    else:
        collect = reduce_eyebox

    def timed(steps, per_call, events=True, sh=None, r_=None, g_=None, coll=None):
        """steps chained traces as calls of per_call traces (distributed.timed_run: barrier, sync,
        trace, eyebox collective, sync, barrier; time MAX and bounces SUM over ranks); with events,
        HIP events around every call on the stream the kernels run on (torch's current stream)."""
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in split_calls(steps, per_call)] if events else []
        hook = (lambda j, what: ev[j][0 if what == "start" else 1].record()) if events else None
        elapsed, b_total, b_local = timed_run(tracer, r_ if r_ is not None else rays, g_ if g_ is not None else rng,
                                              eb, (sh or shard).gid, steps, per_call, stats,
                                              sync=torch.cuda.synchronize, hook=hook, collect=coll or collect)
        check_stats(stats)
        return elapsed, b_total, b_local, [s.elapsed_time(e) for s, e in ev]

    # warm-up: W separate launches (and one fused call, so the fused kernels are loaded too); the
    # first one records the per-ray lifetimes and the bounce kinds of a trace
    per_ray = torch.zeros(shard.n_rays, dtype=torch.int32, device=dev)
    kinds = None
    if shard.n_rays:
        g = shard.gid
        kw = dict(gid_offset=g.offset) if g.offset is not None else dict(
            gid_blocks=torch.as_tensor(g.block_gid, device=dev), gid_block_rays=R)
        st0 = new_stats(dev)
        trace_fullcolor(scene, rays, rng, eb, per_ray_bounces=per_ray, variant=a.variant, stats=st0, **kw)
        s0 = [int(v) for v in st0.cpu()]
        traced = shard.n_rays - s0[1]
        kinds = {"in_coupling": traced, "interactions": s0[5], "hops_switches_exits": s0[0] - traced - s0[5],
                 "note": "one trace's bounces by kind (wgrt_trace_stats): the in-coupling event of every ray "
                         "(GRTF:860-904), the loop iterations with a Monte-Carlo draw (coupler interactions), and "
                         "the iterations without one (miss hops, R3->R4 switches, terminations at GRTF:906 / "
                         "1244-1246)"}
    lifetimes = lifetime_histogram(per_ray)
    if kinds is not None:
        lifetimes["kinds"] = kinds
    run_steps(tracer, rays, rng, eb, shard.gid, max(a.warmup - 1, 0), 1)
    if not a.no_extras:
        run_steps(tracer, rays, rng, eb, shard.gid, 2, 0)
    if world > 1:
        # one untimed eyebox collective: RCCL sets up a collective's connections on its first call
        # of that size class, which would otherwise land in the first timed region
        collect(eb, None)
    torch.cuda.synchronize()
    # the headline: K separate launches with nothing else on the stream; then the same K launches
    # again with a HIP event pair around each, for the kernel duration the roofline divides by
    # (event records between the launches would be part of the timed steps otherwise)
    elapsed, bounces_total, bounces_local, _ = timed(a.steps, 1, events=False)
    value = bounces_total / elapsed
    _el, _bt, ev_bounces_local, call_ms = timed(a.steps, 1)
    binding = None
    if world == 1 and cname == "C3" and shard.n_rays and a.variant in (0, 7):
        binding = binding_record(scene, rays, rng, eb, shard, R, dev, lifetimes)
    extras = {}
    if not a.no_extras:
        for key, steps, note in (("main_job", 4, "the reference's job: 4 chained traces (MAIN:169-177) as one call, "
                                                 "fused into one persistent launch"),
                                 ("fused", a.steps, f"the same {a.steps} steps as one call (one persistent launch)")):
            e_el, e_b, e_bl, e_ms = timed(steps, 0)
            extras[key] = {"value": round(e_b / e_el, 1), "ms_per_step": round(e_el / steps * 1e3, 4),
                           "steps": steps, "kernel_avg_ms": round(float(np.mean(e_ms)), 4), "note": note}
        extras["region"] = region_cost(timed, call_ms, elapsed, _el, a.steps)
        if a.steps < LONG_STEPS:
            l_el, l_b, _, _ = timed(LONG_STEPS, 1, events=False)
            extras["long_region"] = {
                "value": round(l_b / l_el, 1), "ms_per_step": round(l_el / LONG_STEPS * 1e3, 4), "steps": LONG_STEPS,
                "timed_region_s": round(l_el, 4),
                "note": f"the headline's single launches timed over {LONG_STEPS} steps (the K-step region is "
                        f"{elapsed * 1e3:.1f} ms)"}
        if world > 1 and not weak:
            # weak scaling beside the metric's curve: every rank traces a replica of the whole batch
            wshard = replica_shard(nx, ny, len(lambdas), R, world, rank)
            wr, wg = hip_shard_builder(points, nx, ny, lambdas, R, dev)(wshard)
            reserve(scene, wshard.n_rays, 1)
            run_steps(tracer, wr, wg, eb, wshard.gid, 2, 1)
            reduce_eyebox(eb, None)
            w_el, w_b, _, _ = timed(a.steps, 1, events=False, sh=wshard, r_=wr, g_=wg, coll=reduce_eyebox)
            extras["weak"] = {
                "value": round(w_b / w_el, 1), "ms_per_step": round(w_el / a.steps * 1e3, 4), "steps": a.steps,
                "rays_total": w.n_rays * world, "scaling": "weak",
                "note": f"replicas: each of the {world} ranks traces the whole batch with its own global ray ids "
                        "(the batch tiled N times), one RCCL sum-reduce of the eyebox grid; per-GPU work fixed -- "
                        "not the metric's curve"}
            del wr, wg
    emulated = None
    if world == 1 and not a.no_extras and cname == "C3":
        emulated = emulated_strong(a, scene, dev)

    if rank == 0:
        kavg_s = float(np.mean(call_ms)) / 1e3
        bpl = ev_bounces_local / len(call_ms)
        achieved = bpl * ALGO_BYTES_PER_BOUNCE / kavg_s / 1e9
        sha = lib_sha16()
        traffic, traffic_raw, measured, traffic_note = None, None, None, "no PMC pass recorded for this library build"
        try:
            with open(a.traffic_json) as f:
                ent = json.load(f).get(f"{cname}:v{a.variant}")
            if ent and ent.get("lib_sha16") == sha:
                # MI355X_MICROARCH.md (HBM): on gfx950 FETCH_SIZE reports half the bytes of a read, so the
                # corrected fabric traffic is 2 x FETCH_SIZE + WRITE_SIZE; scaled to this launch's bounces
                scale = bpl / ent["bounces_per_launch"]
                traffic_raw = int(round((ent["fetch_bytes_per_launch"] + ent["write_bytes_per_launch"]) * scale))
                traffic = int(round((2 * ent["fetch_bytes_per_launch"] + ent["write_bytes_per_launch"]) * scale))
                measured = round(traffic / kavg_s / 1e9, 3)
                traffic_note = ("rocprofv3 PMC passes of the trace kernel on this build (tools/pmc_traffic.py): traffic "
                                "= 2 x FETCH_SIZE + WRITE_SIZE per launch (the guide's gfx950 correction of FETCH_SIZE; "
                                "L2 <-> fabric bytes, Infinity-Cache hits included, so an upper bound on HBM bytes), "
                                "traffic_raw = FETCH_SIZE + WRITE_SIZE; measured_gbps = traffic / launch_avg_ms.  The x2 "
                                "was calibrated in MI355X_MICROARCH.md on 16-B-per-lane streaming reads; this kernel's "
                                "bytes are mostly 4-B cell-word gathers and 16-B tile reads, for which it is "
                                "uncalibrated, so the true fabric traffic lies between traffic_raw and traffic")
        except (OSError, ValueError, KeyError):
            pass
        valu = pmc_roofline(a.pmc_json, f"{cname}:v{a.variant}", sha)
        roofline = {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBPS, 6), "traffic": traffic, "traffic_raw": traffic_raw,
                    "measured_gbps": measured,
                    "measured_frac": round(measured / HBM_PEAK_GBPS, 6) if measured is not None else None,
                    "traffic_note": traffic_note,
                    "kernel": kernel_name(a.variant, scene), "launch_avg_ms": round(kavg_s * 1e3, 4),
                    "evented_ms_per_step": round(_el / a.steps * 1e3, 4),
                    "algo_bytes_per_bounce": ALGO_BYTES_PER_BOUNCE,
                    "bounces_per_launch": int(round(bpl)),
                    "valu": valu if valu is not None else {
                        "note": "no PMC summary recorded for this library build (tools/pmc_summary.py)"},
                    "binding": binding,
                    "note": "achieved = algorithmic bytes (72 B x bounces) / launch_avg_ms; launch_avg_ms: HIP events "
                            "around each launch (a single launch is the trace kernel alone since round 6: its replay "
                            "runs inside it) on rank 0, in a "
                            "second pass of the same K launches (the timed steps carry no event records); valu: the "
                            "issue-side bound SURVEY.md §8(d) calls binding (VALU busy = SQ_ACTIVE_INST_VALU x 4 / "
                            "(GRBM_GUI_ACTIVE / 8 x 1024 SIMDs))"}
        cpu = None
        if world == 1 and not a.no_cpu_baseline:
            cpu = cpu_baseline(geom, luts, points, nx, ny, lambdas, R, a.cpu_seconds)
        par = (f"replicas x{world} (global ray ids offset per rank)" if weak else
               f"fov-lambda block shards x{world} ({a.assign})")
        if world > 1:
            coll = "gather of own eyebox slabs" if (a.collective == "gather" and not weak) else "reduce(EB)"
            par += (f" + RCCL {coll}" if a.dist_backend == "nccl" else
                    f" + gloo {coll}, rehearsal" + (" on one GPU" if a.one_device else ""))
        line = {
            "metric": w.metric(),
            "value": round(value, 1), "unit": "ray-bounces/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 4), "higher_is_better": True,
            "scaling": a.scaling, "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (seeded LUT and ray origins; geometry from the couplers_coor restatement)",
            "config": {"workload": f"{cname}: {w.name}", "nx": nx, "ny": ny, "lambdas": lambdas,
                       "num_rays_per_FoV": R, "rays_total": w.n_rays * (world if weak else 1),
                       "rays_rank0": shard.n_rays,
                       "lut": f"synthetic seed {a.lut_seed} profile {w.profile}", "gap_scale": w.gap_scale,
                       "parallelism": par, "kernel_variant": a.variant, "steps_per_launch": 1, "lib_sha16": sha,
                       "scene_create_s": round(t_scene, 3), "lifetimes_rank0": lifetimes,
                       "lut_staging": ("BASELINE config 3 names LUT tiles staged in LDS: built and measured "
                                       "slower (single launch +28-37 %, DESIGN.md §5.4), so the tiles are read "
                                       "through L1/L2 and what runs is not LDS-staged")},
            "roofline": roofline,
            "main_job": extras.get("main_job"),
            "fused": extras.get("fused"),
            "long_region": extras.get("long_region"),
            "region": extras.get("region"),
            "weak": extras.get("weak"),
            "emulated_strong": emulated,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    scene.close()
    if world > 1:
        dist.destroy_process_group()


def region_cost(timed, call_ms, elapsed, ev_elapsed, steps):
    """Where a short timed region's fixed cost goes: the region's wall time against
    K x the per-launch time, for regions of 1, 5, 20 and 200 single launches (a least-squares line:
    intercept = fixed cost per region, slope = per step), and inside the headline's evented pass the
    first launch's HIP-event time against the median launch's (the first launch of a region starts on an
    idle GPU after the barrier and synchronize)."""
    ks, ts = [], []
    for k in (1, 5, 20, 200):
        el, _, _, _ = timed(k, 1, events=False)
        ks.append(k)
        ts.append(el * 1e3)
    slope, icpt = np.polyfit(np.array(ks, float), np.array(ts, float), 1)
    med = float(np.median(call_ms))
    return {"regions_ms": {str(k): round(t, 4) for k, t in zip(ks, ts)},
            "fixed_ms_per_region": round(float(icpt), 4), "ms_per_step_fit": round(float(slope), 4),
            "first_launch_ms": round(float(call_ms[0]), 4), "median_launch_ms": round(med, 4),
            "first_minus_median_ms": round(float(call_ms[0]) - med, 4),
            "evented_wall_minus_launches_ms": round(ev_elapsed * 1e3 - float(np.sum(call_ms)), 4),
            "note": f"the headline's {steps}-step region carries the fixed cost once; the fit's slope is the "
                    "steady per-step time (the 200-step long_region's figure)"}


def binding_record(scene, rays, rng, eb, shard, R, dev, lifetimes):
    """What bounds the headline launch, measured on it: one more (untimed) launch of the same batch
    through the wave-timeline instantiation of the same trace kernel (wgrt_debug_opts.timeline): when
    the work queue ran dry, when the last wave ended, and the pass durations before and after.  The
    kernel is not bound by the HBM roof the north star names (``frac``): a launch is its bulk --
    every lane busy, paced by the CU's load path serving the lanes' dependent gathers -- plus the
    drain of its longest ray chains, each bounce a chain of dependent loads (cell word -> block
    line -> taken matrix) and ~600 instructions per wave pass."""
    import torch

    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.engine import timeline_summary, trace_fullcolor
    buf = torch.zeros(8 * 256 * 8 * 4 * 2, dtype=torch.int64, device=dev)
    g = shard.gid
    kw = dict(gid_offset=g.offset) if g.offset is not None else dict(gid_blocks=g.device_blocks(dev),
                                                                     gid_block_rays=R)
    trace_fullcolor(scene, rays, rng, eb, variant=7, debug=dict(timeline=buf), **kw)
    torch.cuda.synchronize()
    t = timeline_summary(buf)
    chain = lifetimes.get("max", 0) * t["drain_us_per_pass"]
    return {"limit": "dependent-gather chain: bulk paced by the CU load path, then the drain of the longest ray "
                     "chains", **t,
            "longest_ray_bounces": lifetimes.get("max"),
            "longest_chain_us_at_drain_pass": round(chain, 1),
            "note": "one untimed launch of the headline batch through the timeline instantiation of the trace "
                    "kernel (s_memrealtime per wave; the instrumented launch runs ~10 % slower): drain_frac = "
                    "(last wave end - median queue-dry time) / last wave end; the HBM frac above is the north "
                    "star's reporting roof, not the binding one"}


def emulate_shards(scene, w, points, N, steps, warmup, dev, variant=0, assign="interleaved", fused=False):
    """Each of the N strong-scaling shards of workload w (distributed.make_shard) traced alone on this
    GPU: ``steps`` single launches (HIP events around them) and 4-chained calls (the reference's
    job shape, MAIN:169-177, one persistent launch; the median of five); with ``fused``, also the bench's
    ``fused`` shape: the ``steps`` chained traces as ONE call (one persistent launch; the median of three).
    Returns the per-rank ms per step and the predicted N-GPU step time = the slowest shard's (the eyebox
    collective not included: see collective_cost)."""
    import torch

    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.distributed import (hip_shard_builder, hip_tracer,
                                                                                make_shard, run_steps)
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.engine import check_stats, new_stats, reserve
    nx, ny, lambdas, R = w.nx, w.ny, list(w.lambdas), w.R
    eb = torch.zeros(scene.eb_shape(), dtype=torch.float32, device=dev)
    stats = new_stats(dev)
    tracer = hip_tracer(scene, variant, stats)
    per_rank = []

    def ev_time(fn):
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        fn()
        t1.record()
        torch.cuda.synchronize()
        return t0.elapsed_time(t1)

    for r in range(N):
        shard = make_shard(nx, ny, len(lambdas), R, N, r, assign)
        rays, rng = hip_shard_builder(points, nx, ny, lambdas, R, dev)(shard)
        reserve(scene, shard.n_rays, max(4, steps if fused else 0))
        run_steps(tracer, rays, rng, eb, shard.gid, warmup, 1)
        run_steps(tracer, rays, rng, eb, shard.gid, 4, 0)
        torch.cuda.synchronize()
        stats.zero_()
        ms = ev_time(lambda: run_steps(tracer, rays, rng, eb, shard.gid, steps, 1)) / steps
        check_stats(stats)
        b = int(stats[0].item()) // steps
        # the median of five 4-chained calls: one call is a sub-millisecond region, and the prediction
        # takes the maximum over the shards, which a single slow call would set
        job = float(np.median([ev_time(lambda: run_steps(tracer, rays, rng, eb, shard.gid, 4, 0)) / 4
                               for _ in range(5)]))
        check_stats(stats)
        rec = {"rank": r, "rays": shard.n_rays, "ms_per_step": round(ms, 4), "job_ms_per_step": round(job, 4),
               "bounces_per_step": b}
        if fused:
            run_steps(tracer, rays, rng, eb, shard.gid, steps, 0)
            rec["fused_ms_per_step"] = round(float(np.median(
                [ev_time(lambda: run_steps(tracer, rays, rng, eb, shard.gid, steps, 0)) / steps for _ in range(3)])), 4)
            check_stats(stats)
        per_rank.append(rec)
        del rays, rng
    worst = max(p["ms_per_step"] for p in per_rank)
    worst_job = max(p["job_ms_per_step"] for p in per_rank)
    total = sum(p["bounces_per_step"] for p in per_rank)
    out = {"steps": steps, "per_rank": per_rank, "predicted_ms_per_step": worst,
           "predicted_value": round(total / (worst / 1e3), 1), "predicted_job_ms_per_step": worst_job,
           "predicted_job_value": round(total / (worst_job / 1e3), 1),
           "note": "each rank's shard timed alone on one MI355X; predicted N-GPU step = max over ranks, "
                   "without the eyebox collective"}
    if fused:
        worst_f = max(p["fused_ms_per_step"] for p in per_rank)
        out.update(predicted_fused_ms_per_step=worst_f, predicted_fused_value=round(total / (worst_f / 1e3), 1))
    return out


def collective_cost(scene, w, N, dev, assign="interleaved", reps=10):
    """The strong-scaling eyebox gather at N ranks (distributed.EyeboxGather) on this GPU: the device
    time of one rank's pack (the largest shard's) and of rank 0's assembly of all N payloads, with the
    reused buffers of the collective (HIP events, median of ``reps``), plus the modelled transfer
    (every rank's payload over its own xGMI link at once, XGMI_LINK_GBPS, plus RCCL_CALL_MS)."""
    import torch

    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.distributed import EyeboxGather, make_shard
    nx, ny, lambdas, R = w.nx, w.ny, list(w.lambdas), w.R
    blocks = [make_shard(nx, ny, len(lambdas), R, N, r, assign).blocks for r in range(N)]
    g = EyeboxGather(blocks, nx, ny, lambdas, scene.num_lmd, device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(N)
    eb = torch.randint(0, 4, scene.eb_shape(), generator=gen, device=dev).to(torch.float32)
    out = torch.empty_like(eb)
    send, recv = g.buffers(dev, eb.dtype, True)
    for r in range(N):
        g.pack(eb, r, out=recv[r])
    big = max(range(N), key=lambda r: g.counts[r])

    def med(fn):
        ts = []
        for _ in range(reps):
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record()
            fn()
            t1.record()
            torch.cuda.synchronize()
            ts.append(t0.elapsed_time(t1))
        return float(np.median(ts))

    fn_pack = lambda: g.pack(eb, big, out=send)
    fn_asm = lambda: g.assemble(out, recv)
    fn_pack()
    fn_asm()
    pack_ms, asm_ms = med(fn_pack), med(fn_asm)
    payload = g.payload_len * 4
    xfer_ms = payload / (XGMI_LINK_GBPS * 1e9) * 1e3 + RCCL_CALL_MS
    return {"pack_ms": round(pack_ms, 4), "assemble_ms": round(asm_ms, 4), "payload_bytes_per_rank": payload,
            "xfer_ms_modelled": round(xfer_ms, 4), "total_ms": round(pack_ms + asm_ms + xfer_ms, 4)}


def emulated_strong(a, scene, dev):
    """The N = 2 / 4 / 8 strong-scaling curve of EMULATE_CONFIGS predicted on one GPU: per N the
    slowest shard's ms per step (emulate_shards, the same event-timed method as the one-GPU
    baseline beside it) and the speedup over one GPU, for single launches and for the reference's
    4-chained job; then the same with the eyebox gather included (collective_cost, once per timed
    region of a.steps steps, and once per 4-trace job)."""
    import torch

    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.configs import CONFIGS, build_inputs
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.engine import Scene
    out = {}
    K = max(a.steps, 1)
    for cname, nsteps in EMULATE_CONFIGS:
        steps = min(a.steps, nsteps)
        w = CONFIGS[cname]
        geom, luts, points = build_inputs(w, lut_seed=a.lut_seed)
        sc = scene if cname == "C3" else Scene.from_geometry(geom, luts, device=dev.index or 0)
        fused = cname in FUSED_EMULATE
        whole = emulate_shards(sc, w, points, 1, steps, 2, dev, a.variant, a.assign, fused=fused)
        one, one_job = whole["predicted_ms_per_step"], whole["predicted_job_ms_per_step"]
        rec = {"one_gpu_ms_per_step": round(one, 4), "one_gpu_job_ms_per_step": one_job, "steps": steps}
        if fused:
            one_f = whole["predicted_fused_ms_per_step"]
            rec["one_gpu_fused_ms_per_step"] = one_f
        for n in (2, 4, 8):
            e = emulate_shards(sc, w, points, n, steps, 2, dev, a.variant, a.assign, fused=fused)
            c = collective_cost(sc, w, n, dev, a.assign)
            ms, job = e["predicted_ms_per_step"], e["predicted_job_ms_per_step"]
            ms_c, job_c = ms + c["total_ms"] / K, job + c["total_ms"] / 4
            rec[str(n)] = {"ms_per_step": ms, "speedup": round(one / ms, 3), "value": e["predicted_value"],
                           "job_ms_per_step": job, "job_speedup": round(one_job / job, 3),
                           "collective": c,
                           "with_collective": {"ms_per_step": round(ms_c, 4), "speedup": round(one / ms_c, 3),
                                               "job_ms_per_step": round(job_c, 4),
                                               "job_speedup": round(one_job / job_c, 3)}}
            if fused:
                # the fused shape: the steps chained traces as one call per rank, the gather once per call
                f = e["predicted_fused_ms_per_step"]
                f_c = f + c["total_ms"] / steps
                rec[str(n)].update(fused_ms_per_step=f, fused_speedup=round(one_f / f, 3))
                rec[str(n)]["with_collective"].update(fused_ms_per_step=round(f_c, 4),
                                                      fused_speedup=round(one_f / f_c, 3))
        if sc is not scene:
            sc.close()
        out[cname] = rec
        torch.cuda.synchronize()
    out["note"] = ("strong scaling predicted on one MI355X: each of the N interleaved FoV x lambda shards "
                   "(bench.py --gpus N --scaling strong) traced alone, the slowest one's step time (HIP events, "
                   "the same method for the one-GPU baseline); single launches and the reference's 4-chained job "
                   "per shard, and for C3 / C4 the fused shape (the steps chained traces as one call per rank; "
                   "fused_speedup against the one-GPU fused call timed the same way).  with_collective adds the "
                   "eyebox gather: pack and rank-0 assembly timed on this GPU, the transfer modelled at "
                   f"{XGMI_LINK_GBPS} GB/s per xGMI link plus {RCCL_CALL_MS} ms per call; once per timed region of "
                   f"{K} steps for single launches, once per 4-trace job, once per fused call")
    return out


def kernel_name(variant, scene):
    """Name of the kernel a single-trace launch runs (include/wgrt.h's variant table: auto = 7
    when the scene has <= 16 polygons, else 9)."""
    if variant == 0:
        variant = 7 if scene.info()["n_polygons"] <= 16 else 9
    return {1: "trace_grid_kernel", 7: "trace_jones_kernel<unsigned int, false, false, false>",
            9: "trace_jones_kernel<unsigned long, false, false, false>"}[variant]


def cpu_baseline(geom, luts, points, nx, ny, lambdas, R, target_s):
    """Time the CPU oracle (oracle/wgrt_oracle.c, float64, OpenMP) on a bounded sample of the
    same workload: successive slices of FoV x wavelength blocks (64 blocks each, wrapping
    around with chained RNG states) until ~target_s seconds of wall time have been spent."""
    from oracle import OracleScene
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.rays import build_rays, rng_seeds
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = min(threads, os.cpu_count() or threads)
    sc = OracleScene.from_geometry(geom, luts)
    nblk = nx * ny * len(lambdas)
    per = min(64, nblk)
    eb = np.zeros(sc.eb_shape(), np.float32)
    tot, dt, n_rays, k = 0, 0.0, 0, 0
    slices = {}
    while dt < target_s and k < 4096:
        lo = (k * per) % nblk
        hi = min(lo + per, nblk)
        if lo not in slices:
            slices[lo] = (build_rays(points, nx, ny, lambdas, R, blocks=(lo, hi)), rng_seeds((hi - lo) * R, lo * R))
        rays, rng = slices[lo]
        t = time.perf_counter()
        b, _ = sc.trace(rays, rng, eb, gid_offset=lo * R, threads=threads)
        dt += time.perf_counter() - t
        tot += b
        n_rays += (hi - lo) * R
        k += 1
    return {"value": round(tot / dt, 1), "unit": "ray-bounces/s", "cores": threads, "kind": "port",
            "sample": f"{k} traces of {per}-block slices ({n_rays} rays of {nblk} FoV x lambda blocks x {R}; "
                      f"{tot} bounces in {dt:.2f} s); oracle/wgrt_oracle.c float64 OpenMP, {threads} threads"}


if __name__ == "__main__":
    main()
