#!/usr/bin/env python3
"""Benchmark: ray-bounces/s of the full-colour waveguide bounce kernel on MI355X.

BASELINE.json metric: "ray-bounces/sec, full-color 21x21 FoV, num_rays_per_FoV=1024;
1/2/4/8 GPU".  A ray-bounce = 1 in-coupling event + 1 per executed iteration of the
reference's bounce loop (GRTF:860-905); counted on the device by the kernel itself.

One step = one trace of every ray of the per-rank batch = one of the reference's
``num_iter`` chained launches (gpu_ray_tracing_pro_fullColor.py:169-177): each step starts
from the RNG states the previous one left and adds its out-couplings to the eyebox grid.
By default the K timed steps run as ONE fused launch (``num_iter = K``, wgrt_launch_opts):
every ray is traced K times in order inside one persistent kernel, so one step's straggler
tail overlaps the next step's bulk; results (RNG states, eyebox grid, bounce counts) are
bit-identical to K separate launches (tests/test_gpu_parity.py::test_fused_iterations_*).
``--fuse 1`` times K separate launches instead; the JSON line reports that rate too
(``unfused``).  At N > 1 the eyebox grid is RCCL-reduced to rank 0 after the steps.
Inputs (ray SoA, RNG, scene) are resident in HBM before timing starts.

Multi-GPU (weak scaling): the job at N GPUs traces num_rays_per_FoV = 1024 * N rays per
FoV x wavelength block and shards the blocks (contiguous global-ray ranges) over the
ranks, so every rank traces 21 x 21 x 3 x 1024 rays per step, with its global ray ids
(RNG seeds are global, results independent of N).  Launch:
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

ALGO_BYTES_PER_BOUNCE = 72      # read + write of the minimal 36-B ray record
HBM_PEAK_GBPS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s


def parse():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--nx", type=int, default=21)
    ap.add_argument("--ny", type=int, default=21)
    ap.add_argument("--rays-per-fov", type=int, default=1024, help="per GPU (weak scaling)")
    ap.add_argument("--lambdas", default="0,1,2")
    ap.add_argument("--lut-profile", default="default")
    ap.add_argument("--lut-seed", type=int, default=0)
    ap.add_argument("--variant", type=int, default=0, help="kernel variant (include/wgrt.h); 0 auto")
    ap.add_argument("--workgroups", type=int, default=0)
    ap.add_argument("--fuse", type=int, default=0,
                    help="steps per launch (0: all timed steps in one fused launch, at most 255)")
    ap.add_argument("--no-unfused", action="store_true", help="skip the separate-launch comparison")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline sample length")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "hbm_traffic.json"),
                    help="PMC-derived HBM bytes per launch (written by tools/pmc_traffic.py)")
    return ap.parse_args()


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.couplers_coor import design_geometry
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.distributed import block_range, reduce_eyebox
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.engine import (Scene, rays_to_device, reserve,
                                                                           trace_fullcolor)
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.luts import synthetic_luts
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.rays import (build_rays, generate_points_in_polygon,
                                                                         rng_seeds)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    lambdas = [int(v) for v in a.lambdas.split(",")]
    nx, ny = a.nx, a.ny
    R = a.rays_per_fov * world                 # global rays per FoV x lambda block
    nblk = nx * ny * len(lambdas)
    lo, hi = block_range(nblk, world, rank)
    geom = design_geometry(nx, ny)
    luts = synthetic_luts(geom, seed=a.lut_seed, profile=a.lut_profile)
    points = generate_points_in_polygon(geom.IC, R // 2, rng=np.random.default_rng(1))
    host_rays = build_rays(points, nx, ny, lambdas, R, blocks=(lo, hi))
    n_local = host_rays["x"].shape[0]
    gid0 = lo * R
    scene = Scene.from_geometry(geom, luts, device=local)
    rays = rays_to_device(host_rays, dev)
    seeds = rng_seeds(n_local, gid0)
    rng = torch.from_numpy(seeds.view(np.int32)).to(dev)
    eb = torch.zeros(scene.eb_shape(), dtype=torch.float32, device=dev)
    stats = torch.zeros(4, dtype=torch.int64, device=dev)

    def launches(steps, fuse):
        """split `steps` steps into launches of at most `fuse` steps (0: as few as possible)"""
        f = min(255, steps if fuse <= 0 else fuse)
        out = []
        while steps > 0:
            out.append(min(f, steps))
            steps -= out[-1]
        return out

    def run(steps, fuse, events=None):
        for j, k in enumerate(launches(steps, fuse)):
            if events is not None:
                events[j][0].record()
            trace_fullcolor(scene, rays, rng, eb, gid_offset=gid0, stats=stats, variant=a.variant,
                            workgroups=a.workgroups, num_iter=k)
            if events is not None:
                events[j][1].record()

    def timed(steps, fuse):
        stats.zero_()
        events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in launches(steps, fuse)]
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(steps, fuse, events)
        if world > 1:
            reduce_eyebox(eb)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        kern_ms = [s.elapsed_time(e) for s, e in events]
        bounces_local = int(stats[0].item())
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        b = torch.tensor([bounces_local], dtype=torch.int64, device=dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dist.all_reduce(b, op=dist.ReduceOp.SUM)
        return float(t.item()), int(b.item()), bounces_local, kern_ms

    # warm-up: W separate launches (the fused kernel then appears in a kernel trace only with
    # the timed launches, so its average duration there is the timed one), scratch reserved for
    # the timed launches' sizes
    reserve(scene, n_local, launches(a.steps, a.fuse)[0])
    run(a.warmup, 1)
    torch.cuda.synchronize()
    elapsed, bounces_total, bounces_local, kern_ms = timed(a.steps, a.fuse)
    value = bounces_total / elapsed
    unfused = None
    if not a.no_unfused and a.fuse != 1:
        u_el, u_b, _, u_ms = timed(a.steps, 1)
        unfused = {"value": round(u_b / u_el, 1), "ms_per_step": round(u_el / a.steps * 1e3, 4),
                   "kernel_avg_ms": round(float(np.mean(u_ms)), 4),
                   "note": "the same K steps as K separate launches (num_iter = 1 each)"}

    if rank == 0:
        steps_per_launch = launches(a.steps, a.fuse)[0]
        kavg_s = float(np.mean(kern_ms)) / 1e3
        bounces_per_launch_local = bounces_local / len(kern_ms)
        achieved = bounces_per_launch_local * ALGO_BYTES_PER_BOUNCE / kavg_s / 1e9
        cfg_key = f"{nx}x{ny}x{len(lambdas)}xR{a.rays_per_fov}:{a.lut_profile}:{a.lut_seed}:v{a.variant}"
        traffic = None
        try:
            with open(a.traffic_json) as f:
                per_bounce = json.load(f).get(cfg_key, {}).get("hbm_bytes_per_bounce")
            if per_bounce is not None:
                traffic = int(round(per_bounce * bounces_per_launch_local))
        except (OSError, ValueError):
            pass
        roofline = {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBPS, 6), "traffic": traffic,
                    "kernel": kernel_name(a.variant, scene, steps_per_launch > 1),
                    "kernel_avg_ms": round(kavg_s * 1e3, 4), "steps_per_launch": steps_per_launch,
                    "algo_bytes_per_bounce": ALGO_BYTES_PER_BOUNCE,
                    "bounces_per_launch": int(round(bounces_per_launch_local))}
        cpu = None
        if world == 1 and not a.no_cpu_baseline:
            cpu = cpu_baseline(geom, luts, points, nx, ny, lambdas, R, a.cpu_seconds)
        line = {
            "metric": "ray-bounces/sec, full-color 21x21 FoV, num_rays_per_FoV=1024",
            "value": round(value, 1), "unit": "ray-bounces/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": f"full-colour {nx}x{ny} FoV x {len(lambdas)} lambda, "
                                   f"num_rays_per_FoV={a.rays_per_fov} per GPU (BASELINE config 3)",
                       "nx": nx, "ny": ny, "lambdas": lambdas, "rays_per_fov_per_gpu": a.rays_per_fov,
                       "rays_per_gpu": n_local, "lut": f"synthetic seed {a.lut_seed} profile {a.lut_profile}",
                       "geometry": "couplers_coor_full_color restatement",
                       "parallelism": f"fov-lambda block shards x{world}" + (" + RCCL reduce(EB)" if world > 1 else ""),
                       "kernel_variant": a.variant,
                       "steps_per_launch": steps_per_launch},
            "roofline": roofline,
            "unfused": unfused,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def kernel_name(variant, scene, fused=False):
    """Name of the kernel a launch runs (wgrt_trace_fullcolor_ex's variant table; auto = 7
    when the scene has <= 16 polygons, else 9; a fused launch of variant 7 or 8 runs the
    fused variant-7 kernel)."""
    if variant == 0:
        variant = 7 if scene.info()["n_polygons"] <= 16 else 9
    if fused and variant >= 7:
        return "trace_jones_kernel<unsigned %s, 3, true>" % ("long" if variant == 9 else "int")
    return {1: "trace_grid_kernel", 2: "trace_persistent_kernel", 3: "trace_persistent_lds_kernel",
            4: "trace_persistent_g_kernel<unsigned long, 4>", 5: "trace_persistent_g_kernel<unsigned int, 3>",
            6: "trace_persistent_g_kernel<unsigned int, 4>", 7: "trace_jones_kernel<unsigned int, 3>",
            8: "trace_jones_kernel<unsigned int, 4>", 9: "trace_jones_kernel<unsigned long, 3>"}[variant]


def cpu_baseline(geom, luts, points, nx, ny, lambdas, R, target_s):
    """Time the CPU oracle (oracle/wgrt_oracle.c, float64, OpenMP) on the same workload:
    chained launches over the whole batch (like the reference's num_iter loop, MAIN:169)
    until ~target_s seconds of wall time have been spent."""
    from oracle import OracleScene
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.rays import build_rays, rng_seeds
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = min(threads, os.cpu_count() or threads)
    sc = OracleScene.from_geometry(geom, luts)
    nblk = nx * ny * len(lambdas)
    rays = build_rays(points, nx, ny, lambdas, R, blocks=(0, nblk))
    rng = rng_seeds(rays["x"].shape[0])
    eb = np.zeros(sc.eb_shape(), np.float32)
    tot, dt, launches = 0, 0.0, 0
    while dt < target_s and launches < 256:
        t = time.perf_counter()
        b, _ = sc.trace(rays, rng, eb, threads=threads)
        dt += time.perf_counter() - t
        tot += b
        launches += 1
    return {"value": round(tot / dt, 1), "unit": "ray-bounces/s", "cores": threads, "kind": "port",
            "sample": f"{launches} chained launches over the full batch ({nblk} FoV x lambda blocks x {R} rays; "
                      f"{tot} bounces in {dt:.2f} s); oracle/wgrt_oracle.c float64 OpenMP, {threads} threads"}


if __name__ == "__main__":
    main()
