"""Full-colour driver (reference ``gpu_ray_tracing_pro_fullColor.py``, MAIN:1-210).

Same flow as the reference script, on the MI355X kernel:

1. coupler geometry (``couplers_coor_full_color``, MAIN:19-25);
2. the seven RCWA LUTs -- the reference's ``.npy`` files when ``lut_dir`` is given
   (MAIN:28-34), otherwise the seeded synthetic set (the files are not available offline);
3. ray batch: ``num_rays_per_FoV / 2`` in-coupler origins shared by every FoV x wavelength
   block, TE then TM halves (MAIN:59-115), RNG seeds ``0x9E3779B9 * (gid + 1)`` (MAIN:158),
   laid out on the device by ``wgrt_rays_init``;
4. ``num_iter`` chained launches of the bounce kernel (MAIN:169-177), as one fused call
   (``num_iter`` traces per ray in one persistent launch; identical results) when a GPU traces
   at most ``FUSE_MAX_RAYS`` rays, else as separate launches (``fuse`` overrides), timed with HIP
   events (no JIT in the timed region, unlike the reference's wall clock);
5. efficiencies ``A = sum(EB) / N / num_iter``, ``eff_c = 3 * sum(A[lambda])`` (MAIN:186-192)
   and ``evaluation(EB / R / num_iter)`` (MAIN:197-198).

Plots and the PNG export (MAIN:199-237) are visual-only and not reproduced.
Multi-GPU: run under ``torch.distributed.run``; each rank traces an interleaved set of FoV x
wavelength blocks and the eyebox slabs are gathered to rank 0 (``distributed.py``).
"""
from __future__ import annotations

import argparse
import json
import os
import time

import numpy as np


# Fusing the num_iter chained traces into one persistent launch overlaps each trace's tail with
# the next one's bulk: 1.5x faster at 1.35M rays per GPU (C3), even at 5.4M (C4), and 13 % slower
# at 82.6M (C5, where the tail is a small part of a launch and the fused kernel runs one wave per
# SIMD fewer).  fuse=None picks by the rays per GPU.
FUSE_MAX_RAYS = 4_000_000


def run(num_FOV_x: int = 100, num_FOV_y: int = 75, num_rays_per_FoV: int = 5000, num_iter: int = 4,
        lambdas=(0, 1, 2), lut_dir: str | None = None, lut_seed: int = 0, lut_profile: str = "default",
        point_seed: int | None = None, evaluate: bool = True, verbose: bool = True, variant: int = 0,
        fuse: bool | None = None) -> dict:
    import torch
    import torch.distributed as dist

    from .couplers_coor import design_geometry
    from .distributed import EyeboxGather, hip_shard_builder, hip_tracer, make_shard, run_steps, split_calls
    from .engine import Scene, check_stats, new_stats, reserve
    from .luts import load_luts, lut_f32_mask, synthetic_luts, validate_luts
    from .rays import generate_points_in_polygon

    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    dev = torch.device("cuda", torch.cuda.current_device())
    say = (lambda *a: print(*a, flush=True)) if (verbose and rank == 0) else (lambda *a: None)

    say("=" * 60 + "\nInitializing system components ...\n" + "=" * 60)
    geom = design_geometry(num_FOV_x, num_FOV_y)
    f32_angles = 0
    if lut_dir:
        raw = load_luts(lut_dir)
        f32_angles = lut_f32_mask(raw)   # complex64 files: float32 cosines, as the compiled reference
        luts = validate_luts(raw, len(geom.lmd), num_FOV_x, num_FOV_y, geom.num_fc_slices, geom.num_oc_slices)
    else:
        luts = synthetic_luts(geom, seed=lut_seed, profile=lut_profile)
    scene = Scene.from_geometry(geom, luts, device=dev.index, lut_f32_angles=f32_angles)
    R = int(num_rays_per_FoV)
    rng_pts = np.random.default_rng(point_seed) if point_seed is not None else None
    points = generate_points_in_polygon(geom.IC, R // 2, rng=rng_pts)
    if world > 1:  # every rank must use the same origins
        t = torch.from_numpy(np.ascontiguousarray(points)).to(dev)
        dist.broadcast(t, src=0)
        points = t.cpu().numpy()
    shard = make_shard(num_FOV_x, num_FOV_y, len(lambdas), R, world, rank)
    # ray columns and RNG seeds built on the device (MAIN:59-158 without the host arrays:
    # 48 B x N of host memory and its upload at the reference's 100 x 75 x 3 x 5000 default)
    rays, rng = hip_shard_builder(points, num_FOV_x, num_FOV_y, lambdas, R, dev)(shard)
    eb = torch.zeros(scene.eb_shape(), dtype=torch.float32, device=dev)
    stats = new_stats(dev)
    num_rays = num_FOV_x * num_FOV_y * len(lambdas) * R
    say(f"Initialization complete: {num_rays:,} rays, {world} GPU(s)\n" + "=" * 60 + "\nSTART GPU RAY TRACING\n" + "=" * 60)

    # the num_iter chained launches of MAIN:169-177; fuse: as one call (wgrt_launch_opts.num_iter,
    # one persistent launch for the Jones-vector variants), with results identical to num_iter calls
    if fuse is None:
        fuse = shard.n_rays <= FUSE_MAX_RAYS
    per_call = 0 if fuse else 1
    calls = split_calls(num_iter, per_call)
    if shard.n_rays and calls:
        reserve(scene, shard.n_rays, max(calls))
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    if shard.n_rays:
        run_steps(hip_tracer(scene, variant, stats), rays, rng, eb, shard.gid, num_iter, per_call)
    t1.record()
    torch.cuda.synchronize()
    kern_s = t0.elapsed_time(t1) / 1e3
    check_stats(stats)
    if world > 1:
        all_blocks = [make_shard(num_FOV_x, num_FOV_y, len(lambdas), R, world, r).blocks for r in range(world)]
        EyeboxGather(all_blocks, num_FOV_x, num_FOV_y, lambdas, scene.num_lmd, device=dev)(eb)
    if world > 1:
        dist.all_reduce(stats)
    matrix_EB = eb.cpu().numpy()
    out = dict(num_rays=num_rays, num_iter=num_iter, gpu_seconds=kern_s, bounces=int(stats[0]),
               eyebox_hits=int(stats[2]), rng_states=rng.cpu().numpy().view(np.uint32))
    if rank != 0:
        scene.close()
        return out
    A = np.sum(matrix_EB, axis=(-2, -1)) / num_rays / num_iter
    names = {0: "Blue", 1: "Green", 2: "Red"}
    eff = {names.get(k, str(k)): float(np.sum(A[k] * 3)) for k in range(A.shape[0])}
    say("Simulation finished.")
    say(f"Number of rays traced : {num_rays * num_iter:,}")
    say(f"GPU calculation time  : {kern_s:.4f} s  ({out['bounces'] / max(kern_s, 1e-12):.3e} ray-bounces/s)")
    for c in ("Red", "Green", "Blue"):
        if c in eff:
            say(f"Efficiency ({c:5s})    : {eff[c] * 100:8.3f} %")
    out.update(matrix_EB=matrix_EB, A=A, efficiency=eff)
    if evaluate:
        from .AR_system_evaluation_functions import evaluation
        delta_e, U_fov, U_EB, output_image = evaluation(matrix_EB / R / num_iter)
        out.update(delta_e=float(delta_e), U_fov=float(U_fov), U_EB=float(U_EB), output_image=output_image)
        say(f"Color dispersion      : {delta_e:8.2f}")
        say(f"FoV uniformity        : {U_fov * 100:8.2f} %")
        say(f"Eyebox uniformity     : {U_EB * 100:8.2f} %")
    scene.close()
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description="MI355X full-colour waveguide ray tracing (reference MAIN flow)")
    ap.add_argument("--num-fov-x", type=int, default=100)
    ap.add_argument("--num-fov-y", type=int, default=75)
    ap.add_argument("--rays-per-fov", type=int, default=5000)
    ap.add_argument("--num-iter", type=int, default=4)
    ap.add_argument("--lut-dir", default=None, help="directory with lut_*_fullColor.npy (default: synthetic)")
    ap.add_argument("--lut-seed", type=int, default=0)
    ap.add_argument("--lut-profile", default="default")
    ap.add_argument("--point-seed", type=int, default=None)
    ap.add_argument("--no-eval", action="store_true")
    ap.add_argument("--fuse", choices=["auto", "yes", "no"], default="auto",
                    help="num_iter chained traces as one fused launch (auto: when a GPU traces <= 4M rays)")
    ap.add_argument("--no-fuse", action="store_true", help="same as --fuse no")
    ap.add_argument("--json", default=None, help="write scalar results here")
    a = ap.parse_args(argv)
    import torch
    import torch.distributed as dist
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    res = run(a.num_fov_x, a.num_fov_y, a.rays_per_fov, a.num_iter, lut_dir=a.lut_dir, lut_seed=a.lut_seed,
              lut_profile=a.lut_profile, point_seed=a.point_seed, evaluate=not a.no_eval,
              fuse=False if a.no_fuse else {"auto": None, "yes": True, "no": False}[a.fuse])
    if a.json and (not dist.is_initialized() or dist.get_rank() == 0):
        keep = {k: v for k, v in res.items() if isinstance(v, (int, float, dict, str))}
        with open(a.json, "w") as f:
            json.dump(keep, f, indent=1)
    if dist.is_initialized():
        dist.destroy_process_group()
    return res


if __name__ == "__main__":
    main()
