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
   and ``evaluation(EB / R / num_iter)`` (MAIN:197-198);
6. the "Eyebox Center View.png" export (MAIN:199-203): the evaluated image at the first eye row,
   last eye column, as 8-bit RGB, rows flipped (``eyebox_center_view``, written without OpenCV).

The matplotlib plots (MAIN:213-237) are visual-only and not reproduced.
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
        fuse: bool | None = None, points: np.ndarray | None = None, png: str | None = None) -> dict:
    """The reference script's job on this engine; returns its printed quantities and arrays.
    ``points``: the R/2 in-coupler origins to use (default: sampled, GRTF:12-23, seeded by
    ``point_seed``); ``png``: where to write the "Eyebox Center View" image (needs ``evaluate``)."""
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
    if points is None:
        points = generate_points_in_polygon(geom.IC, R // 2, rng=rng_pts)
    points = np.ascontiguousarray(points, dtype=np.float64)
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
        out["center_view"] = eyebox_center_view(output_image)
        if png:
            write_png(png, out["center_view"])
            say(f"Wrote {png}")
        say(f"Color dispersion      : {delta_e:8.2f}")
        say(f"FoV uniformity        : {U_fov * 100:8.2f} %")
        say(f"Eyebox uniformity     : {U_EB * 100:8.2f} %")
    scene.close()
    return out


def eyebox_center_view(output_image: np.ndarray) -> np.ndarray:
    """The image MAIN:199-203 exports: ``output_image[:, :, :, 0, n_epx - 1]`` (first eye row, last eye
    column) as uint8 (``* 255`` then truncation), rows flipped -- uint8 RGB [n_FOVy, n_FOVx, 3].  (The
    reference converts it to BGR for cv2.imwrite, which stores the RGB image in the PNG.)"""
    n_epx = output_image.shape[4]
    return np.ascontiguousarray(np.flipud((output_image[:, :, :, 0, n_epx - 1] * 255).astype(np.uint8)))


def write_png(path: str, rgb: np.ndarray) -> None:
    """8-bit RGB PNG (filter 0 on every row, zlib), without OpenCV / PIL."""
    import struct
    import zlib
    a = np.ascontiguousarray(rgb, dtype=np.uint8)
    if a.ndim != 3 or a.shape[2] != 3:
        raise ValueError("expected an [H, W, 3] uint8 image")
    h, w = a.shape[:2]

    def chunk(tag, data):
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)
    raw = b"".join(b"\x00" + a[r].tobytes() for r in range(h))
    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0)) +
                chunk(b"IDAT", zlib.compress(raw, 9)) + chunk(b"IEND", b""))


def read_png(path: str) -> np.ndarray:
    """Decoder of write_png's files (8-bit RGB, filter 0), for the tests."""
    import struct
    import zlib
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, w, h = 8, b"", 0, 0
    while pos < len(data):
        n, tag = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        if tag == b"IHDR":
            w, h = struct.unpack(">II", body[:8])
        elif tag == b"IDAT":
            idat += body
        pos += 12 + n
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 1 + 3 * w)
    assert (raw[:, 0] == 0).all()
    return raw[:, 1:].reshape(h, w, 3).copy()


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
    ap.add_argument("--png", default="Eyebox Center View.png",
                    help="the eyebox-center image (MAIN:199-203); empty string: do not write it")
    a = ap.parse_args(argv)
    import torch
    import torch.distributed as dist
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    res = run(a.num_fov_x, a.num_fov_y, a.rays_per_fov, a.num_iter, lut_dir=a.lut_dir, lut_seed=a.lut_seed,
              lut_profile=a.lut_profile, point_seed=a.point_seed, evaluate=not a.no_eval,
              fuse=False if a.no_fuse else {"auto": None, "yes": True, "no": False}[a.fuse],
              png=a.png or None)
    if a.json and (not dist.is_initialized() or dist.get_rank() == 0):
        keep = {k: v for k, v in res.items() if isinstance(v, (int, float, dict, str))}
        with open(a.json, "w") as f:
            json.dump(keep, f, indent=1)
    if dist.is_initialized():
        dist.destroy_process_group()
    return res


if __name__ == "__main__":
    main()
