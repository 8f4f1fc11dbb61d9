#!/usr/bin/env python3
"""The N > 1 bench path's collectives over RCCL on a one-GPU box (tests/test_gpu_rccl.py runs it).

RCCL refuses two ranks on one GPU, so the driver's 8-GPU run is the first to run the strong-scaling
path with every rank on its own device.  This probe runs what that path asks of RCCL in a one-rank
RCCL communicator (``init_process_group("nccl", device_id=...)``, as bench.py does for N > 1), with
the exact buffers, dtypes and call shapes of ``distributed.EyeboxGather`` and ``timed_run``:

* the eyebox gather of an 8-rank C3 split: virtual rank r traces its interleaved shard into a grid
  of its own, its payload is packed on the device (``wgrt_eyebox_pack``) and moved into rank 0's
  receive row r by ``dist.gather`` (one-rank gather: ``gather_list=[recv[r]]``);
  ``wgrt_eyebox_assemble`` then builds the grid, which must equal the whole batch's trace bit for bit;
* ``dist.reduce`` (SUM, float32) of the grid -- the ``weak`` record's and ``--collective reduce``'s
  collective -- and the two small ``all_reduce``s of ``timed_run`` (MAX float64, SUM int64);
* ``dist.barrier`` with the device bound at init.

Prints one JSON line; exits non-zero on any mismatch.  Launch with RANK=0 WORLD_SIZE=1
MASTER_ADDR=127.0.0.1 MASTER_PORT=<free port> (or under torch.distributed.run)."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch
    import torch.distributed as dist

    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.configs import CONFIGS, build_inputs
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.distributed import (EyeboxGather, hip_shard_builder,
                                                                                make_shard)
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.engine import Scene, new_stats, trace_fullcolor

    if int(os.environ.get("WORLD_SIZE", "1")) != 1:
        raise SystemExit("rccl_probe runs one rank")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    rec = {"backend": dist.get_backend(), "torch": torch.__version__}

    # the C3 batch traced whole (the reference), and split 8 ways as the strong-scaling ranks trace it:
    # virtual rank r traces its interleaved shard into its own grid (its slabs plus their spills)
    w = CONFIGS["C3"]
    nx, ny, lambdas, R = w.nx, w.ny, list(w.lambdas), w.R
    geom, luts, points = build_inputs(w)
    scene = Scene.from_geometry(geom, luts, device=0)
    build = hip_shard_builder(points, nx, ny, lambdas, R, dev)

    def trace(shard, eb, st):
        rays, rng = build(shard)
        gm = shard.gid
        kw = dict(gid_offset=gm.offset) if gm.offset is not None else dict(
            gid_blocks=torch.as_tensor(gm.block_gid, device=dev), gid_block_rays=R)
        trace_fullcolor(scene, rays, rng, eb, stats=st, **kw)

    eb = torch.zeros(scene.eb_shape(), dtype=torch.float32, device=dev)
    st = new_stats(dev)
    trace(make_shard(nx, ny, len(lambdas), R, 1, 0), eb, st)
    world = 8
    shards = [make_shard(nx, ny, len(lambdas), R, world, r) for r in range(world)]
    grids, st_r = [], new_stats(dev)
    for sh in shards:
        grids.append(torch.zeros_like(eb))
        trace(sh, grids[-1], st_r)
    torch.cuda.synchronize()
    hits = int(st[2].item())
    assert hits > 0 and float(eb.sum().item()) == float(hits), "traced grid does not hold the hits"
    assert int(st_r[2].item()) == hits and int(st_r[0].item()) == int(st[0].item()), "shards differ from the batch"

    g = EyeboxGather([sh.blocks for sh in shards], nx, ny, lambdas, scene.num_lmd, device=dev)
    send, recv = g.buffers(dev, eb.dtype, True)
    recv.fill_(float("nan"))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for r in range(world):
        payload = g.pack(grids[r], r, out=send)
        dist.gather(payload, gather_list=[recv[r]], dst=0)
    out = torch.full_like(eb, float("nan"))
    g.assemble(out, recv)
    torch.cuda.synchronize()
    rec["gather_8way_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
    rec["payload_bytes_per_rank"] = int(g.payload_len * 4)
    if not torch.equal(out, eb):
        bad = int((out != eb).sum().item())
        raise SystemExit(f"RCCL gather + assembly of the 8 shards' grids differs from the batch's grid in {bad} cells")
    rec["gather_equal"] = True
    spill = sum(int(g.has_spill[r]) for r in range(world))
    rec["ranks_with_spill_rows"] = spill

    red = eb.clone()
    dist.reduce(red, dst=0, op=dist.ReduceOp.SUM)
    t = torch.tensor([1.25], dtype=torch.float64, device=dev)
    b = torch.tensor([int(st[0].item())], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(b, op=dist.ReduceOp.SUM)
    dist.barrier()
    torch.cuda.synchronize()
    if not (torch.equal(red, eb) and float(t.item()) == 1.25 and int(b.item()) == int(st[0].item())):
        raise SystemExit("one-rank reduce / all_reduce changed their operands")
    rec.update(reduce_equal=True, all_reduce_ok=True, hits=hits, bounces=int(st[0].item()),
               slabs_per_rank=[len(sh.blocks) for sh in shards][:2])
    dist.destroy_process_group()
    scene.close()
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
