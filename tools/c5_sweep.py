"""BASELINE configs[4] / SURVEY C5: spot-diagram sweep, 64 field points x 7 wavelengths x 10M-ray fans
(get_ray_fan, 0.5 deg, 3163 x 3162) through the 14-surface ODT excitation system, float64, final plane
only, spot statistics reduced on the GPU.  One process per GPU (torchrun): field points are split
across ranks (no collective besides the final gather of the small statistics table).

    python tools/c5_sweep.py [--fields 64] [--n-thetas 3163] [--nphis 3162]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fields", type=int, default=64, help="field points (square grid)")
    ap.add_argument("--n-thetas", type=int, default=3163)
    ap.add_argument("--nphis", type=int, default=3162)
    ap.add_argument("--dtype", default="float64")
    ap.add_argument("--devices", default="", help="in-process multi-GPU: 'all' or comma-separated GPU ids")
    ap.add_argument("--warmup", type=int, default=1,
                    help="untimed small sweeps first (plan creation, code-object load on first launch)")
    ap.add_argument("--lib", default="", help="library build to load instead of the in-tree librtpb.so (A/B)")
    args = ap.parse_args()
    import torch
    if args.lib:
        from ray_trace_pb_amd import _capi
        _capi.LIB_PATH = os.path.abspath(args.lib)
    import ray_trace_pb_amd.materials as mat
    import ray_trace_pb_amd.raytrace as rt
    from ray_trace_pb_amd import analysis
    import systems
    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    dev = torch.device("cuda", local % max(torch.cuda.device_count(), 1))
    torch.cuda.set_device(dev)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    n_side = int(round(np.sqrt(args.fields)))
    fields = systems.c5_field_points(n_side)
    mine = fields[rank::world]
    system = systems.c5_system(rt, mat)
    wls = systems.C5_WAVELENGTHS
    theta = 0.5 * np.pi / 180
    devices = None
    if args.devices:
        devices = list(range(torch.cuda.device_count())) if args.devices == "all" else \
            [int(d) for d in args.devices.split(",")]
    for _ in range(args.warmup):
        analysis.spot_sweep(system, mat.Constant(1), mat.Constant(1), mine, wls, theta, 33, 32, device=dev,
                            dtype=args.dtype, devices=devices)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    summ, timing = analysis.spot_sweep(system, mat.Constant(1), mat.Constant(1), mine, wls, theta, args.n_thetas,
                                       args.nphis, device=dev, dtype=args.dtype, devices=devices)
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    rays = timing["rays"]
    if world > 1:
        t = torch.tensor([wall, float(rays)], dtype=torch.float64)
        dist.all_reduce(t[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        wall, rays = float(t[0]), float(t[1])
    if rank == 0:
        S = len(system.surfaces)
        print(json.dumps({"workload": "C5 spot sweep", "fields": len(fields), "wavelengths": len(wls),
                          "rays_per_group": args.n_thetas * args.nphis, "total_rays": rays, "surfaces": S,
                          "n_gpus": world, "seconds": wall, "ray_surface_per_s": rays * S / wall,
                          "per_device_rank0": timing.get("per_device"),
                          "rank0_rms_radius_um_first_fields": (summ["rms_radius"][:2] * 1e3).tolist(),
                          "rank0_count_first_fields": summ["count"][:2].tolist()}))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
