"""Throughput of the §8(f) kernels around the trace (device ray generators, intersect_rays, spot
statistics, propagate_ray2plane, the user-geometry hook kernels) against the HBM roofline.

Each op runs K times back to back through its public Python API on device tensors; HIP events on
the launch stream around the K calls give the average call time (includes the API's own small
host work).  Algorithmic bytes per call = bytes each kernel must read + write once.  Run under
`rocprofv3 --kernel-trace --stats` for the pure kernel durations.

    python tools/bench_aux.py [--rays N] [--reps K]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ray_trace_pb_amd.materials as mat  # noqa: E402
import ray_trace_pb_amd.raytrace as rt  # noqa: E402
from ray_trace_pb_amd import _capi as C  # noqa: E402
from ray_trace_pb_amd import _engine as E  # noqa: E402
from ray_trace_pb_amd import analysis  # noqa: E402

PEAK = 8000.0


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=10_000_000)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    N = args.rays
    nth = int(np.sqrt(N))
    nph = N // nth
    n = nth * nph
    res = {}

    def rec(name, ms, nbytes, units, note):
        res[name] = {"ms": ms, "GBps": nbytes / ms / 1e6, "frac": nbytes / ms / 1e6 / PEAK,
                     "units_per_s": units / ms * 1e3, "bytes_per_call": nbytes, "note": note}

    # f1 generators: write n x 64 B
    fan = lambda: rt.get_ray_fan([0, 0, 0], 0.1, nth, 0.635, nphis=nph, device=dev)  # noqa: E731
    rec("get_ray_fan", timed(fan, args.reps), 64 * n, n, f"{nth} x {nph} fan, f64 rows written")
    col = lambda: rt.get_collimated_rays([0, 0, -5], 10, nth, 0.855, nphis=nph, device=dev)  # noqa: E731
    rec("get_collimated_rays", timed(col, args.reps), 64 * n, n, f"{nth} x {nph} disk, f64 rows written")

    rays = fan()
    # f2 intersect_rays: read two ray sets, write 3 doubles per pair
    r2 = rays.flip(0).contiguous()
    isect = lambda: rt.intersect_rays(rays, r2)  # noqa: E731
    rec("intersect_rays", timed(isect, args.reps), n * (64 + 64 + 24), n, "pairwise, n pairs")
    # f2 spot statistics: read the plane once
    groups = 64
    gs = n // groups
    plane = rays[: groups * gs]
    spot = lambda: analysis.spot_stats_raw(plane, gs)  # noqa: E731
    rec("spot_stats", timed(spot, args.reps), 64 * groups * gs, groups * gs, f"{groups} groups")
    # propagate_ray2plane on device rays: read + write one row, + ts
    prop = lambda: rt.propagate_ray2plane(rays, [0, 0, 1], [0, 0, 50], mat.Bk7())  # noqa: E731
    rec("propagate_ray2plane", timed(prop, args.reps), n * (64 + 64 + 8), n, "Sellmeier medium, ts returned")

    # user-geometry hook kernels (propagate_user_geometry's device part)
    surf = rt.FlatSurface([0, 0, 50], [0, 0, 1], 1e9)
    low = E.lower([surf], [mat.Vacuum(), mat.Bk7()], lambda: np.array([0.635]), C.RTPB_F64)
    plan = E.plan_for(low)
    hits = rt.propagate_ray2plane(rays, [0, 0, 1], [0, 0, 50], mat.Vacuum())[0]
    normals = torch.tensor([0.0, 0.0, 1.0], device=dev, dtype=torch.float64).expand(n, 3).contiguous()
    on = torch.ones(n, dtype=torch.uint8, device=dev)
    out = torch.empty_like(hits)
    lib = C.lib()
    st = torch.cuda.current_stream(dev).cuda_stream
    fs = lambda: C.check(lib.rtpb_front_side(plan, 0, rays.data_ptr(), hits.data_ptr(), n, out.data_ptr(), st))  # noqa: E731,E501
    rec("hook_front_side", timed(fs, args.reps), n * 64 * 3, n, "read rays + hits, write hits")
    it = lambda: C.check(lib.rtpb_interact(plan, 0, C.RTPB_REFRACT, hits.data_ptr(), normals.data_ptr(),  # noqa: E731
                                           on.data_ptr(), n, out.data_ptr(), st))
    rec("hook_interact", timed(it, args.reps), n * (64 + 24 + 1 + 64), n, "Snell, read hits+normals+mask, write")

    for k, v in res.items():
        print(f"{k:22s} {v['ms']:8.4f} ms  {v['GBps']:7.0f} GB/s  frac {v['frac']:.2f}  {v['units_per_s']:.3e}/s  "
              f"({v['note']})")
    print(json.dumps({"rays": n, "results": res}))


if __name__ == "__main__":
    main()
