"""Where should default device histories come from?  The same trace timed into histories allocated by
torch.empty and by the history pool (_engine.pool_empty: shuffled 64 MiB chunks), for history sizes from
64 MiB to 1 GiB of the C2 system (float64, 11 planes) plus C2's own 704 MB (1M rays) and a quarter-size C3
(float32, 19 planes, 7.6 GB).  Several buffers of each kind live at once (placement differs per buffer),
timed interleaved in one process; one line per (size, kind): median and max of the per-buffer medians.

    python tools/history_threshold.py [--buffers 4] [--rounds 3]
"""
import argparse
import gc
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
import systems  # noqa: E402

DEV = torch.device("cuda", 0)
MiB = 1 << 20


def c2_case(hist_bytes):
    n = hist_bytes // (11 * 64)
    rays = torch.from_numpy(systems.c2_rays(n, seed=7)).to(DEV)
    system = systems.c2_system(rt, mat)
    mats = [mat.Vacuum()] + list(system.materials) + [mat.Vacuum()]
    low = E.lower(system.surfaces, mats, lambda: np.unique(rays[:, 7].cpu().numpy()), C.RTPB_F64)
    return f"C2 {n} rays f64 ({11 * 64 * n / MiB:.0f} MiB)", rays, low, torch.float64, len(system.surfaces)


def c3_quarter():
    system = systems.c3_system(rt, mat)
    nt, nph = 1581, 1581
    per = nt * nph
    rays = torch.empty((per * 5, 8), dtype=torch.float64, device=DEV)
    for k, h in enumerate(systems.C3_FIELDS):
        rt.fan_into(rays[k * per:(k + 1) * per], np.array([h, 0, 0]), np.pi / 180, nt, 0.635, nph)
    mats = [mat.Vacuum()] + list(system.materials) + [mat.Vacuum()]
    low = E.lower(system.surfaces, mats, lambda: np.array([0.635]), C.RTPB_F32)
    return (f"C3 quarter {rays.shape[0]} rays f32 ({19 * 32 * rays.shape[0] / MiB:.0f} MiB)", rays, low,
            torch.float32, len(system.surfaces))


def run(case, nbuf, rounds, reps=10):
    label, rays, low, tdt, S = case
    planes = E.resolve_planes("all", S)
    shape = (len(planes), rays.shape[0], 8)
    bufs = []
    for k in range(nbuf):
        bufs.append(("torch", torch.empty(shape, dtype=tdt, device=DEV)))
        bufs.append(("pool", E.pool_empty(shape, tdt, DEV)))
    st = torch.cuda.current_stream(DEV).cuda_stream
    times = [[] for _ in bufs]
    for _ in range(rounds):
        for i, (_, b) in enumerate(bufs):
            E.trace_device(low, rays, planes, out=b, stream=st)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                E.trace_device(low, rays, planes, out=b, stream=st)
            e1.record()
            torch.cuda.synchronize()
            times[i].append(e0.elapsed_time(e1) / reps)
    per = {"torch": [], "pool": []}
    for (kind, _), t in zip(bufs, times):
        per[kind].append(float(np.median(t)))
    for kind, v in per.items():
        print(f"{label:48s} {kind:5s} median {np.median(v):.4f} ms  max {max(v):.4f}  min {min(v):.4f}  "
              f"[{' '.join(f'{x:.4f}' for x in v)}]", flush=True)
    del bufs
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--buffers", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    for mib in (64, 128, 256, 512, 704, 1024):
        run(c2_case(mib * MiB if mib != 704 else 704_000_000), args.buffers, args.rounds)
    run(c3_quarter(), args.buffers, args.rounds)


if __name__ == "__main__":
    main()
