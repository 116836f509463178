"""Bundle-size scan of the C2 trace (f64, full history, AoS): kernel time vs rays, to separate the fixed
per-launch cost (wave ramp-up before the first stores, drain tail) from the streaming rate.  Optional
extra libraries (experiment builds, e.g. -DRTPB_EXP_NO_COMPUTE) are timed on the same buffers, and a
torch fill_ of the output bytes gives the box's write ceiling at each size.

    python tools/size_scan.py [--sizes 250000,1000000,4000000] [exp.so ...]
"""
import argparse
import collections
import ctypes
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
import systems  # noqa: E402


def load(path):
    h = ctypes.CDLL(os.path.abspath(path))
    for name, (res, argt) in C.SIGNATURES.items():
        fn = getattr(h, name)
        fn.restype, fn.argtypes = res, argt
    return h


def timed(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*")
    ap.add_argument("--sizes", default="125000,250000,500000,1000000,2000000,4000000,8000000")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--planes", default="all")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    libs = {"base": C.lib()}
    for p in args.libs:
        libs[os.path.basename(p).replace(".so", "")] = load(p)
    system = systems.c2_system(rt, mat)
    S = len(system.surfaces)
    mats = [mat.Vacuum()] + list(system.materials) + [mat.Vacuum()]
    res = {}
    for n in [int(v) for v in args.sizes.split(",")]:
        rays_np = systems.c2_rays(n)
        x = torch.from_numpy(rays_np).to(dev)
        sel = E.resolve_planes(args.planes, S)
        out = torch.empty((len(sel), n, 8), dtype=torch.float64, device=dev)
        nbytes = n * 64 * (1 + len(sel))
        reps = max(5, min(200, int(2e9 // nbytes)))
        caches = {k: collections.OrderedDict() for k in libs}
        times = {k: [] for k in list(libs) + ["fill"]}
        stream = torch.cuda.current_stream(dev).cuda_stream
        low = E.lower(system.surfaces, mats, lambda: np.unique(rays_np[:, 7]), C.RTPB_F64)
        for _ in range(args.rounds):
            for name, h in libs.items():
                C._lib, E._PLANS = h, caches[name]        # route the engine through this build
                times[name].append(timed(lambda: E.trace_device(low, x, sel, out=out, stream=stream), reps))
            C._lib, E._PLANS = libs["base"], caches["base"]
            times["fill"].append(timed(lambda: out.fill_(1.0), reps))
        row = {}
        for k, v in times.items():
            ms = float(np.median(v))
            b = nbytes if k != "fill" else out.numel() * 8
            row[k] = {"ms": ms, "GBps": b / ms / 1e6}
        res[n] = row
        print(n, json.dumps({k: round(v["ms"], 4) for k, v in row.items()}),
              json.dumps({k: round(v["GBps"]) for k, v in row.items()}), flush=True)
        del out, x
        torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
