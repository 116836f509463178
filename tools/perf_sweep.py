"""Variant sweep of the trace kernel in ONE process (interleaved rounds, median of rounds): storage type,
output layout and stored planes, plus a device-to-device copy as the measured stream peak.
Kernel times come from HIP events recorded around each launch by librtpb (rtpb_timing_*)."""
import argparse
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=1_000_000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--configs", default="c2")
    ap.add_argument("--only", default="", help="comma list of variant-name substrings to keep")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = C.lib()
    res = {}
    recipes = {"c2": lambda: (systems.c2_system(rt, mat), systems.c2_rays(args.rays), mat.Vacuum(), mat.Vacuum()),
               "c5": lambda: (systems.c5_system(rt, mat),
                              systems.c5_rays(rt, 1, 101, max(1, args.rays // 707)), mat.Constant(1), mat.Constant(1)),
               "c4": lambda: (systems.c4_system(rt, mat), systems.c4_rays(rt, 1001, max(1, args.rays // 1001)),
                              mat.Constant(systems.OPM_N1), mat.Vacuum())}
    variants = []
    for cfg in args.configs.split(","):
        system, rays_np, m0, m1 = recipes[cfg]()
        S = len(system.surfaces)
        n = rays_np.shape[0]
        for dtype in ("f64", "f32"):
            code = C.RTPB_F64 if dtype == "f64" else C.RTPB_F32
            tdt = torch.float64 if dtype == "f64" else torch.float32
            low = E.lower(system.surfaces, [m0] + list(system.materials) + [m1], lambda: np.unique(rays_np[:, 7]), code)
            x = torch.from_numpy(rays_np).to(dev, dtype=tdt)
            for planes in ("all", "final"):
                sel = E.resolve_planes(planes, S)
                for layout in ("aos", "aos-nt", "aos-nt-sin", "aos-nt-w5", "aos-direct", "soa"):
                    lc = C.RTPB_SOA if layout == "soa" else C.RTPB_AOS
                    shape = (len(sel), n, 8) if lc == C.RTPB_AOS else (len(sel), 8, n)
                    out = torch.empty(shape, dtype=tdt, device=dev)
                    w = 8 if dtype == "f64" else 4
                    nbytes = n * 8 * w * (1 + len(sel))
                    name = f"{cfg}/{dtype}/{planes}/{layout}"
                    mode = {"aos": 1, "aos-nt": 3, "aos-nt-w5": 3 + 5 * 4, "aos-nt-sin": 3 + 64, "aos-direct": 0,
                            "soa": 0}[layout]
                    variants.append((name, low, x, sel, lc, out, nbytes, n * S, mode))
    if args.only:
        keep = args.only.split(",")
        variants = [v for v in variants if any(k in v[0] for k in keep)]
    # stream peak: device-to-device copy of 768 MB
    src = torch.empty(96_000_000, dtype=torch.float64, device=dev)
    dst = torch.empty_like(src)
    times = {v[0]: [] for v in variants}
    times["copy_768MB"] = []
    rng = np.random.default_rng(0)
    for _ in range(args.rounds):
        order = rng.permutation(len(variants))          # randomise the order every round
        for vi in order:
            name, low, x, sel, lc, out, nbytes, units, staged = variants[vi]
            C.check(lib.rtpb_set_tuning(b"aos_staging", staged & 1))
            C.check(lib.rtpb_set_tuning(b"nt_stores", (staged >> 1) & 1))
            C.check(lib.rtpb_set_tuning(b"stage_input", staged >> 6))
            E.trace_device(low, x, sel, layout_out=lc, out=out)
            torch.cuda.synchronize()
            lib.rtpb_timing_enable(1)
            for _ in range(args.reps):
                E.trace_device(low, x, sel, layout_out=lc, out=out)
            tot, cnt = ctypes.c_double(), ctypes.c_int64()
            C.check(lib.rtpb_timing_collect(ctypes.byref(tot), ctypes.byref(cnt)))
            lib.rtpb_timing_enable(0)
            times[name].append(tot.value / cnt.value)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        dst.copy_(src)
        e0.record()
        for _ in range(args.reps):
            dst.copy_(src)
        e1.record()
        torch.cuda.synchronize()
        times["copy_768MB"].append(e0.elapsed_time(e1) / args.reps)
    C.check(lib.rtpb_set_tuning(b"aos_staging", 1))
    C.check(lib.rtpb_set_tuning(b"nt_stores", 1))
    C.check(lib.rtpb_set_tuning(b"stage_input", 0))
    for name, low, x, sel, lc, out, nbytes, units, staged in variants:
        ms = float(np.median(times[name]))
        res[name] = {"ms": ms, "ms_min": float(np.min(times[name])), "GBps": nbytes / ms / 1e6,
                     "ray_surf_per_s": units / ms * 1e3}
    ms = float(np.median(times["copy_768MB"]))
    res["copy_768MB"] = {"ms": ms, "GBps": 2 * src.numel() * 8 / ms / 1e6}
    for k, v in res.items():
        print(f"{k:28s} " + "  ".join(f"{a}={b:.4g}" for a, b in v.items()))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
