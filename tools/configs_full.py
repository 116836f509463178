"""BASELINE configs[2] (C3: 4f relay, 5 fields x 10M-ray fans, float32) and configs[3] (C4: ideal OPM,
100M-ray fan, float32) at FULL size on one GPU: float64 rays generated on the device, full drop-in history
stored as float32 (float64 arithmetic) kept in HBM, plus an exact check of a random subsample against the
NumPy oracle (the float64 reference trace, rounded once to float32).

    python tools/configs_full.py [--which c3,c4] [--scale 1.0]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", default="c3,c4")
    ap.add_argument("--scale", type=float, default=1.0, help="fraction of the per-axis fan sizes")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--check", type=int, default=20000, help="rays in the exact oracle subsample")
    args = ap.parse_args()
    import torch
    import ray_trace_pb_amd.materials as mat
    import ray_trace_pb_amd.raytrace as rt
    from ray_trace_pb_amd import _capi as C, _engine as E
    from oracle import rt_numpy as O
    from serialize import material_to_dict, surface_to_dict
    import systems
    dev = torch.device("cuda:0")
    lib = C.lib()
    for which in args.which.split(","):
        if which == "c3":
            system, m0, m1 = systems.c3_system(rt, mat), mat.Vacuum(), mat.Vacuum()
            nt, nph = int(3163 * args.scale), int(3162 * args.scale)
            fans = [rt.get_ray_fan(np.array([h, 0, 0]), np.pi / 180, nt, 0.635, nphis=nph, device=dev)
                    for h in systems.C3_FIELDS]
            rays = torch.cat(fans)
            del fans
            label = "C3 4f relay (2x AC508-075 + stop), 5 fields x fan(1 deg, %dx%d)" % (nt, nph)
        else:
            system, m0, m1 = systems.c4_system(rt, mat), mat.Constant(systems.OPM_N1), mat.Vacuum()
            nt, nph = int(10001 * args.scale), int(10000 * args.scale)
            theta = 30 * np.pi / 180
            rays = rt.get_ray_fan([1e-3, 1e-3, 1e-3 * np.tan(theta)], np.arcsin(1.35 / systems.OPM_N1), nt,
                                  systems.OPM_WAVELENGTH, nphis=nph, device=dev)
            label = "C4 ideal OPM (6 PerfectLens + 5 flats), fan(asin(1.35/1.4), %dx%d)" % (nt, nph)
        S = len(system.surfaces)
        n = rays.shape[0]
        mats = [m0] + list(system.materials) + [m1]
        low = E.lower(system.surfaces, mats, lambda: np.unique(rays[:, 7].double().cpu().numpy()), C.RTPB_F32)
        sel = E.resolve_planes("all", S)
        out = torch.empty((len(sel), n, 8), dtype=torch.float32, device=dev)
        E.trace_device(low, rays, sel, out=out)
        torch.cuda.synchronize()
        lib.rtpb_timing_enable(1)
        t0 = time.perf_counter()
        for _ in range(args.reps):
            E.trace_device(low, rays, sel, out=out)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / args.reps
        tot, cnt = ctypes.c_double(), ctypes.c_int64()
        C.check(lib.rtpb_timing_collect(ctypes.byref(tot), ctypes.byref(cnt)))
        lib.rtpb_timing_enable(0)
        kms = tot.value / cnt.value
        nbytes = n * (64 + 32 * len(sel))            # float64 input record, float32 planes
        # exact subsample check against the oracle
        idx = torch.from_numpy(np.sort(np.random.default_rng(1).choice(n, min(args.check, n), replace=False))).to(dev)
        r_in = rays[idx].cpu().numpy()
        ref = O.ray_trace([surface_to_dict(s) for s in system.surfaces], [material_to_dict(m) for m in mats], r_in)
        got = out[:, idx].cpu().numpy()
        exact = bool(np.array_equal(got, ref.astype(np.float32), equal_nan=True))
        live = float((~torch.isnan(out[-1, :, 0])).float().mean())
        print(json.dumps({"config": which, "workload": label, "rays": n, "surfaces": S, "planes": len(sel),
                          "history_GB": out.numel() * 4 / 1e9, "kernel_ms": kms, "wall_ms": wall * 1e3,
                          "ray_surface_per_s": n * S / (kms * 1e-3), "alg_GBps": nbytes / (kms * 1e-3) / 1e9,
                          "live_fraction_final": live, "subsample": len(idx), "subsample_bitexact": exact}),
              flush=True)
        del out, rays
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
