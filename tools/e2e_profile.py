"""Where the drop-in call spends its time beyond the kernel: System.ray_trace(torch rays, ...) on the
device-resident C3 bundle under cProfile (host functions by own time), beside the kernel time from HIP
events around the same calls.

    python tools/e2e_profile.py [--config c3] [--reps 20]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import torch
    from ray_trace_pb_amd import _capi as C
    dev = torch.device("cuda:0")
    wl = bench.Workload(args.config, dev, 0)
    dt = "float32" if wl.code != C.RTPB_F64 else None
    del wl.out
    torch.cuda.empty_cache()
    for _ in range(3):
        h = wl.system.ray_trace(wl.rays, wl.m0, wl.m1, dtype=dt)
        del h
    torch.cuda.synchronize()
    lib = C.lib()
    lib.rtpb_timing_enable(1)
    t0 = time.perf_counter()
    for _ in range(args.reps):
        h = wl.system.ray_trace(wl.rays, wl.m0, wl.m1, dtype=dt)
        del h
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.reps
    import ctypes
    tot, cnt = ctypes.c_double(), ctypes.c_int64()
    C.check(lib.rtpb_timing_collect(ctypes.byref(tot), ctypes.byref(cnt)))
    lib.rtpb_timing_enable(0)
    kern = tot.value / cnt.value * 1e-3
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(args.reps):
        h = wl.system.ray_trace(wl.rays, wl.m0, wl.m1, dtype=dt)
        del h
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
    print(f"{args.config}: System.ray_trace {wall * 1e3:.3f} ms per call, kernel {kern * 1e3:.3f} ms "
          f"(launches timed: {cnt.value}), overhead {(wall - kern) * 1e3:.3f} ms")
    print(s.getvalue())


if __name__ == "__main__":
    main()
