"""End-to-end System.ray_trace on device-resident rays vs the kernel alone (what the drop-in call adds:
lowering, plan cache, distinct wavelengths for TABLE materials, output allocation).

    python tools/e2e_overhead.py [--config c3|c2] [--scale 1.0] [--reps 5]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from ray_trace_pb_amd import _engine as E  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    wl = bench.Workload(args.config, dev, 0, scale=args.scale)
    dtype = "float32" if args.config == "c3" else None
    for _ in range(2):
        wl.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        wl.step()
    torch.cuda.synchronize()
    kern = (time.perf_counter() - t0) / args.reps
    wl.out = None
    torch.cuda.empty_cache()
    col = wl.rays[:, 7]
    for _ in range(2):
        E.distinct_wavelengths(col)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        E.distinct_wavelengths(col)
    torch.cuda.synchronize()
    uniq = (time.perf_counter() - t0) / args.reps
    h = wl.system.ray_trace(wl.rays, wl.m0, wl.m1, dtype=dtype)
    del h
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        h = wl.system.ray_trace(wl.rays, wl.m0, wl.m1, dtype=dtype)
        del h
    torch.cuda.synchronize()
    e2e = (time.perf_counter() - t0) / args.reps
    print(f"{args.config} n={wl.n}: kernel launches {kern * 1e3:.3f} ms, distinct_wavelengths {uniq * 1e3:.3f} ms, "
          f"System.ray_trace end to end {e2e * 1e3:.3f} ms")


if __name__ == "__main__":
    main()
