"""Why the drop-in call's kernel differs from the bench loop's on C3: the same plan traced into the same
buffer, interleaved, (a) as the bench loop does it (trace_device on the bench's stream, no miss flag),
(b) with the table-miss flag, (c) on the current stream, (d) through System.ray_trace (its own history).
Kernel ms from the library's HIP events.

    python tools/e2e_kernel_diff.py [--rounds 5]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import numpy as np  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch
    from ray_trace_pb_amd import _capi as C
    dev = torch.device("cuda:0")
    wl = bench.Workload("c3", dev, 0)
    E = wl._E
    lib = C.lib()
    miss = torch.zeros(1, dtype=torch.int32, device=dev)
    dt = "float32"

    def kernel_ms(fn):
        lib.rtpb_timing_enable(1)
        for _ in range(args.reps):
            fn()
        torch.cuda.synchronize()
        tot, cnt = ctypes.c_double(), ctypes.c_int64()
        C.check(lib.rtpb_timing_collect(ctypes.byref(tot), ctypes.byref(cnt)))
        lib.rtpb_timing_enable(0)
        return tot.value / cnt.value

    variants = {
        "loop (bench stream, no flag)": lambda: E.trace_device(wl.low, wl.rays, wl.planes, out=wl.out, stream=wl.stream),
        "with miss flag": lambda: E.trace_device(wl.low, wl.rays, wl.planes, out=wl.out, stream=wl.stream, miss=miss),
        "current stream": lambda: E.trace_device(wl.low, wl.rays, wl.planes, out=wl.out),
        "System.ray_trace": lambda: wl.system.ray_trace(wl.rays, wl.m0, wl.m1, dtype=dt),
    }
    for f in variants.values():
        f()
    torch.cuda.synchronize()
    res = {k: [] for k in variants}
    for _ in range(args.rounds):
        for k, f in variants.items():
            res[k].append(kernel_ms(f))
    for k, v in res.items():
        print(f"{k:32s} kernel {np.median(v):.4f} ms  (min {min(v):.4f})", flush=True)


if __name__ == "__main__":
    main()
