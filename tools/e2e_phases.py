"""Host phases of the drop-in call System.ray_trace(torch rays, ...) on the device-resident bundle of a
bench config: each phase's host time per call (lowering memo, table keys, miss flag,
history allocation from the history pool (round 5: a torch MemPool) or torch.empty, launch, the miss-flag read), the call's kernel (HIP events inside the
library), and two references -- a bare launch + synchronize into a held buffer (the floor a synchronous call
pays), and the call without its history allocation (out=).

    python tools/e2e_phases.py [--config c3] [--reps 15]
"""
import argparse
import collections
import ctypes
import functools
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]

import numpy as np  # noqa: E402

import bench  # noqa: E402

ACC = collections.defaultdict(float)


def wrap(mod, name, label=None):
    fn = getattr(mod, name)

    @functools.wraps(fn)
    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            ACC[label or name] += time.perf_counter() - t0
    setattr(mod, name, w)


def kernel_ms(lib, C):
    tot, cnt = ctypes.c_double(), ctypes.c_int64()
    C.check(lib.rtpb_timing_collect(ctypes.byref(tot), ctypes.byref(cnt)))
    return tot.value / max(cnt.value, 1), cnt.value


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--reps", type=int, default=15)
    args = ap.parse_args()
    import torch
    from ray_trace_pb_amd import _capi as C
    from ray_trace_pb_amd import _engine as E
    from ray_trace_pb_amd import raytrace as R
    dev = torch.device("cuda:0")
    wl = bench.Workload(args.config, dev, 0)
    dt = "float32" if wl.code != C.RTPB_F64 else None
    lib = C.lib()
    held = wl.out

    # (1) floor: bare launch into the held buffer + synchronize, per call
    for _ in range(3):
        wl.step()
    torch.cuda.synchronize()
    ts = []
    lib.rtpb_timing_enable(1)
    for _ in range(args.reps):
        t0 = time.perf_counter()
        wl.step()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    k, n = kernel_ms(lib, C)
    lib.rtpb_timing_enable(0)
    print(f"bare launch+sync: median {np.median(ts) * 1e3:.3f} ms, kernel {k:.3f} ms -> overhead "
          f"{np.median(ts) * 1e3 - k:.3f} ms (min {min(ts) * 1e3 - k:.3f})", flush=True)

    # (2) the drop-in call with out= (no allocation)
    for _ in range(2):
        wl.system.ray_trace(wl.rays, wl.m0, wl.m1, dtype=dt, out=held)
    torch.cuda.synchronize()
    ts = []
    lib.rtpb_timing_enable(1)
    for _ in range(args.reps):
        t0 = time.perf_counter()
        wl.system.ray_trace(wl.rays, wl.m0, wl.m1, dtype=dt, out=held)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    k, n = kernel_ms(lib, C)
    lib.rtpb_timing_enable(0)
    print(f"ray_trace(out=held): median {np.median(ts) * 1e3:.3f} ms, kernel {k:.3f} ms -> overhead "
          f"{np.median(ts) * 1e3 - k:.3f} ms", flush=True)
    del held, wl.out
    torch.cuda.synchronize()

    # (3) the drop-in call as the bench times it, phase by phase
    for name in ("memo_lookup", "memo_store", "lower", "tabulated", "table_fingerprint", "previous_keys", "trace_device", "history_buffer",
                 "distinct_wavelengths", "pool_empty", "device_empty", "history_pool", "resolve_planes"):
        wrap(E, name)
    wrap(R, "_default_history")
    item = torch.Tensor.item

    def timed_item(self):
        t0 = time.perf_counter()
        try:
            return item(self)
        finally:
            ACC["miss.item"] += time.perf_counter() - t0
    torch.Tensor.item = timed_item
    zeros = torch.zeros

    def timed_zeros(*a, **kw):
        t0 = time.perf_counter()
        try:
            return zeros(*a, **kw)
        finally:
            ACC["torch.zeros"] += time.perf_counter() - t0
    torch.zeros = timed_zeros
    for _ in range(3):
        h = wl.system.ray_trace(wl.rays, wl.m0, wl.m1, dtype=dt)
        del h
    torch.cuda.synchronize()
    ACC.clear()
    ts, dels = [], []
    lib.rtpb_timing_enable(1)
    for _ in range(args.reps):
        t0 = time.perf_counter()
        h = wl.system.ray_trace(wl.rays, wl.m0, wl.m1, dtype=dt)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
        t1 = time.perf_counter()
        del h
        dels.append(time.perf_counter() - t1)
    k, n = kernel_ms(lib, C)
    lib.rtpb_timing_enable(0)
    torch.Tensor.item = item
    torch.zeros = zeros
    print(f"ray_trace(): median {np.median(ts) * 1e3:.3f} ms (min {min(ts) * 1e3:.3f}), kernel {k:.3f} ms -> "
          f"overhead {np.median(ts) * 1e3 - k:.3f} ms; del history {np.median(dels) * 1e3:.3f} ms", flush=True)
    for name, v in sorted(ACC.items(), key=lambda kv: -kv[1]):
        print(f"  {name:24s} {v / args.reps * 1e3:8.3f} ms per call (inclusive)")
    print("  (trace_device includes the launch; miss.item waits for the kernel: its excess over the kernel is "
          "the synchronisation latency)")


if __name__ == "__main__":
    main()
