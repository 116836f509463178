"""Which store patterns are sensitive to the placement of the history buffer?  Allocates --buffers buffers of
one C3 history each (--scale 0.5: 7.6 GB, 1.0: 30.4 GB) with torch and times, interleaved over rounds, a
plain fill (1 plane) and 19-plane patterns with 2 / 8 / 32 KiB per wave and plane, with and without pacing
between planes (tools/store_multi.hip), plus the real C3 trace into the same buffers.

    python tools/store_multi.py [--buffers 24] [--scale 0.5]
"""
import argparse
import collections
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "tests", "golden")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from ray_trace_pb_amd import _capi as C  # noqa: E402
from ray_trace_pb_amd import _engine as E  # noqa: E402
import ab_variants  # noqa: E402

SO = os.path.join(ROOT, "tools", "_build", "libstore_multi.so")
PATTERNS = [("fill", 1, 2, 0), ("p19c2", 19, 2, 0), ("p19c8", 19, 8, 0), ("p19c32", 19, 32, 0),
            ("p19c2s", 19, 2, 4), ("p19c8s", 19, 8, 4)]


def build():
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(SO.replace("_build/lib", "").replace(".so", ".hip")):
        os.makedirs(os.path.dirname(SO), exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", "-o", SO,
                        os.path.join(ROOT, "tools", "store_multi.hip")], check=True)
    return SO


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--buffers", type=int, default=24)
    ap.add_argument("--scale", type=float, default=0.5)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--build-only", action="store_true")
    args = ap.parse_args()
    if args.build_only:
        print(build())
        return
    dev = torch.device("cuda:0")
    lib = C.lib()
    sm = ctypes.CDLL(SO)
    sm.store_multi.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    system, m0, m1, x, code = ab_variants.build_case(f"c3:{args.scale}", dev)
    n, S = x.shape[0], len(system.surfaces)
    low = E.lower(system.surfaces, [m0] + list(system.materials) + [m1], lambda: np.array([0.635]), code)
    sel = E.resolve_planes("all", S)
    P = len(sel)
    lo, hi = E.plane_mask(sel)
    plane_bytes = n * 32
    bufs = [torch.empty((P, n, 8), dtype=torch.float32, device=dev) for _ in range(args.buffers)]
    h = ctypes.c_void_p()
    C.check(lib.rtpb_plan_create(low.surfaces, low.nsurf, low.materials, low.nsurf + 1, low.dtype, ctypes.byref(h)))
    stream = torch.cuda.current_stream(dev).cuda_stream

    def launch(kind, buf):
        if kind == "trace":
            C.check(lib.rtpb_trace(h, 0, x.data_ptr(), C.RTPB_F64, n, C.RTPB_AOS, 0, buf.data_ptr(), C.RTPB_AOS,
                                   n * 8, 0, lo, hi, stream))
            return
        _, planes, chunk, sleep = next(p for p in PATTERNS if p[0] == kind)
        pb = plane_bytes * (19 // planes) // (chunk * 1024) * (chunk * 1024)
        assert sm.store_multi(buf.data_ptr(), pb, planes, chunk, sleep, stream) == 0

    kinds = [p[0] for p in PATTERNS] + ["trace"]
    items = [(k, b) for k in kinds for b in range(len(bufs))]
    times = collections.defaultdict(list)
    rng = np.random.default_rng(0)
    for _ in range(args.rounds):
        for i in rng.permutation(len(items)):
            k, b = items[i]
            launch(k, bufs[b])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                launch(k, bufs[b])
            e1.record()
            torch.cuda.synchronize()
            times[(k, b)].append(e0.elapsed_time(e1) / args.reps)
    print(f"{'buffer':8s} " + " ".join(f"{k:>8s}" for k in kinds))
    for b in range(len(bufs)):
        print(f"buf{b:<5d} " + " ".join(f"{np.median(times[(k, b)]):8.4f}" for k in kinds), flush=True)
    for k in kinds:
        v = [np.median(times[(k, b)]) for b in range(len(bufs))]
        print(f"{k:8s} min {min(v):.4f} median {np.median(v):.4f} max {max(v):.4f} ms  spread {max(v) / min(v):.3f}")


if __name__ == "__main__":
    main()
