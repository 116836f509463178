"""Does the way the history buffer is allocated change the placement effect?  Allocates, alternately,
physically contiguous buffers (hipExtMallocWithFlags(hipDeviceMallocContiguous)) and ordinary torch
buffers, one C3 history each, then times the same C3 trace into every buffer, interleaved over rounds.

    python tools/placement_alloc.py [--pairs 3] [--scale 1.0] [--flag 4] [--kinds s64,s16] [--seed0 N]
"""
import argparse
import collections
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "tests", "golden")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from ray_trace_pb_amd import _capi as C  # noqa: E402
from ray_trace_pb_amd import _engine as E  # noqa: E402
import ab_variants  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=3)
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--flag", type=int, default=4, help="hipExtMallocWithFlags flags (4 = contiguous)")
    ap.add_argument("--kinds", default="contig,torch",
                    help="contig (hipDeviceMallocContiguous), torch, sN (history_buffer: chunks of N MiB mapped in shuffled order)")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--seed0", type=int, default=0, help="first history_buffer shuffle seed (0: the library's default sequence)")
    args = ap.parse_args()
    if args.seed0:
        import itertools
        E._buffer_seed = itertools.count(args.seed0)
    dev = torch.device("cuda:0")
    lib = C.lib()
    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    system, m0, m1, x, code = ab_variants.build_case(f"c3:{args.scale}", dev)
    n, S = x.shape[0], len(system.surfaces)
    low = E.lower(system.surfaces, [m0] + list(system.materials) + [m1], lambda: np.array([0.635]), code)
    sel = E.resolve_planes("all", S)
    P = len(sel)
    lo, hi = E.plane_mask(sel)
    nbytes = P * n * 32
    bufs, raw = {}, []
    import time
    for k in range(args.pairs):
        for kind in args.kinds.split(","):
            t0 = time.perf_counter()
            if kind == "contig":
                p = ctypes.c_void_p()
                rc = hip.hipExtMallocWithFlags(ctypes.byref(p), nbytes, args.flag)
                if rc != 0:
                    print(f"hipExtMallocWithFlags(flag {args.flag}) failed: {rc}", flush=True)
                else:
                    bufs[f"contig{k}"] = p.value
                    raw.append(p.value)
            elif kind == "torch":
                bufs[f"torch{k}"] = torch.empty((P, n, 8), dtype=torch.float32, device=dev)
            else:
                # the product's history buffer (rtpb_buffer_alloc) with N MiB chunks in shuffled order
                bufs[f"{kind}_{k}"] = E.history_buffer((P, n, 8), torch.float32, dev, chunk_bytes=int(kind[1:]) << 20)
            torch.cuda.synchronize()
            print(f"alloc {kind}{k}: {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)
    h = ctypes.c_void_p()
    C.check(lib.rtpb_plan_create(low.surfaces, low.nsurf, low.materials, low.nsurf + 1, low.dtype, ctypes.byref(h)))
    stream = torch.cuda.current_stream(dev).cuda_stream

    def ptr(b):
        return b if isinstance(b, int) else b.data_ptr()

    def trace(b):
        C.check(lib.rtpb_trace(h, 0, x.data_ptr(), C.RTPB_F64, n, C.RTPB_AOS, 0, ptr(b), C.RTPB_AOS, n * 8, 0, lo, hi,
                               stream))

    names = list(bufs)
    times = collections.defaultdict(list)
    rng = np.random.default_rng(0)
    for _ in range(args.rounds):
        for i in rng.permutation(len(names)):
            b = bufs[names[i]]
            trace(b)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                trace(b)
            e1.record()
            torch.cuda.synchronize()
            times[names[i]].append(e0.elapsed_time(e1) / args.reps)
    for name in names:   # allocation order
        print(f"{name:10s} ms={np.median(times[name]):.4f} ({', '.join(f'{t:.3f}' for t in times[name])})", flush=True)
    for p in raw:
        hip.hipFree(p)


if __name__ == "__main__":
    main()
