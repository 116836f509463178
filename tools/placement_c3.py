"""Placement of the C3 history: the same full-size C3 trace (50,007,030 float64 rays -> 19 float32 planes,
30.4 GB) into several separately allocated output buffers, and into buffers whose plane stride is padded
by a few rays (the (P, N, 8) view keeps the drop-in indexing), interleaved over rounds; plus a plain
fill of each buffer.  A per-buffer spread that stays put across rounds is physical placement.

    python tools/placement_c3.py [--buffers 4] [--pads 64,4096,65537] [--scale 1.0] [--libs a.so,b.so]

--libs adds experiment builds: every (library, buffer) pair is timed, interleaved, so a change of the
kernel's write order can be judged over several placements instead of one.
"""
import argparse
import collections
import ctypes
import json
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
    ap.add_argument("--buffers", type=int, default=4)
    ap.add_argument("--pads", default="64,4096,65537", help="extra rays per plane (plane-stride padding)")
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--libs", default="")
    ap.add_argument("--rays-copy", action="store_true",
                    help="also trace from a copy of the input rays allocated after the buffers")
    ap.add_argument("--sequential", action="store_true",
                    help="buffers in allocation order, no interleaving (per-dispatch PMC attribution)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    libs = {"base": C.lib()}
    for path in [q for q in args.libs.split(",") if q]:
        libs[os.path.basename(path).replace(".so", "")] = ab_variants.load(path)
    system, m0, m1, x, code = ab_variants.build_case(f"c3:{args.scale}", dev)
    n, S = x.shape[0], len(system.surfaces)
    low = E.lower(system.surfaces, [m0] + list(system.materials) + [m1], lambda: np.array([0.635]), code)
    sel = E.resolve_planes("all", S)
    P = len(sel)
    lo, hi = E.plane_mask(sel)
    bufs = {}
    for k in range(args.buffers):
        bufs[f"plain{k}"] = (torch.empty((P, n, 8), dtype=torch.float32, device=dev), n)
    for pad in [int(p) for p in args.pads.split(",") if p]:
        b = torch.empty((P, n + pad, 8), dtype=torch.float32, device=dev)
        bufs[f"pad{pad}"] = (b, n + pad)
    stream = torch.cuda.current_stream(dev).cuda_stream
    inputs = {"": x}
    if args.rays_copy:
        inputs["@rays2"] = x.clone()
    plans = {}
    for ln, lib in libs.items():
        h = ctypes.c_void_p()
        C.check(lib.rtpb_plan_create(low.surfaces, low.nsurf, low.materials, low.nsurf + 1, low.dtype,
                                     ctypes.byref(h)))
        plans[ln] = h

    def trace(buf, stride_rays, ln="base", xin=x):
        C.check(libs[ln].rtpb_trace(plans[ln], 0, xin.data_ptr(), C.RTPB_F64, n, C.RTPB_AOS, 0, buf.data_ptr(),
                                    C.RTPB_AOS, stride_rays * 8, 0, lo, hi, stream))

    times, fills = collections.defaultdict(list), collections.defaultdict(list)
    rng = np.random.default_rng(0)
    names = list(bufs)
    items = [(ln + xs, name) for ln in libs for xs in inputs for name in names]
    for _ in range(args.rounds):
        order = range(len(items)) if args.sequential else rng.permutation(len(items))
        for lnx, name in [items[i] for i in order]:
            ln, _, xs = lnx.partition("@")
            xin = inputs["@" + xs] if xs else x
            buf, stride = bufs[name]
            lib = libs[ln]
            trace(buf, stride, ln, xin)
            torch.cuda.synchronize()
            lib.rtpb_timing_enable(1)
            for _ in range(args.reps):
                trace(buf, stride, ln, xin)
            tot, cnt = ctypes.c_double(), ctypes.c_int64()
            C.check(lib.rtpb_timing_collect(ctypes.byref(tot), ctypes.byref(cnt)))
            lib.rtpb_timing_enable(0)
            times[(lnx, name)].append(tot.value / cnt.value)
            if lnx != "base":
                continue
            flat = buf.view(-1)
            chunks = [flat[k:k + (1 << 30)] for k in range(0, flat.numel(), 1 << 30)]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for c in chunks:
                c.fill_(0.0)
            e1.record()
            torch.cuda.synchronize()
            fills[name].append(flat.numel() * 4 / (e0.elapsed_time(e1) * 1e-3) / 1e9)
    # every library / padded / separately allocated trace gives the same history (compare against plain0)
    ref, _ = bufs["plain0"]
    trace(ref, n)
    torch.cuda.synchronize()
    ref = ref.clone()
    res = {"rays": n, "planes": P, "alg_bytes": n * (64 + 32 * P)}
    for lnx in dict.fromkeys(i[0] for i in items):
        ln = lnx.partition("@")[0]
        for name in names:
            buf, stride = bufs[name]
            trace(buf, stride, ln)
            torch.cuda.synchronize()
            same = all(bool(((a == b) | (torch.isnan(a) & torch.isnan(b))).all()) for a, b in zip(ref, buf[:, :n]))
            ms = float(np.median(times[(lnx, name)]))
            res[f"{lnx}:{name}"] = {"ms": ms, "ms_all": [round(t, 4) for t in times[(lnx, name)]],
                                   "alg_GBps": res["alg_bytes"] / ms / 1e6,
                                   "fill_GBps": float(np.median(fills[name])), "identical": same}
            print(f"{lnx:12s} {name:10s} ms={ms:.4f} ({', '.join(f'{t:.3f}' for t in times[(lnx, name)])}) "
                  f"{res['alg_bytes'] / ms / 1e6:.0f} GB/s  fill {np.median(fills[name]):.0f} GB/s  same={same}",
                  flush=True)
        ms = [res[f"{lnx}:{name}"]["ms"] for name in names]
        print(f"{lnx:12s} over buffers: min {min(ms):.4f} median {float(np.median(ms)):.4f} max {max(ms):.4f} ms",
              flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
