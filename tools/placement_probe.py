"""Does the trace time depend on WHERE the output history lives?  Several output buffers of the same
shape are allocated (with differently sized spacer allocations between them), then the same trace is timed
into each, interleaved over rounds (HIP events from librtpb's timing counters).  A spread between buffers
that stays put across rounds points at physical placement (channel / page mapping, translation reach),
not at the kernel.

    python tools/placement_probe.py [--configs c5,c2] [--buffers 6]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c5,c2")
    ap.add_argument("--buffers", type=int, default=6)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rays", type=int, default=1_000_000)
    ap.add_argument("--libs", default="", help="comma list of experiment builds timed on the same buffers")
    ap.add_argument("--kinds", default="torch,hipExtMalloc,contiguous")
    ap.add_argument("--tunings", default="", help="comma list of knob=value variants of the base library "
                                                   "(rtpb_set_tuning), e.g. nt_stores=0")
    ap.add_argument("--order", default="random", choices=["random", "seq"],
                    help="seq: buffers in allocation order (PMC runs map dispatches to buffers by index)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    libs = {"base": C.lib()}
    for p in filter(None, args.libs.split(",")):
        h = ctypes.CDLL(os.path.abspath(p))
        for name, (restype, argt) in C.SIGNATURES.items():
            fn = getattr(h, name)
            fn.restype, fn.argtypes = restype, argt
        libs[os.path.basename(p).replace(".so", "")] = h
    hip = ctypes.CDLL("libamdhip64.so")      # the runtime torch (and librtpb) already loaded
    hip.hipExtMallocWithFlags.restype = ctypes.c_int
    hip.hipFree.restype = ctypes.c_int
    recipes = {"c2": lambda: (systems.c2_system(rt, mat), systems.c2_rays(args.rays), mat.Vacuum(), mat.Vacuum()),
               "c5": lambda: (systems.c5_system(rt, mat),
                              systems.c5_rays(rt, 1, 101, max(1, args.rays // 707)), mat.Constant(1), mat.Constant(1))}
    res = {}
    rng = np.random.default_rng(0)
    for cfg in args.configs.split(","):
        system, rays_np, m0, m1 = recipes[cfg]()
        S = len(system.surfaces)
        low = E.lower(system.surfaces, [m0] + list(system.materials) + [m1], lambda: np.unique(rays_np[:, 7]),
                      C.RTPB_F64)
        x = torch.from_numpy(rays_np).to(dev)
        sel = E.resolve_planes("all", S)
        nbytes = len(sel) * x.shape[0] * 8 * 8
        outs, spacers, kinds = [], [], []
        kinds_on = args.kinds.split(",")
        for b in range(args.buffers if "torch" in kinds_on else 0):
            spacers.append(torch.empty(int(rng.integers(1, 64)) << 20, dtype=torch.uint8, device=dev))
            t = torch.empty((len(sel), x.shape[0], 8), dtype=torch.float64, device=dev)
            outs.append((t.data_ptr(), t))
            kinds.append("torch")
        for flag, name in ((0, "hipExtMalloc"), (4, "contiguous")):
            for b in range(args.buffers // 2 if name in kinds_on else 0):
                ptr = ctypes.c_void_p()
                rc = hip.hipExtMallocWithFlags(ctypes.byref(ptr), ctypes.c_size_t(nbytes), ctypes.c_uint(flag))
                if rc != 0:
                    print(f"{name}: hipExtMallocWithFlags rc={rc}", flush=True)
                    break
                outs.append((ptr.value, None))
                kinds.append(name)
        lo, hi = E.plane_mask(sel)

        caches = {k: collections.OrderedDict() for k in libs}

        def run(lib, ptr):
            C._lib, E._PLANS = lib, caches[[k for k in libs if libs[k] is lib][0]]
            with E.plan_ref(low) as plan:
                C.check(lib.rtpb_trace(plan, 0, x.data_ptr(), E.input_code(x.dtype), x.shape[0], C.RTPB_AOS, 0, ptr, C.RTPB_AOS,
                                       8 * x.shape[0], x.shape[0], lo, hi, torch.cuda.current_stream().cuda_stream))
        tun = {ln: (None, None) for ln in libs}
        for t in filter(None, args.tunings.split(",")):
            knob, val = t.split("=")
            libs[f"base+{t}"] = libs["base"]
            tun[f"base+{t}"] = (knob.encode(), int(val))
        defaults = {"aos_staging": 1, "nt_stores": 1, "stage_input": 0}
        items = [(ln, b) for ln in libs for b in range(len(outs))]
        times = {it: [] for it in items}
        for _ in range(args.rounds):
            for ii in (rng.permutation(len(items)) if args.order == "random" else range(len(items))):
                ln, b = items[ii]
                lib = libs[ln]
                knob, val = tun[ln]
                if knob:
                    C.check(lib.rtpb_set_tuning(knob, val))
                run(lib, outs[b][0])
                torch.cuda.synchronize()
                lib.rtpb_timing_enable(1)
                for _ in range(args.reps):
                    run(lib, outs[b][0])
                tot, cnt = ctypes.c_double(), ctypes.c_int64()
                C.check(lib.rtpb_timing_collect(ctypes.byref(tot), ctypes.byref(cnt)))
                lib.rtpb_timing_enable(0)
                if knob:
                    C.check(lib.rtpb_set_tuning(knob, defaults[knob.decode()]))
                times[(ln, b)].append(tot.value / cnt.value)
        C._lib, E._PLANS = libs["base"], caches["base"]
        # the same buffers written by a plain fill (one contiguous stream): is the spread the kernel's?
        fill_ms = []
        for b in range(len(outs)):
            t = outs[b][1]
            if t is None:
                fill_ms.append(float("nan"))
                continue
            ms = []
            for _ in range(args.rounds):
                t.fill_(1.0)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    t.fill_(1.0)
                e1.record()
                torch.cuda.synchronize()
                ms.append(e0.elapsed_time(e1) / args.reps)
            fill_ms.append(float(np.median(ms)))
        bytes_ = x.shape[0] * 64 * (1 + len(sel))
        res[cfg] = {}
        for ln in libs:
            med = [float(np.median(times[(ln, b)])) for b in range(len(outs))]
            for b in range(len(outs)):
                t = times[(ln, b)]
                print(f"{cfg} {ln:14s} buffer {b} {kinds[b]:12s} addr=0x{outs[b][0]:x} ms median={med[b]:.4f} "
                      f"min={min(t):.4f} max={max(t):.4f} GB/s={bytes_ / med[b] / 1e6:.0f}  "
                      f"fill ms={fill_ms[b]:.4f} GB/s={nbytes / fill_ms[b] / 1e6:.0f}", flush=True)
            print(f"{cfg} {ln:14s} mean over buffers {np.mean(med):.4f} ms", flush=True)
            res[cfg][ln] = {"ms_median_per_buffer": med, "kinds": kinds, "mean": float(np.mean(med)),
                            "spread": max(med) / min(med)}
        torch.cuda.synchronize()
        for (ptr, t), k in zip(outs, kinds):
            if t is None:
                hip.hipFree(ctypes.c_void_p(ptr))
        del outs, spacers
        torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
