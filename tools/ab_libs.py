"""A/B several builds of librtpb.so in ONE process (interleaved, randomised order, median of rounds).

Each extra library is an experiment build of the same sources, e.g.
    python tools/exp_build.py --out ray_trace_pb_amd/exp_noons.so -DRTPB_EXP_NO_ONSURFACE
(`-DRTPB_EXP_NO_ONSURFACE` drops work and is NOT bit-exact) -- used only to find where kernel time goes,
never shipped.

    python tools/ab_libs.py ray_trace_pb_amd/exp_X.so ... [--rays N] [--configs c2,c5]
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


def load(path):
    h = ctypes.CDLL(os.path.abspath(path))          # RTLD_LOCAL: each build keeps its own symbols/kernels
    for name, (res, argt) in C.SIGNATURES.items():
        fn = getattr(h, name, None)          # an older build may lack newer entry points
        if fn is not None:
            fn.restype, fn.argtypes = res, argt
    return h


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*")
    ap.add_argument("--rays", type=int, default=1_000_000)
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--configs", default="c2,c5")
    ap.add_argument("--dtypes", default="f64")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    libs = {"base": C.lib()}
    for p in args.libs:
        libs[os.path.basename(p).replace(".so", "")] = load(p)
    recipes = {"c2": lambda: (systems.c2_system(rt, mat), systems.c2_rays(args.rays), mat.Vacuum(), mat.Vacuum()),
               "c5": lambda: (systems.c5_system(rt, mat),
                              systems.c5_rays(rt, 1, 101, max(1, args.rays // 707)), mat.Constant(1), mat.Constant(1)),
               "c3": lambda: (systems.c3_system(rt, mat), systems.c3_rays(rt, 1001, max(1, args.rays // 5005)),
                              mat.Vacuum(), mat.Vacuum()),
               "c4": lambda: (systems.c4_system(rt, mat), systems.c4_rays(rt, 1001, max(1, args.rays // 1001)),
                              mat.Constant(systems.OPM_N1), mat.Vacuum())}
    cases = []
    for cfg in args.configs.split(","):
        system, rays_np, m0, m1 = recipes[cfg]()
        S = len(system.surfaces)
        for dtype in args.dtypes.split(","):
            code = C.RTPB_F64 if dtype == "f64" else C.RTPB_F32
            tdt = torch.float64 if dtype == "f64" else torch.float32
            low = E.lower(system.surfaces, [m0] + list(system.materials) + [m1], lambda: np.unique(rays_np[:, 7]), code)
            x = torch.from_numpy(rays_np).to(dev, dtype=tdt)
            for planes in ("all", "final"):
                sel = E.resolve_planes(planes, S)
                out = torch.empty((len(sel), x.shape[0], 8), dtype=tdt, device=dev)
                cases.append((f"{cfg}/{dtype}/{planes}", low, x, sel, out))
    caches = {k: collections.OrderedDict() for k in libs}
    items = [(ln, c) for ln in libs for c in range(len(cases))]
    times = collections.defaultdict(list)
    rng = np.random.default_rng(0)
    for _ in range(args.rounds):
        for ii in rng.permutation(len(items)):
            ln, ci = items[ii]
            name, low, x, sel, out = cases[ci]
            C._lib, E._PLANS = libs[ln], caches[ln]
            lib = libs[ln]
            E.trace_device(low, x, sel, out=out)
            torch.cuda.synchronize()
            lib.rtpb_timing_enable(1)
            for _ in range(args.reps):
                E.trace_device(low, x, sel, out=out)
            tot, cnt = ctypes.c_double(), ctypes.c_int64()
            C.check(lib.rtpb_timing_collect(ctypes.byref(tot), ctypes.byref(cnt)))
            lib.rtpb_timing_enable(0)
            times[(ln, name)].append(tot.value / cnt.value)
    # every build must produce the same history as the base build (NaN where it has NaN, equal elsewhere)
    mism = {}
    for name, low, x, sel, out in cases:
        ref = None
        for ln in libs:
            C._lib, E._PLANS = libs[ln], caches[ln]
            E.trace_device(low, x, sel, out=out)
            torch.cuda.synchronize()
            got = out.clone()
            if ref is None:
                ref = got
                continue
            nan_r, nan_g = torch.isnan(ref), torch.isnan(got)
            same = torch.equal(nan_r, nan_g) and torch.equal(ref[~nan_r], got[~nan_g])
            mism[f"{ln}:{name}"] = "identical" if same else "DIFFERENT"
            print(f"{ln:24s} {name:16s} output vs base: {mism[f'{ln}:{name}']}")
    C._lib, E._PLANS = libs["base"], caches["base"]
    res = {"outputs_vs_base": mism}
    for name, *_ in cases:
        base = float(np.median(times[("base", name)]))
        for ln in libs:
            ms = float(np.median(times[(ln, name)]))
            res[f"{ln}:{name}"] = {"ms": ms, "vs_base": ms / base}
            print(f"{ln:24s} {name:16s} ms={ms:.4f}  x{ms / base:.3f}")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
