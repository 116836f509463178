"""A/B kernel variants on the BASELINE configs in ONE process (interleaved, randomised order, medians).

A variant is (library build, tuning knobs): the in-tree librtpb.so with its knobs (e.g. rays_per_lane=2)
and optional experiment builds of other sources or flags, e.g.
    python tools/exp_build.py --out ray_trace_pb_amd/exp_nocomp.so -DRTPB_EXP_NO_COMPUTE
(experiment builds may drop work -- they are never shipped).  Every variant's history is compared with the
first variant's (bit for bit, NaN pattern included) unless its library is marked inexact (name contains
"exp_nocomp").

    python tools/ab_variants.py --libs ray_trace_pb_amd/exp_prev.so --knobs rays_per_lane=1,2 \
        --configs c3:1.0,c2,c4:0.5,c5 --modes all,final
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


def fan(dev, pts, theta, nt, nph, wl, center=(0, 0, 1)):
    per = nt * nph
    x = torch.empty((per * len(pts), 8), dtype=torch.float64, device=dev)
    for k, p in enumerate(pts):
        rt.fan_into(x[k * per:(k + 1) * per], np.asarray(p, dtype=float), theta, nt, wl, nph, center)
    return x


def build_case(cfg, dev):
    """(system, m0, m1, float64 device rays, storage code) of a BASELINE config; cfg 'c3:0.5' scales the
    per-axis fan sizes."""
    name, _, sc = cfg.partition(":")
    scale = float(sc) if sc else 1.0
    if name == "c3":
        x = fan(dev, [[h, 0, 0] for h in systems.C3_FIELDS], np.pi / 180, int(3163 * scale), int(3162 * scale), 0.635)
        return systems.c3_system(rt, mat), mat.Vacuum(), mat.Vacuum(), x, C.RTPB_F32
    if name == "c4":
        theta = 30 * np.pi / 180
        x = fan(dev, [[1e-3, 1e-3, 1e-3 * np.tan(theta)]], np.arcsin(1.35 / systems.OPM_N1), int(10001 * scale),
                int(10000 * scale), systems.OPM_WAVELENGTH)
        return systems.c4_system(rt, mat), mat.Constant(systems.OPM_N1), mat.Vacuum(), x, C.RTPB_F32
    if name == "c5":
        pts = systems.c5_field_points(1)
        x = fan(dev, pts, 0.5 * np.pi / 180, int(3163 * scale), int(3162 * scale), 0.532)
        return systems.c5_system(rt, mat), mat.Constant(1), mat.Constant(1), x, C.RTPB_F64
    rays = systems.c2_rays(int(1_000_000 * scale))
    return systems.c2_system(rt, mat), mat.Vacuum(), mat.Vacuum(), torch.from_numpy(rays).to(dev), C.RTPB_F64


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--base", default="", help="library build to use as the base (default: in-tree)")
    ap.add_argument("--libs", default="", help="comma-separated extra library builds")
    ap.add_argument("--knobs", default="", help="knob=v1,v2 (in-tree library only)")
    ap.add_argument("--configs", default="c3:0.3,c2")
    ap.add_argument("--modes", default="all,final")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    C.lib()
    if args.base:
        C._lib = load(args.base)
    libs = {"base": C.lib()}
    for p in [p for p in args.libs.split(",") if p]:
        libs[os.path.basename(p).replace(".so", "")] = load(p)
    variants = [("base", None, None)]
    if args.knobs:
        k, _, vals = args.knobs.partition("=")
        variants = [("base", k, int(v)) for v in vals.split(",")]
    variants += [(ln, None, None) for ln in libs if ln != "base"]
    caches = {ln: collections.OrderedDict() for ln in libs}
    cases = []
    for cfg in args.configs.split(","):
        system, m0, m1, x, code = build_case(cfg, dev)
        S = len(system.surfaces)
        wl = np.unique(x[:, 7].cpu().numpy())
        low = E.lower(system.surfaces, [m0] + list(system.materials) + [m1], lambda: wl, code)
        for mode in args.modes.split(","):
            sel = E.resolve_planes(mode, S)
            w = 8 if code == C.RTPB_F64 else 4
            out = torch.empty((len(sel), x.shape[0], 8), dtype=torch.float64 if w == 8 else torch.float32, device=dev)
            nbytes = x.shape[0] * (64 + 8 * w * len(sel))
            cases.append((f"{cfg}/{mode}", low, x, sel, out, nbytes, x.shape[0] * S))

    def use(v):
        ln, k, val = v
        C._lib, E._PLANS = libs[ln], caches[ln]
        if k is not None:
            C.check(libs[ln].rtpb_set_tuning(k.encode(), val))
        return libs[ln]

    def vname(v):
        return v[0] + (f"[{v[1]}={v[2]}]" if v[1] else "")

    items = [(vi, ci) for vi in range(len(variants)) for ci in range(len(cases))]
    times = collections.defaultdict(list)
    rng = np.random.default_rng(0)
    for _ in range(args.rounds):
        for ii in rng.permutation(len(items)):
            vi, ci = items[ii]
            name, low, x, sel, out, _, _ = cases[ci]
            lib = use(variants[vi])
            E.trace_device(low, x, sel, out=out)
            torch.cuda.synchronize()
            lib.rtpb_timing_enable(1)
            for _ in range(args.reps):
                E.trace_device(low, x, sel, out=out)
            tot, cnt = ctypes.c_double(), ctypes.c_int64()
            C.check(lib.rtpb_timing_collect(ctypes.byref(tot), ctypes.byref(cnt)))
            lib.rtpb_timing_enable(0)
            times[(vi, ci)].append(tot.value / cnt.value)
    res = {"outputs_vs_first": {}}
    use(variants[0])
    for ci, (name, low, x, sel, out, nbytes, units) in enumerate(cases):
        base = float(np.median(times[(0, ci)]))
        for vi, v in enumerate(variants):
            ms = float(np.median(times[(vi, ci)]))
            res[f"{vname(v)}:{name}"] = {"ms": ms, "vs_first": ms / base, "GBps": nbytes / ms / 1e6,
                                         "frac_8TBs": nbytes / ms / 1e6 / 8000, "ray_surf_per_s": units / ms * 1e3}
            print(f"{vname(v):34s} {name:12s} ms={ms:8.4f} x{ms / base:.3f} {nbytes / ms / 1e6:7.0f} GB/s "
                  f"{units / ms * 1e3:.3e} ray-surf/s", flush=True)
    for ci, (name, low, x, sel, out, nbytes, units) in enumerate(cases):
        ref = None
        for vi, v in enumerate(variants):
            use(v)
            E.trace_device(low, x, sel, out=out)
            torch.cuda.synchronize()
            if ref is None:
                ref = out.clone()
                continue
            if "exp_no" in v[0]:
                continue
            same = all(bool(((a == b) | (torch.isnan(a) & torch.isnan(b))).all()) for a, b in zip(ref, out))
            res["outputs_vs_first"][f"{vname(v)}:{name}"] = "identical" if same else "DIFFERENT"
        del ref
    for k, v in res["outputs_vs_first"].items():
        print(f"{k}: {v}")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
