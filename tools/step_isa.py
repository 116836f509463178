"""Static VALU cost of single surface steps: compiles one small gfx950 kernel per (kind, geometry form) -- load a
ray, run surface_step (rtpb_math.h) with both planes stored, store them -- and prints the VALU instruction count of
each kernel, split into the fall-through (likely) path and the out-of-line blocks, plus a histogram of opcodes on the
likely path.  The history kernels' PMC counts (tools/history_kind_cost.py) are the measured numbers; this shows
where they come from without a GPU.

    python tools/step_isa.py                      # summary table
    python tools/step_isa.py --show flat_xz       # that kernel's likely-path assembly
"""
import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ray_trace_pb_amd import _build  # noqa: E402

CASES = {                      # name: (kind constant, geometry form)
    "flat_gen": ("FLAT", "kGeoGeneral"),
    "flat_xz": ("FLAT", "kGeoXZ"),
    "flat_ax": ("FLAT", "kGeoAxial"),
    "lens_gen": ("PERFECT_LENS", "kGeoGeneral"),
    "lens_xz": ("PERFECT_LENS", "kGeoXZ"),
    "lens_ax": ("PERFECT_LENS", "kGeoAxial"),
    "sphere_gen": ("SPHERE", "kGeoGeneral"),
    "sphere_ax": ("SPHERE", "kGeoAxial"),
}

SRC = r'''
#include "rtpb_internal.h"
using namespace rtpbi;
template <int KIND, int GEO>
__global__ __launch_bounds__(64) void step_kernel(const double* __restrict__ in, cptr<DevSurface<double>> sp,
                                                  double n1, double n2, double* __restrict__ out) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    const Ray<double> r = load_ray<double, RTPB_AOS>(in, i, 0);
    const Rcp<double> iwl = make_wl_rcp(r.wl);
    const DevSurface<double> s = load_surface<double>(sp);
    Ray<double> after;
    surface_step<double, KIND, GEO>(s, r, n1, n2, iwl, [&](const Ray<double>& at) {
        store_ray<double, RTPB_AOS>(out, 2 * i, 0, at); }, after);
    store_ray<double, RTPB_AOS>(out, 2 * i + 1, 0, after);
}
'''

FUNC = re.compile(r"^(_Z\S+):\s*(;.*)?$")
LABEL = re.compile(r"^(\.LBB\S+):")
BRANCH = re.compile(r"^\s*s_(cbranch_\S+|branch)\s+(\S+)")


def compile_all():
    src = SRC + "".join(f"template __global__ void step_kernel<{k}, {g}>(const double* __restrict__, "
                        f"cptr<DevSurface<double>>, double, double, double* __restrict__);\n"
                        for k, g in CASES.values())
    d = tempfile.mkdtemp(prefix="step_isa_")
    path = os.path.join(d, "steps.hip")
    with open(path, "w") as f:
        f.write(src)
    flags = [f for f in _build.FLAGS if f != "-fPIC"] + ["-I", _build.CSRC]
    out = os.path.join(d, "steps.s")
    subprocess.run([_build.HIPCC] + flags + ["--cuda-device-only", "-S", "-o", out, path], check=True)
    return open(out).read().splitlines()


def functions(lines):
    funcs, cur = {}, None
    for ln in lines:
        m = FUNC.match(ln)
        if m:
            cur = m.group(1)
            funcs[cur] = []
            continue
        if cur is not None:
            if ln.strip().startswith(".Lfunc_end"):
                cur = None
                continue
            funcs[cur].append(ln)
    return funcs


def blocks(body):
    """[(label, [instruction lines])] in layout order."""
    out, label, ins = [], "entry", []
    for ln in body:
        m = LABEL.match(ln)
        if m:
            out.append((label, ins))
            label, ins = m.group(1), []
            continue
        s = ln.strip()
        if not s or s.startswith((";", ".")):
            continue
        ins.append(s)
    out.append((label, ins))
    return out


def likely_path(blks):
    """Blocks reached from the entry when every conditional branch falls through (the compiler lays the
    __builtin_expect-likely code out as the fall-through), following unconditional branches."""
    index = {lab: k for k, (lab, _) in enumerate(blks)}
    k, seen, path = 0, set(), []
    while k < len(blks) and k not in seen:
        seen.add(k)
        lab, ins = blks[k]
        path.append(k)
        nxt = k + 1
        for s in ins:
            m = BRANCH.match(s)
            if m and m.group(1) == "branch":
                nxt = index.get(m.group(2), len(blks))
                break
            if s.startswith("s_endpgm"):
                nxt = len(blks)
                break
        k = nxt
    return path


def is_valu(s):
    return s.startswith("v_") and not s.startswith(("v_readfirstlane", "v_readlane", "v_writelane"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--show", default="")
    a = ap.parse_args()
    funcs = {n: b for n, b in functions(compile_all()).items() if "step_kernel" in n}
    names = list(funcs)           # instantiation order == CASES order
    if len(names) != len(CASES):
        sys.exit(f"expected {len(CASES)} kernels, found {len(names)}")
    for (case, _), name in zip(CASES.items(), names):
        blks = blocks(funcs[name])
        path = likely_path(blks)
        on = [s for k in path for s in blks[k][1] if is_valu(s)]
        off = [s for k in range(len(blks)) if k not in path for s in blks[k][1] if is_valu(s)]
        hist = collections.Counter(s.split()[0] for s in on)
        f64 = sum(v for op, v in hist.items() if op.endswith("_f64"))
        print(f"{case:11s} VALU likely path {len(on):4d} (f64 {f64:3d})   out of line {len(off):4d}   "
              f"blocks {len(blks)}")
        if a.show == case:
            for k in path:
                print(f"  -- {blks[k][0]}")
                for s in blks[k][1]:
                    print("    " + s)
            for op, v in hist.most_common():
                print(f"    {op:28s} {v}")


if __name__ == "__main__":
    main()
