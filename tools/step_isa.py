"""Static VALU cost of single surface steps: compiles one small gfx950 kernel per (kind, geometry form) -- load a
ray, run surface_step (rtpb_math.h) with both planes stored, store them -- and prints the VALU instruction count of
each kernel, split into the fall-through (likely) path and the out-of-line blocks, plus a histogram of opcodes on the
likely path.  The history kernels' PMC counts (tools/history_kind_cost.py) are the measured numbers; this shows
where they come from without a GPU.

    python tools/step_isa.py                      # summary table
    python tools/step_isa.py --show flat_xz       # that kernel's likely-path assembly
    python tools/step_isa.py --kernel             # the same forms inside the C4 history kernel's surface loop
    python tools/step_isa.py --kernel --show lens_xz

--kernel compiles the shipped history kernel (trace_kernel, the C4 variant: float64 input, float32 AOS history,
LDS-staged non-temporal stores, PerfectLens code) from a scratch copy of csrc/ whose dispatch_kind always takes one
(kind, geometry form), and counts the VALU of one surface-loop iteration on the fast path -- the per-surface cost
tools/history_kind_cost.py measures with PMC, without a GPU (the kernel's loop runs two surfaces per iteration, so
--kernel reports half an iteration).
"""
import argparse
import collections
import os
import re
import shutil
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

# Every __builtin_expect-hinted branch of the headers becomes an assumption that the hinted side is taken, so the
# compiler drops the rare-lane code (the full division / square-root sequences of the exact fast paths); what is
# left is the code a wave runs when all its lanes stay on the fast paths
SRC = r'''
#define __builtin_expect(c, v) ({ const bool c_ = (c); if (c_ != static_cast<bool>(v)) __builtin_unreachable(); c_; })
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

EXPECT_FAST = ("#define __builtin_expect(c, v) ({ const bool c_ = (c); if (c_ != static_cast<bool>(v)) "
               "__builtin_unreachable(); c_; })")
KERNEL_SRC = r'''
#define __builtin_expect(c, v) ({ const bool c_ = (c); if (c_ != static_cast<bool>(v)) __builtin_unreachable(); c_; })
#include "rtpb_trace_kernel.h"
namespace rtpbi {
template __global__ void trace_kernel<double, float, RTPB_AOS, RTPB_AOS, STORE_BITS, 1, 1>(TraceArgs<double, float>);
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


SWEEP_SRC = r'''
#define __builtin_expect(c, v) ({ const bool c_ = (c); if (c_ != static_cast<bool>(v)) __builtin_unreachable(); c_; })
#include "rtpb_analysis.hip"
'''


def compile_kernel(kind, geo, sweep=False, guards=False, final=False):
    """The C4 history kernel (or, sweep=True, the C5 spot-sweep kernels) with every surface dispatched to
    (kind, geo)."""
    d = tempfile.mkdtemp(prefix="step_isa_k_")
    csrc = os.path.join(d, "csrc")
    shutil.copytree(_build.CSRC, csrc, ignore=shutil.ignore_patterns("_obj", "*.o", "*.so"))
    math_h = os.path.join(csrc, "rtpb_math.h")
    text = open(math_h).read()
    head = ("RTPB_HD void dispatch_code(int code, Step&& step) {\n" if sweep else
            "RTPB_HD void dispatch_kind(const DevSurface<T>& s, Step&& step) {\n")
    if head not in text:
        sys.exit("dispatcher not found in rtpb_math.h")
    text = text.replace(head, head + f"    step(std::integral_constant<int, {kind}>(), std::integral_constant<int, {geo}>());"
                                     "\n    return;\n", 1)
    # C4's media: Constant materials, uniform Snell ratios and lens constants from the descriptor
    for a, b in (("        if (s.rcp_ok & kLensUni) {", "        if (true) {"),
                 ("            if (s.rcp_ok & kRPos) {", "            if (true) {"),
                 ("            } else if (s.rcp_ok & 4) {", "            } else if (true) {"),
                 ("    if (s.rcp_ok & 8) {", "    if (true) {")):
        if a not in text:
            sys.exit(f"rtpb_math.h: {a.strip()!r} not found")
        text = text.replace(a, b, 1)
    open(math_h, "w").write(text)
    kern_h = os.path.join(csrc, "rtpb_trace_kernel.h")
    ktext = open(kern_h).read()
    a = "    auto mat_n = [&](cptr<DevMaterial<T>> mp) -> T {\n"
    if a not in ktext:
        sys.exit("rtpb_trace_kernel.h: mat_n not found")
    open(kern_h, "w").write(ktext.replace(a, a + "        if (true) return load_material<T>(mp).c[0];\n", 1))
    path = os.path.join(csrc, "one_kernel.hip")
    with open(path, "w") as f:
        src = SWEEP_SRC if sweep else KERNEL_SRC.replace("STORE_BITS", "11" if final else "3")
        if guards:   # the shipped code: guard tests, branches and the rare lanes' full sequences
            src = src.replace(EXPECT_FAST, "")
        f.write(src)
    flags = [f for f in _build.FLAGS if f != "-fPIC"] + ["-I", csrc, "-Wno-unused-variable", "-Wno-unused-parameter"]
    out = os.path.join(d, "k.s")
    subprocess.run([_build.HIPCC] + flags + ["--cuda-device-only", "-S", "-o", out, path], check=True,
                   stderr=subprocess.DEVNULL)
    return open(out).read().splitlines()


def label_comments(body):
    """[(line index, label, the label line's comment with the comment-only lines right after it)]."""
    out = []
    for i, ln in enumerate(body):
        m = LABEL.match(ln) or re.match(r"^; %bb\.(\d+):", ln)
        if not m:
            continue
        text, j = ln, i + 1
        while j < len(body) and body[j].strip().startswith(";") and not re.match(r"^; %bb\.", body[j]):
            text += " " + body[j].strip()
            j += 1
        out.append((i, m.group(1), text))
    return out


def loop_blocks(body, depth=1):
    """[(label, [instructions])] of the loops at `depth` (the history kernel's surface loop: 1) in layout order: the
    blocks whose label comment puts them in a loop at that depth ('in Loop: ... Depth=<depth>' or that loop's
    header)."""
    heads = label_comments(body)
    out = []
    for n, (i, lab, text) in enumerate(heads):
        if not re.search(rf"(in Loop: Header=\S+|Loop Header:) Depth={depth}\b", text):
            continue
        end = heads[n + 1][0] if n + 1 < len(heads) else len(body)
        ins = [x.strip() for x in body[i + 1:end]
               if x.strip() and not x.strip().startswith((";", "."))]
        out.append((lab, ins))
    return out


def header_of(body, depth):
    """The label of the (first) loop header at `depth`."""
    for i, lab, text in label_comments(body):
        if re.search(rf"Loop Header: Depth={depth}\b", text):
            return lab
    return None


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


SLOW = ("v_div_scale", "v_ldexp")       # the compiler's full division / square-root sequences (the slow paths)


def is_fill(ins):
    """A NaN fill (kill_if): only moves, one of them the NaN high word."""
    vals = [s for s in ins if s.startswith("v_")]
    return bool(vals) and all(s.startswith("v_mov") for s in vals) and any("0x7ff80000" in s for s in vals)


def likely_path(blks):
    """The blocks a wave runs when every lane takes the fast paths and no row is killed: an execnz branch (to the
    out-of-line code of rare lanes) is not taken; any other conditional forward branch is taken when the code it
    skips holds a full division / square-root sequence or a NaN fill (a slow path or a kill), else not; unconditional
    branches are followed."""
    index = {lab: k for k, (lab, _) in enumerate(blks)}
    k, seen, path = 0, set(), []
    while k < len(blks) and k not in seen:
        seen.add(k)
        lab, ins = blks[k]
        path.append(k)
        nxt = k + 1
        for s in ins:
            m = BRANCH.match(s)
            if m:
                kind, target = m.group(1), index.get(m.group(2), len(blks))
                if kind == "branch":
                    nxt = target
                    break
                if kind.startswith("cbranch_execnz") or target <= k:
                    continue
                skipped = [x for j in range(k + 1, target) for x in blks[j][1]]
                if any(x.startswith(SLOW) for x in skipped) or is_fill(skipped):
                    nxt = target
                    break
            if s.startswith("s_endpgm"):
                nxt = len(blks)
                break
        k = nxt
    return path


def is_valu(s):
    return s.startswith("v_") and not s.startswith(("v_readfirstlane", "v_readlane", "v_writelane"))


def kernel_main(show, final=False):
    for case, (kind, geo) in CASES.items():
        funcs = {n: b for n, b in functions(compile_kernel(kind, geo, final=final)).items() if "trace_kernel" in n}
        (name, body), = funcs.items()
        blks = loop_blocks(body)
        # every loop block but the NaN fills (kills: rows of the wave that fail a test) runs on the fast path of a
        # C4 surface with both planes stored
        on = [x for lab, ins in blks if not is_fill(ins) for x in ins if is_valu(x)]
        hist = collections.Counter(x.split()[0] for x in on)
        f64 = sum(v for op, v in hist.items() if "_f64" in op and not op.startswith(("v_cmp", "v_frexp", "v_cvt")))
        movs = sum(v for op, v in hist.items() if op.startswith("v_mov"))
        g_funcs = {n: b for n, b in functions(compile_kernel(kind, geo, guards=True, final=final)).items()
                   if "trace_kernel" in n}
        (gname, gbody), = g_funcs.items()
        guarded = [x for x in guarded_walk(loop_blocks(gbody, 1), header_of(gbody, 1)) if not x.startswith("v_cvt")]
        on = [x for x in on if not x.startswith("v_cvt")]
        # the surface loop runs two surfaces per iteration (rtpb_trace_kernel.h): per surface = half
        print(f"{case:11s} per surface VALU (+{0 if final else 16} cvt) {len(on) / 2:6.1f} fast path, "
              f"{len(guarded) / 2:6.1f} with the guards  (f64 arithmetic {f64 / 2:5.1f}, moves {movs / 2:4.1f}, "
              f"loop blocks {len(blks)})", flush=True)
        if show == case + "+g":
            for x in guarded:
                print("    " + x)
        if show == case:
            for lab, ins in blks:
                print(f"  -- {lab}{'  (fill)' if is_fill(ins) else ''}")
                for x in ins:
                    print("    " + x)
            for op, v in hist.most_common():
                print(f"    {op:28s} {v}")


def guarded_walk(blks, header):
    """VALU of one loop iteration of the shipped code (guards compiled in), from the loop header, when every lane
    stays on the fast paths: an execnz branch (rare lanes' out-of-line code) is not taken; the else side of an if
    (s_andn2_saveexec, execz) runs when its then side went out of line (an execnz just before), else it is skipped;
    any other exec-mask branch skips code that starts with a full division / square-root sequence or is a NaN fill;
    wave-uniform branches (scc / vcc: loop control, plane stores) fall through; a branch back to the header ends the
    iteration.  Plane stores under uniform branches are not followed (the
    float32 conversions are counted apart)."""
    index = {lab: k for k, (lab, _) in enumerate(blks)}
    k, seen, out = index[header], set(), []
    while k < len(blks) and k not in seen:
        seen.add(k)
        nxt = k + 1
        ins = blks[k][1]
        for i, x in enumerate(ins):
            if is_valu(x):
                out.append(x)
            m = BRANCH.match(x)
            if not m:
                continue
            kind, target = m.group(1), m.group(2)
            if target == header:
                if kind == "branch":
                    return out
                continue
            t = index.get(target)
            if kind == "branch":
                nxt = t if t is not None else len(blks)
                break
            if kind.startswith("cbranch_execnz") or t is None or t <= k:
                continue
            if kind.startswith(("cbranch_scc", "cbranch_vcc")):
                continue        # wave-uniform control (loop tail, plane stores): the surface's own code follows
            if kind.startswith("cbranch_execz") and any(y.startswith("s_andn2_saveexec") for y in ins[:i]):
                prev = blks[k - 1][1] if k > 0 else []
                then_out_of_line = any(y.startswith("s_cbranch_execnz") for y in ins[:i] + prev)
                if not then_out_of_line:
                    nxt = t
                    break
                continue
            skipped = [y for j in range(k + 1, t) for y in blks[j][1]]
            first = blks[k + 1][1] if k + 1 < t else []
            if any(y.startswith(SLOW) for y in first) or is_fill(skipped):
                nxt = t
                break
        k = nxt
    return out


def sweep_main(show):
    """The C5 sweep kernel (bundle rows, host-evaluated media, PerfectLens code: sweep_kernel<double, 17, true>) with
    every surface one form: the innermost loop is one run step for kSweepRays rays per lane."""
    for case in ("sphere_ax", "sphere_gen", "flat_ax", "flat_xz", "lens_ax"):
        kind, geo = CASES[case]
        funcs = {n: b for n, b in functions(compile_kernel(kind, geo, sweep=True)).items()
                 if "sweep_kernelIdLi17ELb1E" in n}
        (name, body), = funcs.items()
        depth = max(int(m.group(1)) for m in re.finditer(r"Depth=(\d+)", "\n".join(body)))
        blks = loop_blocks(body, depth)
        on = [x for lab, ins in blks if not is_fill(ins) for x in ins if is_valu(x)]
        hist = collections.Counter(x.split()[0] for x in on)
        f64 = sum(v for op, v in hist.items() if "_f64" in op and not op.startswith(("v_cmp", "v_frexp", "v_cvt")))
        movs = sum(v for op, v in hist.items() if op.startswith("v_mov"))
        g_body = {n: b for n, b in functions(compile_kernel(kind, geo, sweep=True, guards=True)).items()
                  if "sweep_kernelIdLi17ELb1E" in n}
        (gname, gbody), = g_body.items()
        gdepth = max(int(m.group(1)) for m in re.finditer(r"Depth=(\d+)", "\n".join(gbody)))
        guarded = guarded_walk(loop_blocks(gbody, gdepth), header_of(gbody, gdepth))
        print(f"{case:11s} sweep run-loop VALU {len(on):4d} fast path, {len(guarded):4d} with the guards, for 2 rays "
              f"(f64 arithmetic {f64:3d}, moves {movs:3d}, depth {depth}, blocks {len(blks)})", flush=True)
        if show == case + "+g":
            for x in guarded:
                print("    " + x)
        if show == case:
            for lab, ins in blks:
                print(f"  -- {lab}{'  (fill)' if is_fill(ins) else ''}")
                for x in ins:
                    print("    " + x)
            for op, v in hist.most_common():
                print(f"    {op:28s} {v}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--show", default="")
    ap.add_argument("--kernel", action="store_true")
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--final", action="store_true", help="--kernel: the final-plane-only variant (planes='final', "
                    "what tools/history_kind_cost.py runs)")
    a = ap.parse_args()
    if a.kernel:
        return kernel_main(a.show, a.final)
    if a.sweep:
        return sweep_main(a.show)
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
        f64 = sum(v for op, v in hist.items() if "_f64" in op and not op.startswith(("v_cmp", "v_frexp", "v_cvt")))
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
