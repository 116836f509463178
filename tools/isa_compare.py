"""Compile every csrc/*.hip to gfx950 assembly and compare the per-function bodies with an earlier dump
(used to show that a source cleanup leaves the shipped kernels' ISA byte-identical).

    python tools/isa_compare.py dump DIR          # write DIR/<source>.s
    python tools/isa_compare.py compare DIR_A DIR_B
    python tools/isa_compare.py valu DIR_A DIR_B [REGEX]   # static VALU instruction counts per function
"""
import concurrent.futures
import glob
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ray_trace_pb_amd import _build  # noqa: E402

FUNC = re.compile(r"^(_Z\S+):\s*(;.*)?$")


def dump(outdir, csrc=_build.CSRC):
    os.makedirs(outdir, exist_ok=True)
    flags = [f for f in _build.FLAGS if f != "-fPIC"]

    def one(src):
        out = os.path.join(outdir, os.path.basename(src) + ".s")
        subprocess.run([_build.HIPCC] + flags + ["--cuda-device-only", "-S", "-o", out, src], check=True)
        return out
    srcs = sorted(glob.glob(os.path.join(csrc, "*.hip")))
    with concurrent.futures.ThreadPoolExecutor(8) as ex:
        return list(ex.map(one, srcs))


LABEL = re.compile(r"BB\d+_")


def functions(path):
    """{symbol: body} with basic-block labels renumbered per function (.LBB<function index>_<block>
    depends on the function's position in its file, not on its code)."""
    funcs, cur, body = {}, None, []
    for line in open(path):
        m = FUNC.match(line)
        if m:
            cur, body = m.group(1), []
            continue
        if cur is not None:
            if line.startswith(".Lfunc_end"):
                funcs[cur] = "".join(body)
                cur = None
            else:
                body.append(LABEL.sub("BB_", line))
    return funcs


def compare(a, b):
    fa, fb = {}, {}
    for p in glob.glob(os.path.join(a, "*.s")):
        fa.update(functions(p))
    for p in glob.glob(os.path.join(b, "*.s")):
        fb.update(functions(p))
    same = [k for k in fa if k in fb and fa[k] == fb[k]]
    diff = [k for k in fa if k in fb and fa[k] != fb[k]]
    only_a = [k for k in fa if k not in fb]
    only_b = [k for k in fb if k not in fa]
    print(f"functions: {len(fa)} before, {len(fb)} after; identical {len(same)}, different {len(diff)}, "
          f"removed {len(only_a)}, added {len(only_b)}")
    for k in diff:
        print("DIFFERENT", k)
    for k in only_a:
        print("removed", k)
    for k in only_b:
        print("added", k)
    return not diff


def valu(a, b, pattern="."):
    """Static VALU instruction counts of the functions matching `pattern` in two dumps (code size, not the
    executed count: tools/history_kind_cost.py and the PMC passes measure that)."""
    def counts(d):
        out = {}
        for p in glob.glob(os.path.join(d, "*.s")):
            for k, body in functions(p).items():
                if re.search(pattern, k):
                    out[k] = sum(1 for ln in body.splitlines() if ln.strip().startswith("v_"))
        return out
    ca, cb = counts(a), counts(b)
    for k in sorted(set(ca) | set(cb)):
        print(f"{ca.get(k, '-'):>7} {cb.get(k, '-'):>7}  {k[:140]}")


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    elif sys.argv[1] == "valu":
        valu(*sys.argv[2:5])
    else:
        sys.exit(0 if compare(sys.argv[2], sys.argv[3]) else 1)
