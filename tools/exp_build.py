"""Build an EXPERIMENT variant of librtpb.so: the shipped sources carry no experiment branches, so this
copies ray_trace_pb_amd/csrc to a scratch directory, applies tools/experiments/experiments.patch (which
restores the RTPB_EXP_* switches: NO_COMPUTE, NO_GUARDS, NO_MATERIAL, NO_ONSURFACE, NO_INPUT, XCD_REMAP,
SCATTER, STAGGER, FLUSH_SYNC, PERSIST, MAXW, WPE, STORE_AUX, TRACE_BLOCK, FLOAT_RANGE_CHECKS, the
waves_per_eu=5 knob) and any extra patches, and compiles with the given -D flags.  Never shipped: used by
tools/ab_variants.py / tools/ab_libs.py to find where kernel time goes.

    python tools/exp_build.py --out ray_trace_pb_amd/exp_nocomp.so -DRTPB_EXP_NO_COMPUTE
    python tools/exp_build.py --out ray_trace_pb_amd/exp_x.so --patch my.patch --no-exp-patch
"""
import argparse
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ray_trace_pb_amd import _build  # noqa: E402

EXP_PATCH = os.path.join(ROOT, "tools", "experiments", "experiments.patch")


def build(out, flags=(), patches=(), exp_patch=True):
    with tempfile.TemporaryDirectory() as tmp:
        shutil.copytree(_build.CSRC, os.path.join(tmp, "ray_trace_pb_amd", "csrc"),
                        ignore=shutil.ignore_patterns("_obj"))
        for p in ([EXP_PATCH] if exp_patch else []) + list(patches):
            subprocess.run(["patch", "-p1", "-s", "-d", tmp, "-i", os.path.abspath(p)], check=True)
        return _build.build(force=True, verbose=False, extra_flags=list(flags), out=os.path.abspath(out),
                            csrc=os.path.join(tmp, "ray_trace_pb_amd", "csrc"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--patch", action="append", default=[])
    ap.add_argument("--no-exp-patch", action="store_true")
    args, flags = ap.parse_known_args()
    print(build(args.out, flags, args.patch, not args.no_exp_patch))


if __name__ == "__main__":
    main()
