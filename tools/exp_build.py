"""Build an EXPERIMENT variant of librtpb.so from a patched scratch copy of the sources: the shipped
sources carry no experiment branches.  Applies the given patches (-p1, repository-relative paths) and
compiles with the given -D flags.  Never shipped: used by tools/ab_variants.py to find
where kernel time goes.  Named variants with reviewable source edits: tools/exp_variants.py.  The round-2
switches (RTPB_EXP_NO_COMPUTE, XCD_REMAP, PERSIST, ...) are profiles/r02/experiments/experiments_round2.patch,
which applies to the round-2 sources (commit 7b1cac3).

    python tools/exp_build.py --out ray_trace_pb_amd/exp_x.so --patch my.patch -DMY_SWITCH
    python tools/exp_build.py --out ray_trace_pb_amd/exp_base.so --rev HEAD     # the committed sources (A/B base)
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


def build(out, flags=(), patches=(), rev=None):
    with tempfile.TemporaryDirectory() as tmp:
        if rev:
            # the kernel sources (and include/) of a git revision
            arch = subprocess.run(["git", "-C", ROOT, "archive", rev, "ray_trace_pb_amd/csrc", "include"],
                                  check=True, capture_output=True).stdout
            subprocess.run(["tar", "-x", "-C", tmp], input=arch, check=True)
        else:
            shutil.copytree(_build.CSRC, os.path.join(tmp, "ray_trace_pb_amd", "csrc"),
                            ignore=shutil.ignore_patterns("_obj"))
        for p in patches:
            subprocess.run(["patch", "-p1", "-s", "-d", tmp, "-i", os.path.abspath(p)], check=True)
        return _build.build(force=True, verbose=False, extra_flags=list(flags), out=os.path.abspath(out),
                            csrc=os.path.join(tmp, "ray_trace_pb_amd", "csrc"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--patch", action="append", default=[])
    ap.add_argument("--rev", default=None, help="build the csrc of this git revision instead of the working tree")
    args, flags = ap.parse_known_args()
    print(build(args.out, flags, args.patch, args.rev))


if __name__ == "__main__":
    main()
