"""Build librtpb.so (gfx950) in-tree: ``python -m ray_trace_pb_amd._build``."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "rtpb_device.hip")
OUT = os.path.join(HERE, "librtpb.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

# -ffp-contract=off: no FMA contraction, so f64 results are IEEE-identical to the NumPy reference
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared", "-Wall",
         "-I", os.path.join(ROOT, "include")]


def build(force=False, verbose=True):
    deps = [SRC, os.path.join(HERE, "csrc", "rtpb_math.h"), os.path.join(ROOT, "include", "rtpb.h")]
    if not force and os.path.exists(OUT) and all(os.path.getmtime(OUT) >= os.path.getmtime(d) for d in deps):
        return OUT
    cmd = [HIPCC] + FLAGS + ["-o", OUT + ".tmp", SRC]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
