"""Build librtpb.so (gfx950) in-tree: ``python -m ray_trace_pb_amd._build [--force]``.

Every ``csrc/*.hip`` translation unit is compiled to an object in parallel, then linked into one
shared library next to this file (it travels with the repository snapshot; nothing is installed)."""
import concurrent.futures
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(CSRC, "_obj")
OUT = os.path.join(HERE, "librtpb.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

# -ffp-contract=off: no FMA contraction, so f64 results are IEEE-identical to the NumPy reference
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-Wall",
         "-I", os.path.join(ROOT, "include")]


def sources(csrc=CSRC):
    return sorted(glob.glob(os.path.join(csrc, "*.hip")))


def build(force=False, verbose=True, extra_flags=(), out=None, csrc=CSRC):
    """Compile csrc/*.hip and link them into `out`.  `csrc` / `extra_flags` let tools build experiment
    variants from a patched copy of the sources (tools/exp_build.py); the product build uses neither."""
    out = out or OUT
    srcs = sources(csrc)
    deps = srcs + glob.glob(os.path.join(csrc, "*.h")) + [os.path.join(ROOT, "include", "rtpb.h")]
    if not force and not extra_flags and csrc == CSRC and os.path.exists(out) and \
            all(os.path.getmtime(out) >= os.path.getmtime(d) for d in deps):
        return out
    os.makedirs(OBJ, exist_ok=True)
    tag = f"{os.getpid()}"
    objs = [os.path.join(OBJ, os.path.basename(s)[:-4] + f".{tag}.o") for s in srcs]

    def compile_one(src_obj):
        cmd = [HIPCC] + FLAGS + list(extra_flags) + ["-c", "-o", src_obj[1], src_obj[0]]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)

    try:
        with concurrent.futures.ThreadPoolExecutor(max_workers=min(len(srcs), 8)) as ex:
            list(ex.map(compile_one, zip(srcs, objs)))
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out + ".tmp"] + objs
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(out + ".tmp", out)
    finally:
        for o in objs:
            if os.path.exists(o):
                os.remove(o)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv)
