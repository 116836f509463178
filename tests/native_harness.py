"""Build + load the CPU harness of the kernel arithmetic (tests/native/math_harness.cpp).
TEST INFRASTRUCTURE ONLY."""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "math_harness.cpp")
OUT = os.path.join(HERE, "native", "_build", "libmath_harness.so")
DEPS = [SRC, os.path.join(HERE, "..", "ray_trace_pb_amd", "csrc", "rtpb_math.h"),
        os.path.join(HERE, "..", "include", "rtpb.h")]

_lib = None


def harness():
    global _lib
    if _lib is None:
        os.makedirs(os.path.dirname(OUT), exist_ok=True)
        import fcntl
        with open(OUT + ".lock", "w") as lk:        # several test processes may race to (re)build
            fcntl.flock(lk, fcntl.LOCK_EX)
            if not os.path.exists(OUT) or any(os.path.getmtime(OUT) < os.path.getmtime(d) for d in DEPS):
                tmp = f"{OUT}.{os.getpid()}.tmp"
                subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
                                "-I", os.path.join(HERE, "..", "include"), "-o", tmp, SRC], check=True)
                os.replace(tmp, OUT)
        _lib = ctypes.CDLL(OUT)
        _lib.harness_bounds.argtypes = [ctypes.c_double] * 3 + [ctypes.POINTER(ctypes.c_double)]
        _lib.harness_bounds.restype = None
    return _lib


def surface_flags(low):
    """lower_surface's rcp_ok flags of every surface of a lowered system (bit 6 = kAxial)."""
    fn = harness().harness_surface_flags
    fn.argtypes, fn.restype = [ctypes.c_void_p], ctypes.c_int
    size = ctypes.sizeof(low.surfaces) // low.nsurf
    base = ctypes.addressof(low.surfaces)
    return [fn(base + k * size) for k in range(low.nsurf)]


def harness_trace(low, rays2d, dtype=np.float64):
    """Full history (2S+1, N, 8) of rays2d through a lowered system (ray_trace_pb_amd._engine.lower)."""
    rays2d = np.ascontiguousarray(rays2d, dtype=dtype)
    n = rays2d.shape[0]
    out = np.empty((2 * low.nsurf + 1, n, 8), dtype=dtype)
    fn = harness().harness_trace_f64 if dtype == np.float64 else harness().harness_trace_f32
    rc = fn(low.surfaces, ctypes.c_int32(low.nsurf), low.materials,
                                     rays2d.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(n),
                                     out.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0
    return out


FASTDIV_SRC = os.path.join(HERE, "native", "fastdiv_check.hip")
FASTDIV_OUT = os.path.join(HERE, "native", "_build", "libfastdiv_check.so")
_fastdiv = None


def build_fastdiv():
    """hipcc (gfx950) build of the GPU check of rtpb_math.h's shared-divisor quotients (run by
    __graft_entry__.build(); the GPU box uses the prebuilt library)."""
    deps = [FASTDIV_SRC] + DEPS[1:]
    if os.path.exists(FASTDIV_OUT) and all(os.path.getmtime(FASTDIV_OUT) >= os.path.getmtime(d) for d in deps):
        return FASTDIV_OUT
    os.makedirs(os.path.dirname(FASTDIV_OUT), exist_ok=True)
    tmp = f"{FASTDIV_OUT}.{os.getpid()}.tmp"
    subprocess.run([os.environ.get("HIPCC", "/opt/rocm/bin/hipcc"), "--offload-arch=gfx950", "-O3", "-std=c++17",
                    "-ffp-contract=off", "-fPIC", "-shared", "-I", os.path.join(HERE, "..", "include"),
                    "-o", tmp, FASTDIV_SRC], check=True)
    os.replace(tmp, FASTDIV_OUT)
    return FASTDIV_OUT


def fastdiv_check(a, a2, a3, b, kill):
    """(39, n) float64: div1, a / b, div3 x/y/z, div1_as, tsqrt(b), tsqrt(a), div1 through the host's
    reciprocal RN(1/b), then the GuardDefer forms with their flags (div1, flag, div3 x/y/z, flag,
    tsqrt(b), flag, div1_as, flag), then div3_norm of (a, a2, a3) by its own norm, its GuardDefer form
    and flag, then sphere_root(a, sqrt|b|) and signed_root(a, sqrt|b|), then unit_or_zero of (a, a2, a3) and the phase
    term |(a, a2, a3)| * 2 pi / b, then the axial sphere normal's div3_norm by the host reciprocal of b (without
    div_fixup where b is finite, nonzero and in range), then unit_near1_or_zero of (a, a2, a3), then tsqrt_1m(1 - a a) --
    computed on cuda:0."""
    global _fastdiv
    if _fastdiv is None:
        import torch  # noqa: F401 -- one HIP runtime per process: bind to torch's
        _fastdiv = ctypes.CDLL(build_fastdiv())
        _fastdiv.fastdiv_check.argtypes = [ctypes.c_void_p] * 6 + [ctypes.c_int64, ctypes.c_void_p]
        _fastdiv.fastdiv_check.restype = ctypes.c_int
    with np.errstate(all="ignore"):
        yh = 1.0 / np.asarray(b, dtype=np.float64)
    arrs = [np.ascontiguousarray(x, dtype=np.float64) for x in (a, a2, a3, b, yh)]
    k = np.ascontiguousarray(kill, dtype=np.uint8)
    n = arrs[0].size
    out = np.empty((39, n), dtype=np.float64)
    rc = _fastdiv.fastdiv_check(*[x.ctypes.data for x in arrs], k.ctypes.data, n, out.ctypes.data)
    assert rc == 0, rc
    return out


VMM_SRC = os.path.join(HERE, "native", "vmm_remap_check.hip")
VMM_OUT = os.path.join(HERE, "native", "_build", "vmm_remap_check")


def build_vmm_check():
    """hipcc (gfx950) build of the torch-free HIP virtual-memory remapping check (an executable; run by
    tests/test_gpu_vmm.py and tools/gpu_run.sh vmm)."""
    if os.path.exists(VMM_OUT) and os.path.getmtime(VMM_OUT) >= os.path.getmtime(VMM_SRC):
        return VMM_OUT
    os.makedirs(os.path.dirname(VMM_OUT), exist_ok=True)
    tmp = f"{VMM_OUT}.{os.getpid()}.tmp"
    subprocess.run([os.environ.get("HIPCC", "/opt/rocm/bin/hipcc"), "--offload-arch=gfx950", "-O2", "-std=c++17",
                    "-Wall", "-o", tmp, VMM_SRC], check=True)
    os.replace(tmp, VMM_OUT)
    return VMM_OUT


VMM_LIB = os.path.join(HERE, "native", "_build", "libvmm_remap_check.so")


def build_vmm_check_lib():
    """The same check as a shared library (entry vmm_remap_check_run), for tools/vmm_torch_runtime.py: loaded after
    torch it binds to torch's HIP runtime (one libamdhip64 per process, matched by SONAME), the runtime every
    product process uses."""
    if os.path.exists(VMM_LIB) and os.path.getmtime(VMM_LIB) >= os.path.getmtime(VMM_SRC):
        return VMM_LIB
    os.makedirs(os.path.dirname(VMM_LIB), exist_ok=True)
    tmp = f"{VMM_LIB}.{os.getpid()}.tmp"
    subprocess.run([os.environ.get("HIPCC", "/opt/rocm/bin/hipcc"), "--offload-arch=gfx950", "-O2", "-std=c++17",
                    "-Wall", "-shared", "-fPIC", "-o", tmp, VMM_SRC], check=True)
    os.replace(tmp, VMM_LIB)
    return VMM_LIB
