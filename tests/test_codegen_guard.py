"""Compiler-bug guard (CPU, needs hipcc): compile every HIP source for gfx950 to assembly and reject the
signature of the register-allocation miscompile met in round 2 -- a COPY whose source the virtual-
register rewriter marked undef, lowered to ``; kill: def $vgprA_vgprB killed $vgprC_vgprD killed $exec``
with a different source pair: the value is silently not moved (the float64 SoA-input kernels lost the
phase after the first surface, found by tests/test_gpu_abi_matrix.py; workaround in
csrc/rtpb_internal.h load_ray).  Legitimate KILLs of a register onto itself do not match."""
import concurrent.futures
import glob
import os
import re
import shutil
import subprocess

import pytest

from ray_trace_pb_amd import _build

HIPCC = _build.HIPCC
SIGNATURE = re.compile(r"; kill: def \$vgpr(\d+)_vgpr(\d+) killed \$vgpr(\d+)_vgpr(\d+) killed \$exec")
FUNC = re.compile(r"^(_Z\S+):")


def _asm(src, outdir):
    out = os.path.join(outdir, os.path.basename(src) + ".s")
    flags = [f for f in _build.FLAGS if f not in ("-fPIC",)]
    cmd = [HIPCC] + flags + ["--cuda-device-only", "-S", "-o", out, src]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    return out


def _findings(path):
    bad, func = [], None
    for line in open(path):
        m = FUNC.match(line)
        if m:
            func = m.group(1)
            continue
        m = SIGNATURE.search(line)
        if m and (m.group(1), m.group(2)) != (m.group(3), m.group(4)):
            bad.append((func, line.strip()))
    return bad


@pytest.mark.skipif(not (os.path.exists(HIPCC) or shutil.which(HIPCC)), reason="hipcc not available")
def test_no_undef_copy_kills_in_device_code(tmp_path):
    srcs = sorted(glob.glob(os.path.join(_build.CSRC, "*.hip")))
    assert srcs
    workers = max(1, min(len(srcs), os.cpu_count() or 2, 8))
    with concurrent.futures.ThreadPoolExecutor(workers) as ex:
        outs = list(ex.map(lambda s: _asm(s, str(tmp_path)), srcs))
    bad = [f for o in outs for f in _findings(o)]
    assert not bad, bad[:10]


def test_signature_matcher():
    text = ("_ZN5rtpbi12trace_kernelX:\n"
            "\t; kill: def $vgpr14_vgpr15 killed $vgpr2_vgpr3 killed $exec\n"
            "\t; kill: def $vgpr0 killed $vgpr0 def $vgpr1\n"
            "\t; kill: def $vgpr4_vgpr5 killed $vgpr4_vgpr5 killed $exec\n")
    import tempfile
    with tempfile.NamedTemporaryFile("w", suffix=".s", delete=False) as f:
        f.write(text)
    try:
        got = _findings(f.name)
    finally:
        os.unlink(f.name)
    assert got == [("_ZN5rtpbi12trace_kernelX", "; kill: def $vgpr14_vgpr15 killed $vgpr2_vgpr3 killed $exec")]
