"""The shipped kernel sources carry no experiment switches; the experiments live in
tools/experiments/experiments.patch (applied by tools/exp_build.py to a scratch copy) and that patch must
keep applying to the current sources."""
import glob
import os
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ray_trace_pb_amd", "csrc")


def test_no_experiment_switches_in_shipped_sources():
    hits = []
    for p in glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(CSRC, "*.hip")):
        for k, line in enumerate(open(p), 1):
            if "RTPB_EXP_" in line or "RTPB_FLOAT_RANGE_CHECKS" in line:
                hits.append(f"{os.path.basename(p)}:{k}")
    assert not hits, hits


@pytest.mark.skipif(not shutil.which("patch"), reason="patch(1) not available")
def test_experiments_patch_applies():
    with tempfile.TemporaryDirectory() as tmp:
        shutil.copytree(CSRC, os.path.join(tmp, "ray_trace_pb_amd", "csrc"), ignore=shutil.ignore_patterns("_obj"))
        r = subprocess.run(["patch", "-p1", "--dry-run", "-d", tmp, "-i",
                            os.path.join(ROOT, "tools", "experiments", "experiments.patch")],
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stdout + r.stderr
