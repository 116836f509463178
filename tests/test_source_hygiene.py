"""The shipped kernel sources carry no experiment switches: experiments are source edits applied to a
scratch copy (tools/exp_variants.py, tools/exp_build.py); the round-2 switches are kept as a patch against
the round-2 sources (profiles/r02/experiments/experiments_round2.patch)."""
import glob
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ray_trace_pb_amd", "csrc")


def test_no_experiment_switches_in_shipped_sources():
    hits = []
    for p in glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(CSRC, "*.hip")):
        for k, line in enumerate(open(p), 1):
            if "RTPB_EXP_" in line or "RTPB_FLOAT_RANGE_CHECKS" in line:
                hits.append(f"{os.path.basename(p)}:{k}")
    assert not hits, hits
