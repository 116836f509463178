"""The timed CPU baseline (oracle/rt_refcost.py: the reference's data flow, bench.py's cpu_baseline leg)
computes exactly the reference's histories: bit for bit against every golden vector."""
import numpy as np
import pytest

from oracle import rt_refcost as RC
from parity import same_bits, CASES, load_case


@pytest.mark.parametrize("name", CASES)
def test_refcost_port_matches_reference_bitwise(name):
    spec, rays, ref = load_case(name)
    got = RC.ray_trace(spec["surfaces"], spec["materials"], rays)
    assert got.shape == ref.shape
    assert same_bits(got, ref)


def test_refcost_port_input_ranks():
    import json
    import os
    from parity import GOLDEN
    d = np.load(os.path.join(GOLDEN, "shapes.npz"))
    spec = json.loads(str(d["system_json"]))
    for k in ("1", "2", "3"):
        got = RC.ray_trace(spec["surfaces"], spec["materials"], d["rays" + k])
        assert same_bits(got, d["out" + k]), k
