"""The kernel's per-ray arithmetic (rtpb_math.h, instantiated on the host by a test-only harness)
reproduces the reference's golden histories BIT FOR BIT, through the product's own lowering
(ray_trace_pb_amd._engine.lower).  Runs without a GPU."""
import numpy as np
import pytest

import ray_trace_pb_amd.materials as mat
import ray_trace_pb_amd.raytrace as rt
from ray_trace_pb_amd import _capi as C
from ray_trace_pb_amd import _engine as E
from native_harness import harness_trace
from parity import CASES, load_case
from serialize import system_from_json
import json


def lowered_case(name):
    d = np.load(f"{__import__('parity').GOLDEN}/{name}.npz")
    system, m0, m1 = system_from_json(rt, mat, str(d["system_json"]))
    rays = d["rays_in"]
    low = E.lower(system.surfaces, [m0] + list(system.materials) + [m1],
                  lambda: np.unique(rays[:, 7]), C.RTPB_F64)
    return low, rays, d["history"]


@pytest.mark.parametrize("name", CASES)
def test_kernel_math_bitwise_vs_reference(name):
    low, rays, ref = lowered_case(name)
    got = harness_trace(low, rays)
    assert np.array_equal(got, ref, equal_nan=True)
