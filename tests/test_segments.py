"""Host logic of long systems (> RTPB_MAX_SURFACES = 63 surfaces per fused launch): the segmentation
in ray_trace_pb_amd.raytrace._trace_segmented, checked on the CPU with the launch replaced by the
NumPy oracle (test-only stand-in for E.trace_host).  The GPU run of the same systems is
tests/test_gpu_multidevice.py::test_long_system_*."""
import numpy as np
import pytest

import ray_trace_pb_amd.materials as mat
import ray_trace_pb_amd.raytrace as rt
from ray_trace_pb_amd import _capi as C
from ray_trace_pb_amd import _engine as E
from oracle import rt_numpy as O
from serialize import material_to_dict, surface_to_dict
import systems
from parity import same_bits  # noqa: E402


@pytest.fixture
def oracle_launch(monkeypatch):
    """E.trace_host replaced by the oracle on the lowered segment (so no GPU is needed); records the
    surface counts of the launches."""
    launches = []
    real_lower = E.lower

    def lower(surfaces, materials, wavelengths, dtype):
        low = real_lower(surfaces, materials, wavelengths, dtype)
        low.src = ([surface_to_dict(s) for s in surfaces], [material_to_dict(m) for m in materials])
        return low

    def trace_host(low, rays2d, planes, devices=None, out=None):
        launches.append(low.nsurf)
        assert low.nsurf <= C.RTPB_MAX_SURFACES
        h = O.ray_trace(low.src[0], low.src[1], np.asarray(rays2d, dtype=np.float64))[list(planes)]
        h = h.astype(np.float64 if low.dtype == C.RTPB_F64 else np.float32)
        if out is not None:
            out[...] = h
            return out
        return h

    monkeypatch.setattr(E, "lower", lower)
    monkeypatch.setattr(E, "trace_host", trace_host)
    return launches


def test_long_system_segments_match_whole_trace(oracle_launch, monkeypatch):
    # E.Lowered uses __slots__: give lowered objects a dict so the stand-in can attach the source
    monkeypatch.setattr(E, "Lowered", type("Lowered", (), {}))
    system = systems.long_system(rt, mat)
    S = len(system.surfaces)
    assert S > 2 * C.RTPB_MAX_SURFACES - 30
    rays = systems.long_rays(300)
    m0, m1 = mat.Vacuum(), mat.Vacuum()
    ref = O.ray_trace([surface_to_dict(s) for s in system.surfaces],
                      [material_to_dict(m) for m in [m0] + list(system.materials) + [m1]], rays)
    assert ref.shape == (2 * S + 1, 300, 8)
    got = system.ray_trace(rays, m0, m1)
    assert oracle_launch == [63, S - 63]
    assert same_bits(got, ref)
    live = np.isfinite(ref[-1, :, 0]).sum()
    assert 0 < live < 300
    sel = [0, 5, 125, 126, 127, 200, 2 * S]
    assert same_bits(system.ray_trace(rays, m0, m1, planes=sel), ref[sel])
    assert same_bits(system.ray_trace(rays, m0, m1, planes="final"), ref[-1:])
    f32 = system.ray_trace(rays, m0, m1, dtype="float32")
    assert f32.dtype == np.float32 and same_bits(f32, ref.astype(np.float32))
    # 3-D history input is extended (RT:1175-1178)
    h3 = np.stack((rays, rays))
    got3 = system.ray_trace(h3, m0, m1)
    assert got3.shape == (2 * S + 2, 300, 8)
    assert same_bits(got3[2:], ref[1:]) and np.array_equal(got3[:2], h3)
