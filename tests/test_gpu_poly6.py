"""RTPB_POLY6 materials (include/rtpb.h: the six-term polynomial dispersion of Ebaf11, MAT:128-144) on the
GPU.  The Python layer lowers Ebaf11 as a host-evaluated table (bit-exact with NumPy); a C-ABI caller may
send the polynomial itself, which the kernels evaluate with the device pow().  NumPy's SIMD power and the
device pow() may differ in the last bit, so POLY6 traces are checked against the table (= reference)
traces within a tolerance, with identical NaN masks: trace kernels (all planes, final plane, float32
storage) and the fused spot sweep (whose POLY6 plans evaluate n per surface instead of per group)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import ray_trace_pb_amd.materials as mat  # noqa: E402
import ray_trace_pb_amd.raytrace as rt  # noqa: E402
from ray_trace_pb_amd import _capi as C  # noqa: E402
from ray_trace_pb_amd import analysis  # noqa: E402
from parity import same_bits, compare  # noqa: E402
import systems  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


class Ebaf11Poly(mat.Ebaf11):
    """Ebaf11 sent to the kernels as RTPB_POLY6 (device pow) instead of a host table."""

    def _rtpb_lower(self):
        return C.RTPB_POLY6, tuple(self.params)


def _poly_system(system):
    mats = [Ebaf11Poly() if type(m) is mat.Ebaf11 else m for m in system.materials]
    assert any(isinstance(m, Ebaf11Poly) for m in mats)
    return rt.System(system.surfaces, mats)


def test_poly6_trace_matches_table_trace():
    system = systems.c3_system(rt, mat)
    poly = _poly_system(system)
    m0, m1 = mat.Vacuum(), mat.Vacuum()
    rays = systems.c3_rays(rt, 41, 40)
    x = torch.from_numpy(rays).to(DEV)
    ref = system.ray_trace(x, m0, m1).cpu().numpy()
    assert np.isfinite(ref[-1]).all(axis=1).mean() > 0.5
    got = poly.ray_trace(x, m0, m1).cpu().numpy()
    ok, rep = compare(got, ref, rtol=1e-12)
    assert ok and rep["mask_flips"] == 0, rep
    fin = poly.ray_trace(x, m0, m1, planes="final").cpu().numpy()
    assert same_bits(fin[0], got[-1])
    f32 = poly.ray_trace(x, m0, m1, dtype="float32").cpu().numpy()
    ok, rep = compare(f32, ref, rtol=1e-6)
    assert ok and rep["mask_flips"] == 0, rep


@pytest.mark.parametrize("deg", [1, 10])
def test_poly6_spot_sweep_matches_table_sweep(deg):
    """deg=10 vignettes 12 % of the rays at intermediate surfaces: a lane whose first ray dies there keeps
    evaluating its second ray's media at the group's wavelength (not at the dead ray's NaN)."""
    system = systems.c3_system(rt, mat)
    poly = _poly_system(system)
    fields = np.array([[0.0, 0.0, 0.0], [8.0, 0.0, 0.0], [16.0, 0.0, 0.0]])
    wls = (0.532, 0.635)
    th = deg * np.pi / 180
    ref, _ = analysis.spot_sweep(system, mat.Vacuum(), mat.Vacuum(), fields, wls, th, 65, 64, device=DEV)
    got, _ = analysis.spot_sweep(poly, mat.Vacuum(), mat.Vacuum(), fields, wls, th, 65, 64, device=DEV)
    assert np.array_equal(got["count"], ref["count"])
    for k in ("rms_radius", "centroid"):
        if k in ref:
            np.testing.assert_allclose(got[k], ref[k], rtol=1e-11, atol=1e-14)
