"""The axial-geometry surface steps (rtpb_math.h `kAxial`: normal / input axis exactly (+0, +0, 1), center
on the z axis) rewrite the reference's dot and cross products with the exact identities v - (+0) == v,
v * 1 == v and RN(RN(a * 0) + b) == fma(a, 0, b).  These tests drive those paths with adversarial rays --
+-0, +-inf and NaN in every field, rays on the axis with either zero sign, normal incidence, directions
that are not unit vectors -- and require the results BIT-IDENTICAL to the NumPy oracle (the reference's
numerics, oracle/rt_numpy.py), zero signs included:
  * on the CPU through the host instantiation of the kernel arithmetic (tests/native/math_harness.cpp);
  * on the GPU through System.ray_trace (librtpb.so)."""
import numpy as np
import pytest

import ray_trace_pb_amd.materials as mat
import ray_trace_pb_amd.raytrace as rt
from ray_trace_pb_amd import _capi as C
from ray_trace_pb_amd import _engine as E
from native_harness import harness_trace, surface_flags
from oracle import rt_numpy as O
from parity import same_bits
from serialize import material_to_dict, surface_to_dict
import systems

K_AXIAL = 64
K_PLANE_XZ = 4096
SPECIAL = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1.0, -1.0, 5e-324, 1e300, -1e-300])


def axial_lens_system():
    """Flat, two on-axis spheres, an on-axis PerfectLens between Constant media, a final flat -- every
    kind that has an axial step, with Constant, Vacuum and Sellmeier media."""
    return rt.System([rt.FlatSurface([0, 0, 0], [0, 0, 1], 20),
                      rt.SphericalSurface.get_on_axis(40, 5, 15),
                      rt.SphericalSurface.get_on_axis(-60, 9, 15),
                      rt.PerfectLens(20, [0, 0, 40], [0, 0, 1], 0.9),
                      rt.FlatSurface([0, 0, 70], [0, 0, 1], 50)],
                     [mat.Bk7(), mat.Constant(1.2), mat.Constant(1.4), mat.Vacuum()]), mat.Vacuum(), mat.Constant(1.0)


def tilted_xz_system():
    """Surfaces tilted in the x-z plane (kPlaneXZ): flats and PerfectLens steps with normals (-sin t, 0, cos t) and
    centers off the axis in x, between Constant, Sellmeier and Vacuum media -- uniform-media lenses (F, B in the
    plane: the focal planes' x-z center form) and a lens beside a Sellmeier glass (per-ray focal points)."""
    def n(t):
        return [-np.sin(t), 0.0, np.cos(t)]
    return rt.System([rt.FlatSurface([0.3, 0, 0], n(0.2), 20),
                      rt.PerfectLens(15, [0.5, 0, 10], n(0.3), 0.8),
                      rt.FlatSurface([1.0, 0, 22], n(0.25), 40),
                      rt.PerfectLens(-12, [-0.7, 0, 35], n(-0.4), 0.7),
                      rt.FlatSurface([0.0, 0, 50], n(0.1), 60)],
                     [mat.Constant(1.3), mat.Vacuum(), mat.Bk7(), mat.Constant(1.1)]), mat.Vacuum(), mat.Constant(1.0)


CASES = {
    "c1": lambda: (lambda c: (c[0], c[2], c[3]))(systems.c1_plano_convex(rt, mat, nrays=3)),
    "c5": lambda: (systems.c5_system(rt, mat), mat.Constant(1), mat.Constant(1)),
    "c4": lambda: (systems.c4_system(rt, mat), mat.Constant(systems.OPM_N1), mat.Vacuum()),
    "lens": axial_lens_system,
    "xz": tilted_xz_system,
}


def adversarial_rays(n=6000, seed=7, wl=0.55):
    """Near-axis bundles with every field replaced by a special value at random (30 %), plus on-axis,
    normal-incidence rays with each zero sign."""
    rng = np.random.default_rng(seed)
    r = np.zeros((n, 8))
    r[:, 0:2] = rng.normal(scale=2.0, size=(n, 2))
    r[:, 2] = -3.0 + rng.normal(scale=0.5, size=n)
    th, ph = rng.uniform(0, 0.2, n), rng.uniform(0, 2 * np.pi, n)
    r[:, 3:6] = np.stack((np.sin(th) * np.cos(ph), np.sin(th) * np.sin(ph), np.cos(th)), axis=1)
    r[:, 6] = rng.uniform(-1, 1, n)
    r[:, 7] = wl
    hit = rng.random((n, 8)) < np.array([0.06, 0.06, 0.03, 0.06, 0.06, 0.03, 0.03, 0.01])
    r[hit] = rng.choice(SPECIAL, size=int(hit.sum()))
    # exact axis rays: x, y in {+0, -0}, d = (+-0, +-0, 1 or 0.5), every sign combination
    signs = np.array([[a, b, c, d] for a in (0.0, -0.0) for b in (0.0, -0.0) for c in (0.0, -0.0)
                      for d in (0.0, -0.0)])
    ax = np.zeros((2 * len(signs), 8))
    ax[:, 0:2] = np.tile(signs[:, 0:2], (2, 1))
    ax[:, 2] = -2.0
    ax[:, 3:5] = np.tile(signs[:, 2:4], (2, 1))
    ax[:, 5] = np.repeat([1.0, 0.5], len(signs))
    ax[:, 6] = -0.0
    ax[:, 7] = wl
    return np.concatenate((r, ax), axis=0)


def oracle(system, m0, m1, rays):
    with np.errstate(all="ignore"):
        return O.ray_trace([surface_to_dict(s) for s in system.surfaces],
                           [material_to_dict(m) for m in [m0] + list(system.materials) + [m1]], rays)


def lowered(system, m0, m1, rays):
    wl = np.unique(rays[:, 7])
    return E.lower(system.surfaces, [m0] + list(system.materials) + [m1], lambda: wl, C.RTPB_F64)


@pytest.mark.parametrize("name", sorted(CASES))
def test_axial_flags_set_where_the_geometry_is_axial(name):
    system, m0, m1 = CASES[name]()
    flags = surface_flags(lowered(system, m0, m1, adversarial_rays(10)))
    for s, f in zip(system.surfaces, flags):
        axial = (np.array_equal(np.asarray(s.center, float)[:2].view(np.uint64), [0, 0])
                 and np.array_equal(np.asarray(s.input_axis, float).view(np.uint64),
                                    np.array([0.0, 0.0, 1.0]).view(np.uint64)))
        if isinstance(s, rt.PlaneMirror):
            axial = False
        assert bool(f & K_AXIAL) == axial, (type(s).__name__, s.center, s.input_axis)
    assert any(f & K_AXIAL for f in flags) or name == "xz"


@pytest.mark.parametrize("name", sorted(CASES))
def test_plane_xz_flags_set_where_the_geometry_allows(name):
    """kPlaneXZ (the x-z-plane steps, GEO = kGeoXZ): flats and PerfectLens surfaces that are not axial and whose
    center, normal (and, for a flat, input axis) have y components exactly +0 -- C4's five surfaces behind the 30 deg
    tilt (scripts/2022_01_25_ray_trace_ideal_opm.py:59-80)."""
    system, m0, m1 = CASES[name]()
    flags = surface_flags(lowered(system, m0, m1, adversarial_rays(10)))
    p0 = lambda v: np.asarray(v, float).view(np.uint64)[1] == 0          # noqa: E731
    for s, f in zip(system.surfaces, flags):
        want = (not f & K_AXIAL and isinstance(s, (rt.FlatSurface, rt.PerfectLens)) and p0(s.center) and p0(s.normal)
                and (isinstance(s, rt.PerfectLens) or p0(s.input_axis)))
        assert bool(f & K_PLANE_XZ) == want, (type(s).__name__, s.center, s.normal)
    if name == "c4":
        assert sum(bool(f & K_PLANE_XZ) for f in flags) == 5
    if name == "xz":
        assert all(f & K_PLANE_XZ for f in flags)


@pytest.mark.parametrize("name", sorted(CASES))
def test_axial_steps_bitwise_vs_oracle_cpu(name):
    system, m0, m1 = CASES[name]()
    rays = adversarial_rays(wl=0.532 if name == "c4" else 0.55)
    ref = oracle(system, m0, m1, rays)
    got = harness_trace(lowered(system, m0, m1, rays), rays)
    assert same_bits(got, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_axial_steps_bitwise_vs_oracle_gpu(name):
    torch = pytest.importorskip("torch")
    system, m0, m1 = CASES[name]()
    rays = adversarial_rays(wl=0.532 if name == "c4" else 0.55)
    ref = oracle(system, m0, m1, rays)
    got = system.ray_trace(torch.from_numpy(rays).to("cuda:0"), m0, m1)
    assert same_bits(got.cpu().numpy(), ref)
    assert same_bits(system.ray_trace(rays, m0, m1, planes="final")[0], ref[-1])
