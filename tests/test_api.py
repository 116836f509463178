"""Host-side API parity with the reference (no GPU): system construction (Doublet, concatenate,
reverse, paraxial placement), paraxial analysis, ray generators and ray utilities against golden
values produced by the reference, and the lowering to C-ABI descriptors."""
import collections
import json
import os

import numpy as np
import pytest

import ray_trace_pb_amd.materials as mat
import ray_trace_pb_amd.raytrace as rt
from ray_trace_pb_amd import _capi as C
from ray_trace_pb_amd import _engine as E
from parity import same_bits, CASES, F32IN_CASES, GOLDEN
from serialize import system_to_json, system_from_json
import systems


@pytest.mark.parametrize("name", CASES + F32IN_CASES)
def test_recipe_builds_the_reference_system(name):
    """The same recipe built with this package serialises to EXACTLY the reference's system (every
    center, axis, radius and coefficient bit for bit -- concatenate's shifts and get_cardinal_points
    included) and generates exactly the reference's input rays."""
    base = name[:-len("_f32in")] if name.endswith("_f32in") else name
    system, rays, m0, m1 = systems.RECIPES[base](rt, mat)
    d = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    assert json.loads(system_to_json(system, m0, m1)) == json.loads(str(d["system_json"]))
    rays = np.asarray(rays, dtype=d["rays_in"].dtype)
    assert same_bits(rays, d["rays_in"])


def _paraxial():
    with open(os.path.join(GOLDEN, "paraxial.json")) as f:
        return json.load(f)


def test_paraxial_matrices_and_cardinal_points():
    par = _paraxial()
    for case in par["cases"]:
        system, _, m0, m1 = systems.RECIPES[case["name"]](rt, mat)
        wl = case["wavelength"]
        np.testing.assert_allclose(system.get_ray_transfer_matrix(wl, m0, m1), case["rtm"], rtol=1e-12, atol=1e-14)
        for got, ref in zip(system.get_cardinal_points(wl, m0, m1), case["cardinal"]):
            np.testing.assert_allclose(np.asarray(got, dtype=float), ref, rtol=1e-10, atol=1e-10)
        np.testing.assert_allclose(system.auto_focus(wl, m0, m1, mode="paraxial-collimated"),
                                   case["auto_focus_paraxial_collimated"], rtol=1e-12)


def test_seidel_kidger_table():
    """tests/rt_unittest.py of the reference: Kidger 8.2.2 doublet Seidel sums."""
    l1 = rt.Doublet(mat.Nsk11(), mat.Nsf19(), radius_crown=64.1, radius_flint=-183.685, radius_interface=-43.249,
                    thickness_crown=3.5, thickness_flint=1.5, aperture_radius=10., input_collimated=True)
    system = l1.concatenate(rt.FlatSurface([0, 0, 0], [0, 0, 1], 25.4), mat.Vacuum(), 10)
    system.set_aperture_stop(0)
    ab = system.seidel_third_order(0.5876, mat.Vacuum(), mat.Vacuum(), object_distance=np.inf, object_angle=0.01746)
    np.testing.assert_allclose(ab, _paraxial()["kidger_seidel"], rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(ab.sum(axis=0), [0.001889, -0.000088, 0.000295, 0.000210, 0.000002], atol=1e-5)


def test_generators_and_utilities_match_reference():
    g = np.load(os.path.join(GOLDEN, "generators.npz"))
    assert np.array_equal(rt.get_ray_fan([1., 2., 3.], 0.3, 7, 0.5, nphis=5, center_ray=(0, 0, 1)), g["fan"])
    assert np.array_equal(rt.get_ray_fan([0., 0., 0.], 0.2, 5, 0.6, nphis=3,
                                         center_ray=tuple(systems.unit([0.6, 0, 0.8]))), g["fan_tilted"])
    assert np.array_equal(rt.get_collimated_rays([0., 1., -2.], 3., 5, 0.5, nphis=4, phi_start=0.3), g["coll"])
    assert np.array_equal(rt.get_collimated_rays([0., 0., 0.], 2., 4, 0.5, nphis=3,
                                                 normal=[np.sin(0.2), 0, np.cos(0.2)]), g["coll_tilted"])
    assert np.array_equal(rt.get_collimated_rays([0., 0., 0.], 2., 3, 0.5, nphis=2, normal=[0, 1, 0]), g["coll_y"])
    assert same_bits(rt.intersect_rays(g["intersect_in1"], g["intersect_in2"]), g["intersect_out"])
    fan = rt.get_ray_fan([0., 0., 0.], 0.1, 5, 0.5)
    assert same_bits(rt.intersect_rays(fan[1], fan), g["intersect_fan_out"])
    ang, na = rt.ray_angle_about_axis(g["intersect_in1"], np.array([0., 0., 1.]))
    assert same_bits(ang, g["angle_out"]) and same_bits(na, g["angle_na"])


def test_generator_argument_errors():
    with pytest.raises(ValueError):
        rt.get_ray_fan([0, 0, 0], 0.1, 3, 0.5, center_ray=(0, 0, 2))
    with pytest.raises(ValueError):
        rt.get_collimated_rays([0, 0, 0], 1, 3, 0.5, normal=(0, 0, 2))


def test_system_validation():
    f = rt.FlatSurface([0, 0, 0], [0, 0, 1], 1)
    with pytest.raises(ValueError):
        rt.System([f, f, f], [mat.Vacuum(), mat.Vacuum(), mat.Vacuum()])
    s = rt.System([f, f], [mat.Vacuum()])
    with pytest.raises(ValueError):
        s.ray_trace(np.zeros((2, 8)), mat.Vacuum(), mat.Vacuum(), planes=[5])
    s.materials = []
    with pytest.raises(ValueError):
        s.ray_trace(np.zeros((2, 8)), mat.Vacuum(), mat.Vacuum())
    with pytest.raises(ValueError):      # as in the reference: [init] + [] + [final] has 2 != 0 + 1 entries
        rt.System([], []).ray_trace(np.ones((2, 8)), mat.Vacuum(), mat.Vacuum())


def test_lowering_descriptors():
    system, rays, m0, m1 = systems.stress(rt, mat)
    mats = [m0] + list(system.materials) + [m1]
    low = E.lower(system.surfaces, mats, lambda: np.unique(rays[:, 7]), C.RTPB_F64)
    kinds = [low.surfaces[k].kind for k in range(low.nsurf)]
    assert kinds == [0, 1, 1, 0, 1, 1, 3, 0, 1, 2, 0]
    sph = system.surfaces[1]
    assert low.surfaces[1].radius_sq == sph.radius ** 2 and low.surfaces[1].on_tol == 1e-12
    lens = system.surfaces[6]
    assert low.surfaces[6].sin_alpha == np.sin(lens.alpha) and low.surfaces[6].focal_len == lens.focal_len
    mk = [low.materials[k].kind for k in range(low.nsurf + 1)]
    assert mk == [C.RTPB_SELLMEIER, C.RTPB_SELLMEIER, C.RTPB_SELLMEIER, C.RTPB_SELLMEIER, C.RTPB_CONSTANT,
                  C.RTPB_TABLE, C.RTPB_SELLMEIER, C.RTPB_SELLMEIER, C.RTPB_TABLE, C.RTPB_SELLMEIER,
                  C.RTPB_SELLMEIER, C.RTPB_SELLMEIER]
    uniq = np.unique(rays[:, 7])
    for tab, m in zip(low.tables, (mats[5], mats[8])):      # Ebaf11 (host NumPy power) and the user Cauchy
        tab = tab.reshape(-1, 2)
        assert same_bits(tab[:, 0], uniq) and np.isnan(tab[-1, 0])
        assert same_bits(tab[:, 1], m.n(uniq))
    # same content -> same plan-cache key; different dtype -> different key
    low2 = E.lower(system.surfaces, mats, lambda: np.unique(rays[:, 7]), C.RTPB_F64)
    assert low.key == low2.key
    low3 = E.lower(system.surfaces, mats, lambda: np.unique(rays[:, 7]), C.RTPB_F32)
    assert low3.key != low.key and low3.surfaces[1].on_tol == 1e-12    # float64 arithmetic for both storage types


def test_custom_surface_geometry_is_not_lowered_to_the_fused_kernel():
    class Wobbly(rt.FlatSurface):
        def get_normal(self, pts):
            return super().get_normal(pts) * 1.0
    # the fused kernel never runs a surface whose geometry the user replaced ...
    with pytest.raises(NotImplementedError):
        E.lower([Wobbly([0, 0, 0], [0, 0, 1], 1)], [mat.Vacuum(), mat.Vacuum()], lambda: np.array([0.5]),
                C.RTPB_F64)
    # ... System.ray_trace routes it through propagate_user_geometry (GPU hook kernels) instead
    assert Wobbly([0, 0, 0], [0, 0, 1], 1)._rtpb_user_geometry()

    class Plain(rt.SphericalSurface):     # subclass that does not touch the geometry: still lowerable
        pass
    low = E.lower([Plain(10, [0, 0, 10], 5)], [mat.Vacuum(), mat.Bk7()], lambda: np.array([0.5]), C.RTPB_F64)
    assert low.surfaces[0].kind == C.RTPB_SPHERE


def test_reverse_and_concatenate_semantics():
    d = rt.Doublet(mat.Bk7(), mat.Sf2(), radius_crown=106.2, radius_flint=-409.4, radius_interface=-92.1,
                   thickness_crown=10.6, thickness_flint=6.0, aperture_radius=25.4)
    r = d.reverse()
    assert [type(m).__name__ for m in r.materials] == ["Sf2", "Bk7"]
    assert np.array_equal(r.surfaces[0].input_axis, [0, 0, -1])
    assert np.array_equal(d.surfaces[0].input_axis, [0, 0, 1])     # deep-copied, original untouched
    c = d.concatenate(rt.FlatSurface([0, 0, 0], [0, 0, 1], 5), mat.Vacuum(), distance=7)
    assert np.allclose(c.surfaces[-1].center, [0, 0, 16.6 + 7])
    assert list(c.surfaces_by_name) == [0, 0, 0, 1]


def test_material_catalogue_values():
    # N-BK7 at the d-line, n_d = 1.5168 (Schott), Abbe 64.17
    assert abs(mat.Bk7().n(0.5876) - 1.5168) < 1e-4
    assert abs(mat.Bk7().vd - 64.17) < 0.05
    assert mat.Vacuum().n(0.5) == 1.0
    assert mat.Constant(1.33).n(0.5) == 1.33
    assert np.array_equal(mat.Constant(1.33).n(np.array([0.5, 0.6])), [1.33, 1.33])
    assert abs(mat.Ebaf11().n(0.5876) - 1.666) < 2e-3


def test_user_propagate_detection():
    class MyFlat(rt.FlatSurface):
        def propagate(self, ray_array, material1, material2):
            return ray_array

    class Geo(rt.FlatSurface):
        def get_intersect(self, rays, material):
            return rays
    assert MyFlat([0, 0, 0], [0, 0, 1], 1)._rtpb_user_propagate()
    assert not rt.FlatSurface([0, 0, 0], [0, 0, 1], 1)._rtpb_user_propagate()
    assert not rt.PlaneMirror([0, 0, 0], [0, 0, 1], 1)._rtpb_user_propagate()
    assert not rt.PerfectLens(1, [0, 0, 0], [0, 0, 1], 0.5)._rtpb_user_propagate()
    assert not Geo([0, 0, 0], [0, 0, 1], 1)._rtpb_user_propagate()
    with pytest.raises(NotImplementedError):
        Geo([0, 0, 0], [0, 0, 1], 1)._rtpb_kind()
    # user geometry hooks (keep the base propagate): traced through propagate_user_geometry
    class Bare(rt.RefractingSurface):
        pass

    class LensGeo(rt.PerfectLens):
        def get_normal(self, pts):
            return pts

    class MirrorGeo(rt.ReflectingSurface):
        def get_intersect(self, rays, material):
            return rays
    assert Geo([0, 0, 0], [0, 0, 1], 1)._rtpb_user_geometry()
    assert Bare([0, 0, 1], [0, 0, 1], [0, 0, 0], [0, 0, 0], 1)._rtpb_user_geometry()
    assert MirrorGeo([0, 0, 1], [0, 0, 1], [0, 0, 0], [0, 0, 0], 1)._rtpb_user_geometry()
    assert not MirrorGeo([0, 0, 1], [0, 0, 1], [0, 0, 0], [0, 0, 0], 1)._rtpb_user_propagate()
    assert not MyFlat([0, 0, 0], [0, 0, 1], 1)._rtpb_user_geometry()
    assert not LensGeo(1, [0, 0, 0], [0, 0, 1], 0.5)._rtpb_user_geometry()
    assert LensGeo(1, [0, 0, 0], [0, 0, 1], 0.5)._rtpb_kind() == C.RTPB_PERFECT_LENS
    for s in (rt.FlatSurface([0, 0, 0], [0, 0, 1], 1), rt.PlaneMirror([0, 0, 0], [0, 0, 1], 1),
              rt.SphericalSurface(1, [0, 0, 1], 1), rt.PerfectLens(1, [0, 0, 0], [0, 0, 1], 0.5)):
        assert not s._rtpb_user_geometry() and not s._rtpb_user_propagate()
    # a system made only of user surfaces never touches the GPU
    s = rt.System([MyFlat([0, 0, 0], [0, 0, 1], 1)], [])
    x = np.ones((2, 8))
    assert s.ray_trace(x, mat.Vacuum(), mat.Vacuum()) is x


def test_plan_cache_never_frees_a_plan_in_use(monkeypatch):
    """LRU eviction only marks a plan that a trace holds; the last user frees it (no use-after-free
    when another thread fills the cache meanwhile).  Library calls are stubbed: no GPU needed."""
    destroyed, created = [], []

    class FakeLib:
        def rtpb_plan_create(self, s, ns, m, nm, dt, out):
            created.append(1)
            out._obj.value = len(created)
            return 0

        def rtpb_plan_destroy(self, p):
            destroyed.append(p.value)
            return 0

    monkeypatch.setattr(C, "lib", lambda: FakeLib())
    monkeypatch.setattr(E, "_PLANS", collections.OrderedDict())
    monkeypatch.setattr(E, "_PLANS_MAX", 2)

    class Low:
        surfaces = materials = None
        nsurf, dtype = 1, 0

        def __init__(self, k):
            self.key = k
    with E.plan_ref(Low("a")) as pa:
        E.plan_for(Low("b"))
        E.plan_for(Low("c"))                 # evicts "a" while it is in use
        assert pa.value not in destroyed
    assert destroyed == [pa.value]           # freed by its last user
    E.plan_for(Low("d"))                     # evicts "b" (unused): freed at once
    assert len(destroyed) == 2


def test_host_generators_per_ray_wavelengths_match_reference_fixtures():
    """The host generators with one wavelength per ray (RT:94, RT:159) against the reference's output."""
    import os
    from parity import GOLDEN, same_bits
    import systems
    d = np.load(os.path.join(GOLDEN, "generators.npz"))
    assert same_bits(rt.get_ray_fan([1., 2., 3.], 0.3, 7, d["fan_wl_wl"], nphis=5), d["fan_wl"])
    assert same_bits(rt.get_ray_fan([0., 0., -5.], 0.02, 11, d["fan_wl3_wl"], nphis=12), d["fan_wl3"])
    assert same_bits(rt.get_ray_fan([0., 0., 0.], 0.2, 5, d["fan_wl1_wl"], nphis=3,
                                    center_ray=tuple(systems.unit([0.6, 0, 0.8]))), d["fan_wl1"])
    assert same_bits(rt.get_collimated_rays([0., 1., -2.], 3., 5, d["coll_wl_wl"], nphis=4, phi_start=0.3),
                     d["coll_wl"])
    assert same_bits(rt.get_collimated_rays([0., 0., 0.], 2., 4, d["coll_wl_tilted_wl"], nphis=3,
                                            normal=[np.sin(0.2), 0, np.cos(0.2)]), d["coll_wl_tilted"])


def test_wavelength_column_follows_numpy_assignment():
    col = rt._wavelength_column(np.float32([0.5, 0.6, 0.7]), 3)
    assert col.dtype == np.float64 and np.array_equal(col, np.float32([0.5, 0.6, 0.7]).astype(np.float64))
    assert rt._wavelength_column(0.5, 10) is None and rt._wavelength_column(np.array([0.5]), 10) is None
    with pytest.raises(ValueError):
        rt._wavelength_column(np.ones(4), 3)


def test_lowering_memo_follows_in_place_changes():
    """The lowering memo is keyed by content: a system changed in place between traces (a material's index, a
    surface's radius, a center array edited element-wise) is lowered again, and changing it back finds the first
    lowering."""
    system = systems.c2_system(rt, mat)
    mats = [mat.Vacuum()] + list(system.materials) + [mat.Vacuum()]
    low0 = E.lower(system.surfaces, mats, None, C.RTPB_F64)
    assert E.lower(system.surfaces, mats, None, C.RTPB_F64) is low0
    const = mat.Constant(1.5)
    mats2 = mats[:1] + [const] + mats[2:]
    a = E.lower(system.surfaces, mats2, None, C.RTPB_F64)
    const._n = 1.6
    b = E.lower(system.surfaces, mats2, None, C.RTPB_F64)
    assert b is not a and bytes(b.materials) != bytes(a.materials)
    sph = next(s for s in system.surfaces if isinstance(s, rt.SphericalSurface))
    r0 = sph.radius
    sph.radius = r0 * 1.01
    c = E.lower(system.surfaces, mats, None, C.RTPB_F64)
    assert c is not low0 and bytes(c.surfaces) != bytes(low0.surfaces)
    sph.radius = r0
    assert E.lower(system.surfaces, mats, None, C.RTPB_F64) is low0
    z0 = system.surfaces[-1].center[2]
    system.surfaces[-1].center[2] = z0 + 1.0
    d = E.lower(system.surfaces, mats, None, C.RTPB_F64)
    assert d is not low0 and bytes(d.surfaces) != bytes(low0.surfaces)
    system.surfaces[-1].center[2] = z0
    assert E.lower(system.surfaces, mats, None, C.RTPB_F64) is low0


def _memo_low(*args):
    r = E.memo_lookup(*args)
    return None if r is None else r[0]


def test_call_memo_follows_every_change():
    """The drop-in call's memo (a repeated System.ray_trace skips the content key) returns the
    previous lowering only while nothing it read can have changed: in-place array edits, attribute rebinding on a
    surface or a material, a swapped surface or medium and another storage type each miss; undoing an in-place
    edit hits again (the bytes match)."""
    system = systems.c2_system(rt, mat)
    m0, m1 = mat.Vacuum(), mat.Vacuum()

    def mats():
        return [m0] + list(system.materials) + [m1]
    low = E.lower(system.surfaces, mats(), None, C.RTPB_F64)
    E.memo_store(system.surfaces, mats(), C.RTPB_F64, low)
    assert _memo_low(system.surfaces, mats(), C.RTPB_F64) is low
    assert _memo_low(system.surfaces, mats(), C.RTPB_F32) is None
    z0 = system.surfaces[-1].center[2]
    system.surfaces[-1].center[2] = z0 + 1.0                      # in place: the bytes differ
    assert _memo_low(system.surfaces, mats(), C.RTPB_F64) is None
    system.surfaces[-1].center[2] = z0
    assert _memo_low(system.surfaces, mats(), C.RTPB_F64) is low
    system.surfaces[-1].normal[2] = system.surfaces[-1].normal[2]     # an int64 normal array, unchanged bytes
    assert _memo_low(system.surfaces, mats(), C.RTPB_F64) is low
    sph = system.surfaces[1]
    sph.radius = sph.radius                                          # any rebinding counts
    assert _memo_low(system.surfaces, mats(), C.RTPB_F64) is None
    E.memo_store(system.surfaces, mats(), C.RTPB_F64, low)
    m0.b1 = m0.b1                                                    # a material attribute
    assert _memo_low(system.surfaces, mats(), C.RTPB_F64) is None
    E.memo_store(system.surfaces, mats(), C.RTPB_F64, low)
    assert _memo_low(system.surfaces, [mat.Vacuum()] + mats()[1:], C.RTPB_F64) is None   # another medium
    old = system.surfaces[0]
    system.surfaces[0] = rt.FlatSurface(old.center, old.normal, old.aperture_rad)            # another surface
    assert _memo_low(system.surfaces, mats(), C.RTPB_F64) is None
    system.surfaces[0] = old
    assert _memo_low(system.surfaces, mats(), C.RTPB_F64) is None    # (constructing a surface counted too)
    E.memo_store(system.surfaces, mats(), C.RTPB_F64, low)
    assert _memo_low(system.surfaces, mats(), C.RTPB_F64) is low
    del sph.radius                                                   # deletion counts too
    assert _memo_low(system.surfaces, mats(), C.RTPB_F64) is None


def test_call_memo_of_tabulated_systems():
    """A tabulated system's memo (Ebaf11: the previous bundle's table keys, still checked by the kernel's table-miss
    flag) holds only while the key sets are unchanged (any remember_keys) and the material's coefficient list is
    unchanged in place."""
    system = systems.c3_system(rt, mat)
    m0 = m1 = mat.Vacuum()
    mats = [m0] + list(system.materials) + [m1]
    eb = next(m for m in mats if type(m).__name__ == "Ebaf11")
    low = E.lower(system.surfaces, mats, lambda: np.array([0.635]), C.RTPB_F32)
    E.memo_store(system.surfaces, mats, C.RTPB_F32, low, tabulated=True)
    assert E.memo_lookup(system.surfaces, mats, C.RTPB_F32) == (low, True)
    p0 = eb.params[0]
    eb.params[0] = p0 * 1.001                                    # in place: no __setattr__
    assert E.memo_lookup(system.surfaces, mats, C.RTPB_F32) is None
    eb.params[0] = p0
    assert E.memo_lookup(system.surfaces, mats, C.RTPB_F32) == (low, True)
    E.remember_keys(None, np.array([0.5]))                     # some key set changed
    assert E.memo_lookup(system.surfaces, mats, C.RTPB_F32) is None
