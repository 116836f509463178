"""GPU parity: the HIP path (librtpb.so through the C ABI) against the reference's golden vectors and
the NumPy oracle.  Float64 results must be BIT-IDENTICAL (NaN pattern included); float32 results
must agree with the float64 oracle to rtol 1e-5 (column-scaled)."""
import ctypes
import json
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import ray_trace_pb_amd.materials as mat  # noqa: E402
import ray_trace_pb_amd.raytrace as rt  # noqa: E402
from ray_trace_pb_amd import _capi as C  # noqa: E402
from ray_trace_pb_amd import _engine as E  # noqa: E402
from oracle import rt_numpy as O  # noqa: E402
from parity import same_bits, CASES, F32IN_CASES, GOLDEN, compare, load_case  # noqa: E402
from serialize import material_to_dict, surface_to_dict, system_from_json  # noqa: E402
import systems  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def build_case(name):
    d = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    system, m0, m1 = system_from_json(rt, mat, str(d["system_json"]))
    return system, m0, m1, d["rays_in"], d["history"]


def oracle(system, m0, m1, rays):
    return O.ray_trace([surface_to_dict(s) for s in system.surfaces],
                       [material_to_dict(m) for m in [m0] + list(system.materials) + [m1]], rays)


@pytest.mark.parametrize("name", CASES)
def test_numpy_path_bitwise_vs_reference(name):
    system, m0, m1, rays, ref = build_case(name)
    got = system.ray_trace(rays, m0, m1)
    assert isinstance(got, np.ndarray) and got.dtype == np.float64 and got.flags.c_contiguous
    assert got.shape == ref.shape
    assert same_bits(got, ref)


@pytest.mark.parametrize("name", CASES)
def test_device_path_bitwise_vs_reference(name):
    system, m0, m1, rays, ref = build_case(name)
    got = system.ray_trace(torch.from_numpy(rays).to(DEV), m0, m1)
    torch.cuda.synchronize()
    assert got.is_cuda and got.dtype == torch.float64
    assert same_bits(got.cpu().numpy(), ref)


def test_input_ranks_and_extend_history():
    d = np.load(os.path.join(GOLDEN, "shapes.npz"))
    system, m0, m1 = system_from_json(rt, mat, str(d["system_json"]))
    for k in ("1", "2", "3"):
        got = system.ray_trace(d["rays" + k], m0, m1)
        assert got.shape == d["out" + k].shape, k
        assert same_bits(got, d["out" + k]), k
        got_t = system.ray_trace(torch.from_numpy(np.ascontiguousarray(d["rays" + k])).to(DEV), m0, m1)
        assert same_bits(got_t.cpu().numpy(), d["out" + k]), k


def test_surface_propagate_appends_two_planes():
    system, m0, m1, rays, ref = build_case("c1_plano_convex")
    mats = [m0] + list(system.materials) + [m1]
    h = rays
    for i, s in enumerate(system.surfaces):
        h = s.propagate(h, mats[i], mats[i + 1])
    assert same_bits(h, ref)


def test_large_bundle_bitwise_vs_oracle_subsample():
    """C2 at the full BASELINE size (1M rays): GPU vs the oracle on a 100k-ray random subsample."""
    system = systems.c2_system(rt, mat)
    rays = systems.c2_rays(1_000_000)
    got = system.ray_trace(rays, mat.Vacuum(), mat.Vacuum())
    idx = np.random.default_rng(0).choice(rays.shape[0], 100_000, replace=False)
    ref = oracle(system, mat.Vacuum(), mat.Vacuum(), rays[idx])
    assert same_bits(got[:, idx], ref)


def test_full_size_properties_c2():
    """Size-independent properties at full size: unit directions, Snell invariant at the flats,
    OPL monotone along the ray, wavelengths preserved."""
    system = systems.c2_system(rt, mat)
    rays = systems.c2_rays(1_000_000)
    h = system.ray_trace(torch.from_numpy(rays).to(DEV), mat.Vacuum(), mat.Vacuum()).cpu().numpy()
    live = ~np.isnan(h[-1]).any(axis=1)
    assert live.mean() > 0.99
    d = h[:, live, 3:6]
    assert np.allclose(np.linalg.norm(d, axis=-1), 1.0, atol=1e-12)
    assert np.array_equal(h[:, live, 7], np.broadcast_to(rays[live, 7], (h.shape[0], live.sum())))
    assert np.all(np.diff(h[:, live, 6], axis=0) >= -1e-9)
    # flat at z=0 between vacuum and vacuum: direction unchanged
    assert np.array_equal(h[2, live, 3:6], h[0, live, 3:6])


def test_planes_final_and_subset_match_full():
    system, m0, m1, rays, ref = build_case("c5_odt")
    fin = system.ray_trace(rays, m0, m1, planes="final")
    assert fin.shape == (1,) + ref.shape[1:]
    assert same_bits(fin[0], ref[-1])
    sel = [0, 3, 4, 17, 28]
    sub = system.ray_trace(rays, m0, m1, planes=sel)
    assert same_bits(sub, ref[sel])
    t = system.ray_trace(torch.from_numpy(rays).to(DEV), m0, m1, planes=[1, 28])
    assert same_bits(t.cpu().numpy(), ref[[1, 28]])


def test_soa_layout_matches_aos():
    system, m0, m1, rays, ref = build_case("stress")
    soa = system.ray_trace(torch.from_numpy(rays).to(DEV), m0, m1, layout="soa")
    assert tuple(soa.shape) == (ref.shape[0], 8, ref.shape[1])
    assert same_bits(soa.transpose(1, 2).cpu().numpy(), ref)


@pytest.mark.parametrize("knob", [("aos_staging", 0), ("nt_stores", 0), ("stage_input", 1)])
def test_tuning_variants_bitwise(knob):
    """Every store/load strategy is a pure data-movement change: bit-identical histories."""
    system, m0, m1, rays, ref = build_case("stress")
    lib = C.lib()
    default = {"aos_staging": 1, "nt_stores": 1, "stage_input": 0}[knob[0]]
    C.check(lib.rtpb_set_tuning(knob[0].encode(), knob[1]))
    try:
        r32 = rays.astype(np.float32)
        ref32 = oracle(system, m0, m1, r32.astype(np.float64))
        for dt, r, exp in (("float64", rays, ref), ("float32", r32, ref32.astype(np.float32)),
                           ("float32", rays, ref.astype(np.float32)), ("float64", r32, ref32)):
            got = system.ray_trace(torch.from_numpy(r).to(DEV), m0, m1, dtype=dt).cpu().numpy()
            assert same_bits(got, exp), (knob, dt, r.dtype)
    finally:
        C.check(lib.rtpb_set_tuning(knob[0].encode(), default))


def test_lens_and_flat_kernel_variant_every_store_path():
    """C4's OPM -- PerfectLens and Flat surfaces in the axial and x-z forms only, so its plan takes the lens-and-flat
    kernel variant (rtpb_plan::feat 33, dispatch_kind's kKindsLensFlat) -- through every store path of that variant:
    float64 / float32 storage, AOS and SoA, the final plane, a plane subset, float32 input and each tuning knob."""
    system, m0, m1, rays, ref = build_case("c4_opm")
    assert {type(s).__name__ for s in system.surfaces} == {"PerfectLens", "FlatSurface"}
    r32 = rays.astype(np.float32)
    ref32 = oracle(system, m0, m1, r32.astype(np.float64))
    lib = C.lib()

    def run(r, **kw):
        out = system.ray_trace(torch.from_numpy(r).to(DEV), m0, m1, **kw)
        return out.cpu().numpy()

    def sweep(tag):
        for r, exp in ((rays, ref), (r32, ref32)):
            for dt, e in (("float64", exp), ("float32", exp.astype(np.float32))):
                assert same_bits(run(r, dtype=dt), e), (tag, r.dtype, dt, "all")
                assert same_bits(run(r, dtype=dt, planes="final")[0], e[-1]), (tag, r.dtype, dt, "final")
                assert same_bits(run(r, dtype=dt, planes=[1, 5, 22]), e[[1, 5, 22]]), (tag, r.dtype, dt, "subset")
                soa = run(r, dtype=dt, layout="soa")
                assert same_bits(np.swapaxes(soa, 1, 2), e), (tag, r.dtype, dt, "soa")

    sweep("default")
    for knob, value, default in (("aos_staging", 0, 1), ("aos_staging", 2, 1), ("nt_stores", 0, 1),
                                 ("stage_input", 1, 0)):
        C.check(lib.rtpb_set_tuning(knob.encode(), value))
        try:
            sweep(f"{knob}={value}")
        finally:
            C.check(lib.rtpb_set_tuning(knob.encode(), default))


def test_sharded_host_trace_is_bitwise_equal():
    """Ray sharding over devices (here: two shards on GPU 0) gives exactly the unsharded history."""
    system, m0, m1, rays, ref = build_case("stress")
    got = system.ray_trace(rays, m0, m1, devices=[0, 0])
    assert same_bits(got, ref)
    got3 = system.ray_trace(rays, m0, m1, devices=[0, 0, 0])
    assert same_bits(got3, ref)


@pytest.mark.parametrize("name", [c for c in CASES if c.startswith("fuzz_")])
def test_fuzz_sharded_host_trace_and_float32_storage(name):
    """The seeded random systems through rtpb_trace_host split over three shards of GPU 0 (host threads,
    chunked pipeline), float64 and float32 storage, all and final planes: the reference's history
    (rounded once for float32) bit for bit."""
    system, m0, m1, rays, ref = build_case(name)
    assert same_bits(system.ray_trace(rays, m0, m1, devices=[0, 0, 0]), ref)
    got32 = system.ray_trace(rays, m0, m1, dtype="float32", devices=[0, 0, 0])
    assert same_bits(got32, ref.astype(np.float32))
    fin = system.ray_trace(rays, m0, m1, planes="final", devices=[0, 0])
    assert same_bits(fin, ref[-1:])


def test_user_material_subclass_lowers_to_table():
    """A Material subclass overriding n() (the reference's plugin point) traces on the GPU via a
    per-wavelength table, bit-identical to evaluating its n() per ray."""
    system, m0, m1, rays, ref = build_case("stress")
    assert any(type(m).__name__ == "Cauchy" for m in system.materials)
    got = system.ray_trace(rays, m0, m1)
    assert same_bits(got, ref)


@pytest.mark.parametrize("name", CASES)
def test_float32_storage_of_float64_input_is_the_rounded_reference(name):
    """dtype='float32' is float32 STORAGE: float64 rays are read as float64 and traced in float64, so the
    history is the reference's float64 history rounded once to float32 -- bit for bit, NaN pattern
    included (no ray the reference keeps is lost), hence within 1e-5 column-scaled with no mask flip.
    NumPy and torch paths, all planes / final plane / SoA (the mixed-type kernel variants)."""
    system, m0, m1, rays, ref = build_case(name)
    exp = ref.astype(np.float32)
    got = system.ray_trace(rays, m0, m1, dtype="float32")
    assert got.dtype == np.float32 and same_bits(got, exp)
    ok, rep = compare(got, ref, rtol=1e-5)
    assert ok and rep["mask_flips"] == 0, rep
    x = torch.from_numpy(rays).to(DEV)
    got_t = system.ray_trace(x, m0, m1, dtype="float32")
    assert got_t.dtype == torch.float32 and same_bits(got_t.cpu().numpy(), exp)
    fin = system.ray_trace(x, m0, m1, dtype="float32", planes="final")
    assert same_bits(fin.cpu().numpy(), exp[-1:])
    soa = system.ray_trace(x, m0, m1, dtype="float32", layout="soa")
    assert same_bits(soa.transpose(1, 2).cpu().numpy(), exp)


@pytest.mark.parametrize("name", CASES + F32IN_CASES)
def test_float32_input_bitwise_vs_oracle_on_widened_input(name):
    """float32 rays are widened exactly in the kernel (as NumPy promotes them) and traced in float64:
    float32 storage gives the oracle's float64 trace of the widened input rounded once, float64 storage
    gives it exactly."""
    system, m0, m1, rays, ref = build_case(name)
    r32 = rays.astype(np.float32)
    full = oracle(system, m0, m1, r32.astype(np.float64))
    exp = full.astype(np.float32)
    got = system.ray_trace(r32, m0, m1, dtype="float32")
    assert got.dtype == np.float32
    assert same_bits(got, exp)
    got_t = system.ray_trace(torch.from_numpy(r32).to(DEV), m0, m1, dtype="float32")
    assert got_t.dtype == torch.float32 and same_bits(got_t.cpu().numpy(), exp)
    got64 = system.ray_trace(r32, m0, m1)
    assert got64.dtype == np.float64 and same_bits(got64, full)
    got64_t = system.ray_trace(torch.from_numpy(r32).to(DEV), m0, m1)
    assert got64_t.dtype == torch.float64 and same_bits(got64_t.cpu().numpy(), full)


@pytest.mark.parametrize("name", F32IN_CASES)
def test_float32_input_vs_reference_run_on_float32_input(name):
    """Against the reference handed the SAME float32 arrays (fixtures <recipe>_f32in): NaN masks
    identical, values within 1e-6 column-scaled for float64 storage and 1e-5 for float32 storage.  (Not
    bitwise: NumPy evaluates a few first-surface sub-expressions of the reference in float32, see
    tests/test_oracle_golden.py.)"""
    system, m0, m1, rays, ref = build_case(name)
    assert rays.dtype == np.float32
    for dt, rtol in ((None, 1e-6), ("float32", 1e-5)):
        got = system.ray_trace(rays, m0, m1, dtype=dt)
        ok, rep = compare(got, ref, rtol=rtol)
        assert ok and rep["mask_flips"] == 0, (dt, rep)


def test_float32_storage_c4_fan_40k_rays():
    """BASELINE C4 (ideal OPM, six PerfectLenses + tilted flats) on a 201 x 200 = 40,200-ray fan of the
    script's shape, float32 storage of the float64 fan: the float64 oracle history rounded to float32,
    bit for bit (the NA clip of RT:1757-1760 keeps exactly the reference's rays), NumPy fan and
    device-generated fan."""
    system, m0, m1 = systems.c4_system(rt, mat), mat.Constant(systems.OPM_N1), mat.Vacuum()
    theta = 30 * np.pi / 180
    args = ([1e-3, 1e-3, 1e-3 * np.tan(theta)], np.arcsin(1.35 / systems.OPM_N1), 201, systems.OPM_WAVELENGTH)
    fan = rt.get_ray_fan(*args, nphis=200)
    assert fan.shape == (40200, 8) and fan.dtype == np.float64
    ref = oracle(system, m0, m1, fan)
    killed = np.isnan(ref[-1]).all(axis=1).sum()
    assert 0 < killed < fan.shape[0]                      # the NA clip is exercised
    got = system.ray_trace(fan, m0, m1, dtype="float32")
    assert same_bits(got, ref.astype(np.float32))
    ok, rep = compare(got, ref, rtol=1e-5)
    assert ok and rep["mask_flips"] == 0, rep
    fan_d = rt.get_ray_fan(*args, nphis=200, device=DEV)
    got_d = system.ray_trace(fan_d, m0, m1, dtype="float32")
    assert same_bits(got_d.cpu().numpy(), ref.astype(np.float32))


def test_kat_perfect_lens_equal_phase():
    """scripts/2021_10_28_test_perfect_lens_phase.py: a tilted plane wave focuses in phase."""
    system, rays, m0, m1 = systems.kat_perfect_lens_phase(rt, mat)
    out = system.ray_trace(rays, m0, m1)
    assert np.ptp(out[-1, :, 6]) == 0.0


def test_kat_plano_convex_opl_analytic():
    """scripts/2022_10_27_plano_convex_lens.py:39-59: traced OPL equals the analytic formula."""
    system, rays, m0, m1 = systems.c1_plano_convex(rt, mat, nrays=101)
    out = system.ray_trace(rays, m0, m1)
    n, R, t0, t1, dz, k = 1.3, 100, 2.679486355, 1, 5, 2 * np.pi / 0.5
    h = rays[:, 0]
    opl = (dz + n * t0 + n * t1 - n * (R - np.sqrt(R ** 2 - h ** 2)) +
           (R - np.sqrt(R ** 2 - h ** 2)) / (np.sqrt(1 - n ** 2 * h ** 2 / R ** 2) * np.sqrt(R ** 2 - h ** 2) / R +
                                             n * h ** 2 / R ** 2))
    assert np.max(np.abs(out[-1, :, 6] / k - opl)) < 1e-12


@pytest.mark.parametrize("kw", [dict(pt=[0.5, -0.25, 1.0], th=0.3, nt=101, nph=64, c=(0, 0, 1)),
                                dict(pt=[1e-3, 1e-3, 1e-3 * np.tan(np.pi / 6)], th=np.arcsin(1.35 / 1.4), nt=1001,
                                     nph=1000, c=(0, 0, 1)),
                                dict(pt=[0., 2., -1.], th=0.5 * np.pi / 180, nt=317, nph=316,
                                     c=(0.6, 0.0, 0.8))])
def test_device_ray_fan_bitwise_vs_host_generator(kw):
    """The device fan equals the reference-style NumPy fan bit for bit (1M rays in the C4-shaped case)."""
    fan_h = rt.get_ray_fan(kw["pt"], kw["th"], kw["nt"], 0.635, nphis=kw["nph"], center_ray=kw["c"])
    fan_d = rt.get_ray_fan(kw["pt"], kw["th"], kw["nt"], 0.635, nphis=kw["nph"], center_ray=kw["c"],
                           device=DEV).cpu().numpy()
    assert fan_d.shape == fan_h.shape
    assert np.array_equal(fan_d, fan_h)
    f32 = rt.get_ray_fan(kw["pt"], kw["th"], kw["nt"], 0.635, nphis=kw["nph"], center_ray=kw["c"], device=DEV,
                         dtype="float32").cpu().numpy()
    assert np.array_equal(f32, fan_h.astype(np.float32))


def test_errors_are_loud():
    system, m0, m1, rays, _ = build_case("c1_plano_convex")
    with pytest.raises(ValueError):
        system.ray_trace(rays, m0, m1, planes=[99])
    with pytest.raises(ValueError):
        rt.System(system.surfaces, system.materials).ray_trace(rays, m0, m1, planes="bogus")
    with pytest.raises(C.RtpbError):
        system.ray_trace(rays, m0, m1, devices=[1000])


def test_empty_bundle():
    system, m0, m1, rays, _ = build_case("c1_plano_convex")
    out = system.ray_trace(rays[:0], m0, m1)
    assert out.shape == (7, 0, 8)
    out = system.ray_trace(torch.zeros((0, 8), dtype=torch.float64, device=DEV), m0, m1)
    assert tuple(out.shape) == (7, 0, 8)


def test_timing_counters():
    system, m0, m1, rays, _ = build_case("c2_achromat")
    lib = C.lib()
    lib.rtpb_timing_enable(1)
    x = torch.from_numpy(rays).to(DEV)
    for _ in range(3):
        system.ray_trace(x, m0, m1)
    tot, cnt = ctypes.c_double(), ctypes.c_int64()
    C.check(lib.rtpb_timing_collect(ctypes.byref(tot), ctypes.byref(cnt)))
    lib.rtpb_timing_enable(0)
    assert cnt.value == 3 and tot.value > 0


def test_user_surface_with_own_propagate_runs_between_gpu_segments():
    """A Surface subclass supplying its own propagate (the reference's plugin point) is called with the
    growing history; built-in surfaces around it run as fused GPU traces.  Here the user surface is a
    FlatSurface whose propagate delegates to the oracle, so the whole history must equal the reference."""
    system, m0, m1, rays, ref = build_case("c5_odt")

    class OracleFlat(rt.FlatSurface):
        calls = 0

        def propagate(self, ray_array, material1, material2):
            OracleFlat.calls += 1
            h = np.asarray(ray_array)
            sd = surface_to_dict(self)
            sd["type"] = "FlatSurface"
            return O.ray_trace([sd], [material_to_dict(material1), material_to_dict(material2)], h)

    surfs = list(system.surfaces)
    last = surfs[-1]
    surfs[-1] = OracleFlat(last.center, last.normal, last.aperture_rad)
    custom = rt.System(surfs, system.materials)
    got = custom.ray_trace(rays, m0, m1)
    assert OracleFlat.calls == 1
    assert same_bits(got, ref)
    with pytest.raises(ValueError):
        custom.ray_trace(rays, m0, m1, planes="final")


# ---------------------------------------------------------------- user geometry hooks (RT:1071-1156)
# Surface subclasses written the way a reference user writes them: own get_intersect / get_normal /
# is_pt_on_surface (the reference's formulas, restated here with NumPy -- or torch for device
# histories), inheriting RefractingSurface / ReflectingSurface.propagate.
def _xp(a):
    return torch if torch.is_tensor(a) else np


def _rows(pts):
    return pts if torch.is_tensor(pts) else np.atleast_2d(pts)


def _norm3(v):
    return _xp(v).sqrt((v[..., 0] * v[..., 0] + v[..., 1] * v[..., 1]) + v[..., 2] * v[..., 2])


def _tile(vec, pts):
    pts = _rows(pts)
    if torch.is_tensor(pts):
        return torch.as_tensor(vec, device=pts.device).expand(pts.shape[0], 3)
    return np.tile(vec, (pts.shape[0], 1))


def _on_plane(pts, center, normal, aperture):
    pts = _rows(pts)
    rel = pts[..., 0:3] - (torch.as_tensor(center, device=pts.device) if torch.is_tensor(pts) else center)
    dot = (rel[..., 0] * normal[0] + rel[..., 1] * normal[1]) + rel[..., 2] * normal[2]
    return (abs(dot) < 1e-12) & (_norm3(rel) <= aperture)


class UserFlat(rt.RefractingSurface):
    def __init__(self, center, normal, aperture_rad):
        self.normal = np.asarray(normal, dtype=float)
        super().__init__(self.normal, self.normal, center, center, aperture_rad)

    def get_normal(self, pts):
        return _tile(self.normal, pts)

    def get_intersect(self, rays, material):
        return rt.propagate_ray2plane(rays, self.normal, self.center, material, exclude_backward_propagation=True)[0]

    def is_pt_on_surface(self, pts):
        return _on_plane(pts, self.center, self.normal, self.aperture_rad)


class UserMirror(rt.ReflectingSurface):
    def __init__(self, center, normal, aperture_rad):
        self.normal = np.asarray(normal, dtype=float)
        super().__init__(self.normal, self.normal, center, center, aperture_rad)

    def get_normal(self, pts):
        return _tile(self.normal, pts)

    def get_intersect(self, rays, material):
        out, ts = rt.propagate_ray2plane(rays, self.normal, self.center, material)
        out[ts < 0] = float("nan")
        return out

    def is_pt_on_surface(self, pts):
        return _on_plane(pts, self.center, self.normal, self.aperture_rad)


class UserSphere(rt.RefractingSurface):
    def __init__(self, radius, center, aperture_rad, input_axis):
        self.radius = radius
        ax = np.asarray(input_axis, dtype=float)
        super().__init__(ax, ax, center, np.asarray(center) - radius * ax, aperture_rad)

    def get_normal(self, pts):
        pts = np.atleast_2d(pts)[:, :3]
        return (pts - self.center[None, :]) / self.radius

    def get_intersect(self, rays, material):
        rays = np.atleast_2d(rays)
        xo, yo, zo, dx, dy, dz, ph, wl = rays.T
        xc, yc, zc = self.center
        B = 2 * (dx * (xo - xc) + dy * (yo - yc) + dz * (zo - zc))
        Cq = (xo - xc) ** 2 + (yo - yc) ** 2 + (zo - zc) ** 2 - self.radius ** 2
        with np.errstate(invalid="ignore"):
            ts = np.stack((0.5 * (-B + np.sqrt(B ** 2 - 4 * Cq)), 0.5 * (-B - np.sqrt(B ** 2 - 4 * Cq))), axis=1)
            ts[ts < 0] = np.inf
        t = np.min(ts, axis=1)
        t[t == np.inf] = np.nan
        p0 = np.stack((xo, yo, zo), axis=1)
        pts = p0 + np.stack((dx, dy, dz), axis=1) * t[:, None]
        shift = np.linalg.norm(pts - p0, axis=1) * 2 * np.pi / wl * material.n(wl)
        return np.concatenate((pts, np.stack((dx, dy, dz, ph + shift, wl), axis=1)), axis=1)

    def is_pt_on_surface(self, pts):
        pts = np.atleast_2d(pts)
        dist = np.linalg.norm(pts[..., 0:3] - self.center, axis=-1)
        ortho = pts[..., :3] - np.sum(pts[..., :3] * self.input_axis, axis=-1)[..., None] * self.input_axis
        return (np.abs(dist - abs(self.radius)) < 1e-12) & (np.linalg.norm(ortho, axis=-1) <= self.aperture_rad)


def _hooked(system, spheres=True):
    out = []
    for s in system.surfaces:
        if type(s) is rt.FlatSurface:
            out.append(UserFlat(s.center, s.normal, s.aperture_rad))
        elif type(s) is rt.PlaneMirror:
            out.append(UserMirror(s.center, s.normal, s.aperture_rad))
        elif type(s) is rt.SphericalSurface and spheres:
            out.append(UserSphere(s.radius, s.center, s.aperture_rad, s.input_axis))
        else:
            out.append(s)
    return rt.System(out, system.materials)


@pytest.mark.parametrize("name", ["stress", "c4_mirror", "c2_achromat", "tir_prism", "c1_plano_convex"] +
                         [c for c in CASES if c.startswith("fuzz_")])
def test_user_geometry_hooks_bitwise_vs_reference(name):
    """User geometry hooks + GPU front-side / Snell / reflection reproduce the reference history
    exactly, including misses, back-facing rays, TIR, aperture clipping and user materials."""
    system, m0, m1, rays, ref = build_case(name)
    hooked = _hooked(system)
    n_user = sum(s._rtpb_user_geometry() for s in hooked.surfaces)
    assert n_user >= 1
    got = hooked.ray_trace(rays, m0, m1)
    assert got.shape == ref.shape
    assert same_bits(got, ref)
    # one surface through Surface.propagate on its own
    s0 = hooked.surfaces[0]
    if s0._rtpb_user_geometry():
        mats = [m0] + list(system.materials) + [m1]
        one = s0.propagate(rays, mats[0], mats[1])
        assert same_bits(one, ref[:3])


def test_user_geometry_hooks_on_device_history():
    """torch CUDA histories: the hooks receive torch tensors and the result stays on the device."""
    system, m0, m1, rays, ref = build_case("c4_mirror")
    hooked = _hooked(system, spheres=False)
    assert any(s._rtpb_user_geometry() for s in hooked.surfaces)
    got = hooked.ray_trace(torch.from_numpy(rays).to(DEV), m0, m1)
    assert got.is_cuda
    assert same_bits(got.cpu().numpy(), ref)


@pytest.mark.parametrize("material", ["Ebaf11", "Nsf11", "Bk7", "Cauchy"])
def test_material_dispersion_bitwise_over_wavelength_sweep(material):
    """n(lambda) of every material kind reproduced bit for bit over 20k distinct wavelengths (the
    golden cases use a handful): a tilted slab of the material, rays of random colour."""
    m = systems.cauchy_class(mat)() if material == "Cauchy" else getattr(mat, material)()
    system = rt.System([rt.FlatSurface([0, 0, 0], [0, 0, 1], 50),
                        rt.FlatSurface([0, 0, 5], systems.unit([0.2, 0, 1]), 50)], [m])
    rng = np.random.default_rng(7)
    n = 20000
    rays = np.zeros((n, 8))
    rays[:, 0:2] = rng.uniform(-5, 5, (n, 2))
    rays[:, 2] = -1.0
    d = np.stack((rng.normal(scale=0.1, size=n), rng.normal(scale=0.1, size=n), np.ones(n)), axis=1)
    rays[:, 3:6] = d / np.linalg.norm(d, axis=1)[:, None]
    rays[:, 7] = rng.uniform(0.35, 2.0, n)
    got = system.ray_trace(rays, mat.Vacuum(), mat.Vacuum())
    ref = oracle(system, mat.Vacuum(), mat.Vacuum(), rays)
    assert same_bits(got, ref)


@pytest.mark.parametrize("n_wl", [1, 127, 128, 129, 255, 256, 257])
def test_table_materials_lds_and_global_lookup(n_wl):
    """TABLE materials (Ebaf11 + a user Material subclass) around the LDS-table size limit: kernels copy
    the plan's (wavelength, n) pairs into LDS when all of them fit (kLdsTablePairs = 256 pairs in total,
    here 2 * n_wl), else they search global memory.  Every variant is bit-exact vs the oracle: NumPy path,
    torch path, float32 storage, and the unstaged four-wave-workgroup kernels."""
    system = rt.System([rt.FlatSurface([0, 0, 0], [0, 0, 1], 50),
                        rt.SphericalSurface.get_on_axis(40.0, 5.0, 30.0),
                        rt.FlatSurface([0, 0, 12], systems.unit([0.1, 0, 1]), 50)],
                       [mat.Ebaf11(), systems.cauchy_class(mat)()])
    rng = np.random.default_rng(n_wl)
    n = 4099
    rays = np.zeros((n, 8))
    rays[:, 0:2] = rng.uniform(-8, 8, (n, 2))
    rays[:, 2] = -1.0
    d = np.stack((rng.normal(scale=0.05, size=n), rng.normal(scale=0.05, size=n), np.ones(n)), axis=1)
    rays[:, 3:6] = d / np.linalg.norm(d, axis=1)[:, None]
    wls = np.linspace(0.4, 1.6, n_wl)
    rays[:, 7] = wls[rng.integers(0, n_wl, n)]
    m0, m1 = mat.Vacuum(), mat.Vacuum()
    ref = oracle(system, m0, m1, rays)
    assert same_bits(system.ray_trace(rays, m0, m1), ref)
    x = torch.from_numpy(rays).to(DEV)
    assert same_bits(system.ray_trace(x, m0, m1).cpu().numpy(), ref)
    r32 = rays.astype(np.float32)
    exp32 = oracle(system, m0, m1, r32.astype(np.float64)).astype(np.float32)
    got32 = system.ray_trace(torch.from_numpy(r32).to(DEV), m0, m1, dtype="float32").cpu().numpy()
    assert same_bits(got32, exp32)
    # float64 rays into float32 storage: the table keys are the rays' own float64 wavelengths
    got32_64 = system.ray_trace(x, m0, m1, dtype="float32").cpu().numpy()
    assert same_bits(got32_64, ref.astype(np.float32))
    assert np.isfinite(got32_64[-1, :, 0]).sum() > n // 2
    lib = C.lib()
    C.check(lib.rtpb_set_tuning(b"aos_staging", 0))
    try:
        assert same_bits(system.ray_trace(x, m0, m1).cpu().numpy(), ref)
    finally:
        C.check(lib.rtpb_set_tuning(b"aos_staging", 1))


def test_more_than_2_31_rays_in_one_launch():
    """Maximum sizes: one trace of 2^31 + 4633 rays (int64 ray indexing, > 2^25 workgroups), float32
    storage, final plane only (68.7 GB in + 68.7 GB out of HBM).  Rays on both sides of index 2^31 and
    at the very end are bit-exact against the oracle on the same float32 input."""
    system, m0, m1, _, _ = build_case("c1_plano_convex")
    nt = nph = 46341                                  # 46341^2 = 2^31 + 4633
    n = nt * nph
    assert n > 2 ** 31
    rays = torch.empty((n, 8), dtype=torch.float32, device=DEV)
    rt.fan_into(rays, [0.0, 0.0, -5.0], 0.2, nt, 0.5, nph)
    out = system.ray_trace(rays, m0, m1, planes="final", dtype="float32")
    assert out.shape == (1, n, 8)
    picks = np.r_[0:64, 2 ** 31 - 2048:2 ** 31 + 2048, n - 2048:n]
    idx = torch.from_numpy(picks).to(DEV)
    r_in = rays.index_select(0, idx).double().cpu().numpy()
    got = out[0].index_select(0, idx).cpu().numpy()
    del rays, out
    torch.cuda.empty_cache()
    ref = oracle(system, m0, m1, r_in)[-1].astype(np.float32)
    assert same_bits(got, ref)
    assert np.isfinite(got[:, 0]).sum() > 1000        # not an all-NaN comparison


def test_concurrent_host_threads_give_identical_results():
    """Several Python threads tracing different systems at once (NumPy and torch paths, shared plan
    cache, one device): every result equals its single-threaded trace."""
    import threading
    cases = ["c1_plano_convex", "c2_achromat", "c4_mirror", "stress"]
    built = [build_case(c) for c in cases]
    want = [b[4] for b in built]
    got = [[None] * 3 for _ in cases]
    errors = []

    def work(k):
        try:
            system, m0, m1, rays, _ = built[k]
            for it in range(3):
                if it % 2:
                    got[k][it] = system.ray_trace(torch.from_numpy(rays).to(DEV), m0, m1).cpu().numpy()
                else:
                    got[k][it] = system.ray_trace(rays, m0, m1)
        except Exception as e:  # noqa: BLE001
            errors.append(e)
    th = [threading.Thread(target=work, args=(k,)) for k in range(len(cases))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    for k in range(len(cases)):
        for it in range(3):
            assert same_bits(got[k][it], want[k]), (cases[k], it)


def test_snell_and_reflection_invariants_at_full_size():
    """SURVEY §4 property tests on 1M-ray bundles: at every refracting sphere of C2,
    n1 |d_in x N| = n2 |d_out x N| and d_in, N, d_out are coplanar; at the C4 mirror the normal
    component flips and the tangential one is kept (angle in = angle out)."""
    system = systems.c2_system(rt, mat)
    rays = systems.c2_rays(1_000_000)
    h = system.ray_trace(torch.from_numpy(rays).to(DEV), mat.Vacuum(), mat.Vacuum()).cpu().numpy()
    mats = [mat.Vacuum()] + list(system.materials) + [mat.Vacuum()]
    wl = rays[:, 7]
    checked = 0
    for i, s in enumerate(system.surfaces):
        if type(s) is not rt.SphericalSurface:
            continue
        at, after, before = h[2 * i + 1], h[2 * i + 2], h[2 * i]
        live = ~np.isnan(after).any(axis=1)
        N = (at[live, :3] - s.center) / s.radius
        d1, d2 = before[live, 3:6], after[live, 3:6]
        n1, n2 = mats[i].n(wl[live]), mats[i + 1].n(wl[live])
        s1 = np.linalg.norm(np.cross(d1, N), axis=1)
        s2 = np.linalg.norm(np.cross(d2, N), axis=1)
        np.testing.assert_allclose(n1 * s1, n2 * s2, rtol=0, atol=1e-12)
        assert np.max(np.abs(np.sum(np.cross(d1, N) * d2, axis=1))) < 1e-12
        checked += live.sum()
    assert checked > 2_000_000
    # mirror: a tilted PlaneMirror hit by a 1M-ray fan
    mirror = rt.System([rt.PlaneMirror([0, 0, 10], systems.unit([0.0, 0.3, -1.0]), 50)], [])
    fan = rt.get_ray_fan([0, 0, 0], 0.2, 1001, 0.5, nphis=1000, device=DEV)
    hm = mirror.ray_trace(fan, mat.Vacuum(), mat.Vacuum()).cpu().numpy()
    live = ~np.isnan(hm[2]).any(axis=1)
    assert live.mean() > 0.99
    N = systems.unit([0.0, 0.3, -1.0])
    din, dout = hm[0, live, 3:6], hm[2, live, 3:6]
    np.testing.assert_allclose(dout @ N, -(din @ N), rtol=0, atol=1e-14)
    np.testing.assert_allclose(dout - (dout @ N)[:, None] * N, din - (din @ N)[:, None] * N, rtol=0, atol=1e-14)
