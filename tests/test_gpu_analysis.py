"""GPU: device ray generators and device analysis against the reference's
host semantics (golden vectors) and NumPy."""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import ray_trace_pb_amd.materials as mat  # noqa: E402
import ray_trace_pb_amd.raytrace as rt  # noqa: E402
from ray_trace_pb_amd import analysis  # noqa: E402
from oracle import rt_numpy as O  # noqa: E402
from parity import same_bits, GOLDEN  # noqa: E402
from serialize import material_to_dict, surface_to_dict  # noqa: E402
import systems  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("kw", [dict(pt=[0., 1., -2.], dmax=3., n=5, nphis=4, phi_start=0.3, normal=(0, 0, 1)),
                                dict(pt=[0., 0., 0.], dmax=2., n=4, nphis=3, phi_start=0.,
                                     normal=(np.sin(0.2), 0, np.cos(0.2))),
                                dict(pt=[0., 0., 0.], dmax=2., n=3, nphis=2, phi_start=0., normal=(0, 1, 0)),
                                dict(pt=[1., 2., 3.], dmax=25.4, n=1001, nphis=64, phi_start=0.1, normal=(0, 0, 1))])
def test_device_collimated_rays_match_host(kw):
    h = rt.get_collimated_rays(kw["pt"], kw["dmax"], kw["n"], 0.5, nphis=kw["nphis"], phi_start=kw["phi_start"],
                               normal=kw["normal"])
    d = rt.get_collimated_rays(kw["pt"], kw["dmax"], kw["n"], 0.5, nphis=kw["nphis"], phi_start=kw["phi_start"],
                               normal=kw["normal"], device=DEV).cpu().numpy()
    assert d.shape == h.shape
    assert np.array_equal(d, h)                 # bit-identical: host-side constants come from NumPy


def test_device_intersect_rays_bitwise_vs_reference():
    g = np.load(os.path.join(GOLDEN, "generators.npz"))
    got = rt.intersect_rays(torch.from_numpy(g["intersect_in1"]).to(DEV), torch.from_numpy(g["intersect_in2"]).to(DEV))
    assert same_bits(got.cpu().numpy(), g["intersect_out"])
    fan = rt.get_ray_fan([0., 0., 0.], 0.1, 5, 0.5)
    got = rt.intersect_rays(torch.from_numpy(fan[1]).to(DEV), torch.from_numpy(fan).to(DEV))
    assert same_bits(got.cpu().numpy(), g["intersect_fan_out"])


def test_device_auto_focus_style_focus_finding():
    """The reference's focus finder: trace a fan, intersect the traced rays pairwise (RT:832-836)."""
    system, rays, m0, m1 = systems.c1_plano_convex(rt, mat, nrays=101)
    h = system.ray_trace(torch.from_numpy(rays).to(DEV), m0, m1)
    got = rt.intersect_rays(h[-1, 51:], h[-1, 50:51])
    ref = rt.intersect_rays(h[-1, 51:].cpu().numpy(), h[-1, 50:51].cpu().numpy())
    assert same_bits(got.cpu().numpy(), ref)


def test_spot_stats_match_numpy():
    rng = np.random.default_rng(3)
    G, per = 7, 1000
    plane = rng.normal(size=(G * per, 8)) * np.array([1, 2, 3, 1, 1, 1, 1, 1]) + 5.0
    plane[rng.random(G * per) < 0.1] = np.nan
    raw = analysis.spot_stats_raw(torch.from_numpy(plane).to(DEV), per).cpu().numpy()
    p = plane.reshape(G, per, 8)
    ok = np.isfinite(p[..., 0]) & np.isfinite(p[..., 1])
    x, y, z = (np.where(ok, p[..., k], 0.0) for k in range(3))
    ref = np.stack((ok.sum(1), x.sum(1), y.sum(1), z.sum(1), (x * x).sum(1), (y * y).sum(1), (x * y).sum(1)), 1)
    np.testing.assert_allclose(raw, ref, rtol=1e-12)
    again = analysis.spot_stats_raw(torch.from_numpy(plane).to(DEV), per).cpu().numpy()
    assert np.array_equal(raw, again)                          # deterministic reduction


def test_spot_sweep_matches_oracle_c5_small():
    """C5 spot sweep (ODT excitation system) at small size vs the oracle traced on host-built fans."""
    system = systems.c5_system(rt, mat)
    fields = systems.c5_field_points(2)
    wls = [0.405, 0.785]
    theta, nt, nph = 0.5 * np.pi / 180, 21, 7
    summ, timing = analysis.spot_sweep(system, mat.Constant(1), mat.Constant(1), fields, wls, theta, nt, nph,
                                       device=DEV, groups_per_batch=3)
    S = [surface_to_dict(s) for s in system.surfaces]
    M = [material_to_dict(m) for m in [mat.Constant(1)] + list(system.materials) + [mat.Constant(1)]]
    raws = []
    for f in fields:
        for w in wls:
            fin = O.ray_trace(S, M, rt.get_ray_fan(f, theta, nt, w, nphis=nph))[-1]
            ok = np.isfinite(fin[:, 0]) & np.isfinite(fin[:, 1])
            x, y, z = (np.where(ok, fin[:, k], 0.0) for k in range(3))
            raws.append([ok.sum(), x.sum(), y.sum(), z.sum(), (x * x).sum(), (y * y).sum(), (x * y).sum()])
    ref = analysis.summarize(np.array(raws).reshape(len(fields), len(wls), 7))
    assert np.array_equal(summ["count"], ref["count"])
    np.testing.assert_allclose(summ["centroid"], ref["centroid"], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(summ["rms_radius"], ref["rms_radius"], rtol=1e-6, atol=1e-9)
    assert timing["rays"] == len(fields) * len(wls) * nt * nph


@pytest.mark.parametrize("dtype", ["float64", "float32"])
@pytest.mark.parametrize("case", ["c5", "c5_bundles", "c5_backward", "c2", "tir", "tir_last", "stress", "c4", "xz"])
def test_fused_spot_sweep_bitwise_equals_unfused(case, dtype):
    """One-kernel sweep (generate + trace + reduce) == fan kernel + trace(planes='final') + spot stats,
    bit for bit, for a lens system (C5) and a lens-free one (C2), in both storage types; several
    batches, ragged group size (not a multiple of 256).  The sweep runs the surface steps with final-position
    semantics (no per-surface TIR position fill, the final plane's rule applied at the end) and carries
    x x + y y between axial spheres: the TIR prism (total internal reflection mid-path and, in 'tir_last', at
    the final surface), and the stress system (every surface kind, a mirror, misses, aperture and NA kills,
    tabulated and polynomial materials) check those against the full-semantics trace kernel."""
    gpb = 4
    if case == "c5":
        system, m0, m1 = systems.c5_system(rt, mat), mat.Constant(1), mat.Constant(1)
        fields, wls, theta = systems.c5_field_points(2), [0.405, 0.532, 0.785], 0.5 * np.pi / 180
    elif case == "c5_bundles":
        # batches of 13 groups over 2 fields x 9 wavelengths: bundle rows of 8 and 4 groups of one field point and
        # single rows (the odd ones out) -- the first surface's shared state serves up to 8 refractions
        system, m0, m1 = systems.c5_system(rt, mat), mat.Constant(1), mat.Constant(1)
        fields, wls, theta = systems.c5_field_points(2), list(np.linspace(0.4, 0.8, 9)), 0.5 * np.pi / 180
        gpb = 13
    elif case == "c5_backward":
        # field points inside the first sphere's ball (forward roots on its far side, u2 < 0), in the glass between
        # surfaces, and beyond the whole system (both roots of every sphere behind the rays): the sweep's forward-root
        # kill and one-compare discriminant guard against the full-semantics trace
        system, m0, m1 = systems.c5_system(rt, mat), mat.Constant(1), mat.Constant(1)
        fields, wls, theta = [[0.0, 0.0, 195.0], [0.7, -0.4, 250.0], [1.0, 0.5, 2500.0], [0.0, 0.0, 0.0]], \
            [0.405, 0.532, 0.785], 0.6
    elif case == "c2":
        system, m0, m1 = systems.c2_system(rt, mat), mat.Vacuum(), mat.Vacuum()
        fields, wls, theta = [[0.0, 0.0, -5.0], [1.0, -2.0, -5.0]], list(systems.C2_WAVELENGTHS), 0.05
    elif case == "c4":
        # the OPM: axial lenses and flats, then five surfaces in the x-z plane (kPlaneXZ) behind the 30 deg tilt
        system, m0, m1 = systems.c4_system(rt, mat), mat.Constant(systems.OPM_N1), mat.Vacuum()
        fields, wls, theta = [[1e-3, 1e-3, 1e-3 * np.tan(np.pi / 6)], [0.0, 0.0, 0.0]], \
            [systems.OPM_WAVELENGTH, 0.9 * systems.OPM_WAVELENGTH], np.arcsin(1.35 / systems.OPM_N1)
    elif case == "xz":
        # tilted flats and PerfectLens steps in the x-z plane, Constant / Sellmeier / Vacuum media (test_axial.py)
        from test_axial import tilted_xz_system
        system, m0, m1 = tilted_xz_system()
        fields, wls, theta = [[0.0, 0.0, -3.0], [0.4, -0.3, -3.0]], [0.5, 0.6], 0.2
    elif case in ("tir", "tir_last"):
        system, _, m0, m1 = systems.tir_prism(rt, mat)
        if case == "tir_last":
            system = rt.System(system.surfaces[:2], system.materials[:1])
        fields, wls, theta = [[0.0, 0.0, -5.0], [2.0, -1.0, -5.0]], [0.45, 0.55, 0.7], 0.5
    else:
        system, m0, m1 = systems.stress_system(rt, mat), mat.Vacuum(), mat.Vacuum()
        fields, wls, theta = [[0.0, 0.0, -10.0], [3.0, -2.0, -10.0], [-1.5, 2.5, -10.0]], [0.5, 0.6328], 0.3
    args = (system, m0, m1, fields, wls, theta, 301, 77)
    fu, _ = analysis.spot_sweep(*args, device=DEV, dtype=dtype, groups_per_batch=gpb, fused=True)
    un, _ = analysis.spot_sweep(*args, device=DEV, dtype=dtype, groups_per_batch=5, fused=False)
    assert fu.keys() == un.keys()
    for k in fu:
        assert same_bits(fu[k], un[k]), k
    if case != "c5_backward":
        assert fu["count"].min() > 0
    if case not in ("c5", "c5_bundles", "c2", "xz"):
        assert (fu["count"] < 301 * 77).any()            # some rays of the bundle are lost on the way
    if case == "c5_backward":
        assert (fu["count"] == 0).any()                  # the field beyond the system: every row killed


@pytest.mark.parametrize("case", ["astig_relay", "reversed_doublet", "fuzz_01", "fuzz_03", "fuzz_06", "fuzz_13",
                                  "fuzz_23", "fuzz_29", "fuzz_00", "fuzz_08"])
def test_fused_sweep_bitwise_on_golden_systems(case):
    """The bundle rows' shared first surface on every first-surface form: non-axial spheres and flats (the general
    tangent basis), an axial flat, and systems whose first surface is not shared (a PerfectLens, a mirror) -- fused
    == unfused, bit for bit, with 2 fields x 5 wavelengths (bundles of 4 and a single per field point).  Field points
    and the fan axis come from the golden bundle of the system."""
    import json
    from parity import load_case
    from serialize import system_from_json
    spec, rays, _ = load_case(case)
    system, m0, m1 = system_from_json(rt, mat, json.dumps(spec))
    fin = rays[np.isfinite(rays).all(axis=1)]
    p0 = fin[:, :3].mean(axis=0)
    d = fin[:, 3:6].mean(axis=0)
    d = d / np.linalg.norm(d)
    axis = tuple(d) if np.linalg.norm(d) == 1 else (0.0, 0.0, 1.0)
    fields = np.stack((p0, p0 + 0.05 * np.cross(axis, (0.3, 0.5, 0.81)) / np.linalg.norm(np.cross(axis, (0.3, 0.5, 0.81)))))
    wls = sorted(set(np.round(fin[:, 7], 6).tolist()))[:1] or [0.55]
    wls = [wls[0] * f for f in (0.8, 0.9, 1.0, 1.1, 1.2)]
    args = (system, m0, m1, fields, wls, 0.02, 67, 23)
    fu, _ = analysis.spot_sweep(*args, center_ray=axis, device=DEV)
    un, _ = analysis.spot_sweep(*args, center_ray=axis, device=DEV, groups_per_batch=3, fused=False)
    for k in fu:
        assert same_bits(fu[k], un[k]), k
    if case not in ("fuzz_08", "fuzz_23", "fuzz_29"):      # (these three bundles miss their systems)
        assert fu["count"].sum() > 0


def test_dist_pt2plane_bitwise_vs_reference():
    g = np.load(os.path.join(GOLDEN, "generators.npz"))
    dist, near = rt.dist_pt2plane(g["intersect_in1"][:, :3], np.array([0., 0.6, 0.8]), np.array([1., 2., 3.]))
    assert same_bits(dist, g["dist_out"])
    assert same_bits(near, g["dist_near"])


@pytest.mark.parametrize("exclude", [False, True])
def test_propagate_ray2plane_device_bitwise_vs_oracle(exclude):
    """Per-ray planes (the PerfectLens front-focal-plane case, RT:1693) and broadcast planes; a user
    Material subclass goes through the wavelength table."""
    rays = systems.stress_rays(3000, seed=11)
    rng = np.random.default_rng(2)
    nrm = rng.normal(size=(3000, 3))
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    ctr = rng.normal(size=(3000, 3)) * 5
    Cauchy = systems.cauchy_class(mat)
    for m, md in ((mat.Bk7(), material_to_dict(mat.Bk7())), (mat.Constant(1.4), {"type": "Constant", "n": 1.4}),
                  (Cauchy(), {"type": "Cauchy", "a": 1.5046, "b": 0.0042})):
        for nv, cv in ((nrm, ctr), (np.array([0., 0.6, 0.8]), np.array([1., 2., 3.]))):
            got, ts = rt.propagate_ray2plane(rays, nv, cv, m, exclude_backward_propagation=exclude)
            R = O.Rays.from_array(rays)
            nn = tuple(nv[:, k] for k in range(3)) if nv.ndim == 2 else tuple(nv)
            cc = tuple(cv[:, k] for k in range(3)) if cv.ndim == 2 else tuple(cv)
            ref, tref = O.to_plane(R, nn, cc, O.refractive_index(md, R.wl), exclude)
            assert same_bits(got, ref.to_array())
            assert same_bits(ts, tref)
    t_out, t_ts = rt.propagate_ray2plane(torch.from_numpy(rays).to(DEV), nrm, ctr, mat.Bk7())
    assert t_out.is_cuda and t_ts.is_cuda


@pytest.mark.parametrize("layout", ["scattered", "polar_fan"])
def test_gpu_griddata_matches_scipy(layout):
    """GridInterpolator == scipy.interpolate.griddata(method='linear'): same NaN (outside-hull) mask,
    bit-identical values except where a grid point sits on a shared triangle edge (within scipy's eps),
    which may differ by a rounding."""
    from scipy.interpolate import griddata
    rng = np.random.default_rng(3)
    if layout == "scattered":
        pts = rng.uniform(-2, 2, (2000, 2))
    else:                                   # a ray fan seen in a pupil: rings x spokes, incl. y = 0 spokes
        th, ph = np.meshgrid(np.linspace(-1, 1, 61), np.arange(37) * 2 * np.pi / 37)
        r = 2.0 * np.sin(1.1 * th) / np.sin(1.1)
        pts = np.stack((r * np.cos(ph), r * np.sin(ph)), axis=-1).reshape(-1, 2)
    vals = 1e4 + 3.0 * pts[:, 0] ** 2 - 2.0 * pts[:, 1] + rng.normal(scale=1e-3, size=len(pts))
    xs = 0.013 * np.arange(401)
    xs -= xs.mean()
    ys = xs[::2].copy()
    got = analysis.griddata_linear(pts, vals, xs, ys, device=DEV).cpu().numpy()
    xx, yy = np.meshgrid(xs, ys)
    ref = griddata(pts, vals, np.stack((xx.ravel(), yy.ravel()), 1)).reshape(xx.shape)
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    fin = ~np.isnan(ref)
    assert fin.sum() > 10000
    assert (got[fin] == ref[fin]).mean() > 0.99
    assert np.max(np.abs(got[fin] - ref[fin])) <= 1e-12 * np.max(np.abs(ref[fin]))


@pytest.mark.parametrize("interp", ["gpu", "host"])
def test_pupil_psf_matches_host_pipeline(interp):
    """§8f #4: GPU trace + griddata + GPU FFT vs the reference script's NumPy pipeline on the oracle."""
    from numpy import fft
    from scipy.interpolate import griddata
    wavelength, n1, na, mag, ftl = 532e-6, 1.4, 1.35, 100, 200
    alpha = np.arcsin(na / n1)
    f1 = ftl / mag
    r1 = na * f1
    system = rt.System([rt.PerfectLens(f1, [0, 0, n1 * f1], [0, 0, 1], alpha),
                        rt.FlatSurface([0, 0, n1 * f1 + f1], [0, 0, 1], 4 * r1),
                        rt.PerfectLens(ftl, [0, 0, n1 * f1 + f1 + ftl], [0, 0, 1], na / mag),
                        rt.FlatSurface([0, 0, n1 * f1 + f1 + 2 * ftl], [0, 0, 1], r1)],
                       [mat.Vacuum(), mat.Vacuum(), mat.Vacuum()])
    srcs = [[0, 0, -1e-4], [0, 0, 0], [0, 0, 1e-4]]
    psf, pupil, xs = analysis.pupil_psf(system, mat.Constant(n1), mat.Vacuum(), srcs, wavelength, alpha, 41, 21,
                                        pupil_plane=4, pupil_radius=r1, grid_step=0.05, device=DEV, interp=interp)
    S = [surface_to_dict(s) for s in system.surfaces]
    M = [material_to_dict(m) for m in [mat.Constant(n1)] + list(system.materials) + [mat.Vacuum()]]
    xx, yy = np.meshgrid(xs, xs)
    ref = []
    for p in srcs:
        h = O.ray_trace(S, M, rt.get_ray_fan(p, alpha, 41, wavelength, nphis=21))[4]
        ok = ~np.isnan(h[:, 0]) & ~np.isnan(h[:, 1])
        ph = griddata(h[ok, :2], h[ok, 6], np.stack((xx.ravel(), yy.ravel()), 1)).reshape(xx.shape)
        e = np.exp(1j * ph)
        e[np.sqrt(xx ** 2 + yy ** 2) > r1] = 0
        e[np.isnan(ph)] = 0
        ref.append(np.abs(fft.fftshift(fft.fft2(fft.ifftshift(e)))) ** 2)
    ref = np.array(ref)
    ref /= ref.max()
    np.testing.assert_allclose(psf, ref, rtol=0, atol=1e-9)
    assert psf.shape == (3, len(xs), len(xs)) and abs(psf.max() - 1) < 1e-15


def test_spot_sweep_over_devices_is_bitwise_equal():
    """In-process multi-GPU sweep (groups split in contiguous ranges per device, launched round-robin):
    statistics bit-identical to one device; per-device kernel times reported (here: shards on GPU 0,
    plus every visible GPU when there are several)."""
    import torch
    system = systems.c5_system(rt, mat)
    fields = systems.c5_field_points(3)
    wls = [0.405, 0.532, 0.785]
    theta, nt, nph = 0.5 * np.pi / 180, 101, 37
    one, t1 = analysis.spot_sweep(system, mat.Constant(1), mat.Constant(1), fields, wls, theta, nt, nph, device=DEV,
                                  groups_per_batch=4)
    lists = [[0, 0, 0]] + ([list(range(torch.cuda.device_count()))] if torch.cuda.device_count() > 1 else [])
    for devs in lists:
        many, tm = analysis.spot_sweep(system, mat.Constant(1), mat.Constant(1), fields, wls, theta, nt, nph,
                                       devices=devs, groups_per_batch=4)
        for k in ("count", "centroid", "rms_radius"):
            assert same_bits(many[k], one[k]), (devs, k)
        assert [p["device"] for p in tm["per_device"]] == devs
        assert sum(p["rays"] for p in tm["per_device"]) == t1["rays"]
        assert all(p["kernel_ms"] > 0 for p in tm["per_device"])


def test_spot_sweep_group_order_does_not_matter():
    """rtpb_spot_sweep gathers the groups of one field point into bundle rows whatever their order: fields and
    wavelengths given in another order (groups interleaved differently in one batch) give the same statistics,
    bit for bit, in the new order."""
    system = systems.c5_system(rt, mat)
    fields = systems.c5_field_points(2)
    wls = [0.405, 0.465, 0.532, 0.561, 0.785]
    theta, nt, nph = 0.5 * np.pi / 180, 61, 29
    ref, _ = analysis.spot_sweep(system, mat.Constant(1), mat.Constant(1), fields, wls, theta, nt, nph, device=DEV)
    fo, wo = [2, 0, 3, 1], [3, 1, 4, 0, 2]
    got, _ = analysis.spot_sweep(system, mat.Constant(1), mat.Constant(1), fields[fo], [wls[k] for k in wo], theta,
                                 nt, nph, device=DEV, groups_per_batch=7)      # batches of 7 mix field points
    for k in ("count", "centroid", "rms_radius"):
        assert same_bits(got[k], ref[k][fo][:, wo]), k


def fixed_order_sums(plane, group_size, tile=256):
    """The spot kernels' reduction restated in NumPy, operation for operation (csrc/rtpb_analysis.hip
    spot_partial_kernel / sweep_kernel + spot_final_kernel): per 256-ray tile a pairwise tree
    (red[t] += red[t + w], w = 128 ... 1) of (1, x, y, z, x*x, y*y, x*y) over rays with finite x and y;
    per group, thread t adds tiles t, t + 256, ... in order, then the same tree over the 256 threads."""
    p = np.asarray(plane, dtype=np.float64).reshape(-1, group_size, plane.shape[-1])
    G = p.shape[0]
    tiles = -(-group_size // tile)
    x, y, z = p[..., 0], p[..., 1], p[..., 2]
    with np.errstate(invalid="ignore"):
        ok = (x - x == 0.0) & (y - y == 0.0)
    v = np.zeros((G, tiles * tile, 7))
    with np.errstate(invalid="ignore", over="ignore"):
        terms = np.stack((np.ones_like(x), x, y, z, x * x, y * y, x * y), -1)
    v[:, :group_size] = np.where(ok[..., None], terms, 0.0)
    v = v.reshape(G, tiles, tile, 7)
    w = tile // 2
    while w:
        v[:, :, :w] = v[:, :, :w] + v[:, :, w:2 * w]
        w //= 2
    part = v[:, :, 0]                                            # (G, tiles, 7)
    acc = np.zeros((G, tile, 7))
    for c in range(0, tiles, tile):
        blk = part[:, c:c + tile]
        acc[:, :blk.shape[1]] = acc[:, :blk.shape[1]] + blk
    w = tile // 2
    while w:
        acc[:, :w] = acc[:, :w] + acc[:, w:2 * w]
        w //= 2
    return acc[:, 0]


def test_spot_stats_bitwise_vs_fixed_order_oracle():
    """rtpb_spot_stats: every raw sum bit-identical to the NumPy restatement of its reduction order, with
    ragged groups and more than 256 tiles per group (the second stage's sequential chains)."""
    rng = np.random.default_rng(8)
    G, per = 3, 256 * 300 + 77
    plane = rng.normal(size=(G * per, 8)) * np.array([1, 2, 3, 1, 1, 1, 1, 1]) + 5.0
    plane[rng.random(G * per) < 0.1, 0] = np.nan
    plane[rng.random(G * per) < 0.01, 1] = np.inf
    raw = analysis.spot_stats_raw(torch.from_numpy(plane).to(DEV), per).cpu().numpy()
    assert np.array_equal(raw, fixed_order_sums(plane, per))


@pytest.mark.parametrize("dtype", ["float64", "float32"])
def test_spot_sweep_sums_bitwise_vs_oracle(dtype):
    """The fused C5 sweep (BASELINE configs[4] system: fan generation + trace + reduction in one kernel)
    against the oracle: each group's fan from the reference generator, traced by the NumPy oracle, final
    plane (rounded to the storage type) reduced in the kernel's order -- count and every sum bit for bit,
    hence identical centroids and RMS radii.  Groups of 301 x 300 rays: 353 tiles, a ragged last tile."""
    system = systems.c5_system(rt, mat)
    fields = systems.c5_field_points(2)[1:3]
    wls = [0.405, 0.635]
    theta, nt, nph = 0.5 * np.pi / 180, 301, 300
    summ, _ = analysis.spot_sweep(system, mat.Constant(1), mat.Constant(1), fields, wls, theta, nt, nph,
                                  device=DEV, dtype=dtype)
    S = [surface_to_dict(s) for s in system.surfaces]
    M = [material_to_dict(m) for m in [mat.Constant(1)] + list(system.materials) + [mat.Constant(1)]]
    finals = []
    for f in fields:
        for w in wls:
            rays = rt.get_ray_fan(f, theta, nt, w, nphis=nph)
            if dtype == "float32":
                rays = rays.astype(np.float32).astype(np.float64)
            fin = O.ray_trace(S, M, rays)[-1]
            finals.append(fin.astype(np.float32).astype(np.float64) if dtype == "float32" else fin)
    ref = fixed_order_sums(np.concatenate(finals), nt * nph).reshape(len(fields), len(wls), 7)
    assert np.array_equal(summ["raw"], ref)
    assert summ["count"].min() > 0
    exp = analysis.summarize(ref)
    for k in ("count", "centroid", "rms_radius"):
        assert same_bits(summ[k], exp[k]), k
