"""Optical-system recipes shared by the golden-vector generator and the tests.

Every recipe takes the ray-tracer module ``rt`` and the materials module ``mat`` as arguments, so the
SAME code builds a system either with the reference package (``raytrace.raytrace`` /
``raytrace.materials`` imported from /root/reference/src, only inside ``make_golden.py``'s subprocess)
or with this repository's drop-in (``ray_trace_pb_amd.raytrace`` / ``ray_trace_pb_amd.materials``).

The systems restate the reference's example scripts (the benchmark configurations C1-C5 of
SURVEY.md §8d) plus edge-case systems written for this repository:

* C1  plano-convex singlet      -- scripts/2022_10_27_plano_convex_lens.py:25-31
* C2  AC508-100-B achromat      -- scripts/2022_08_04_ACT508-100-B.py:62-72,90-96,121-139
* C3  4f relay of two AC508-075 -- scripts/2024_08_08_achromat_imaging.py:13-70,97-106
* C4  ideal OPM (PerfectLens)   -- scripts/2022_01_25_ray_trace_ideal_opm.py:9-92
* C4m plane-mirror system       -- scripts/2021_07_25_mirror.py:9-18
* C5  ODT excitation path       -- scripts/2021_10_06_ray_trace_system.py:9-145
* KAT perfect-lens phase        -- scripts/2021_10_28_test_perfect_lens_phase.py:12-38
* off-axis relay (astigmatism)  -- scripts/2022_08_24_relay_astigmatism.py:9-86
* lightsheet with ETL           -- scripts/2024_04_01_lightsheet.py:23-133

Ray bundles are built with ``rt.get_ray_fan`` / ``rt.get_collimated_rays`` (reference RT:45-161) or
with plain NumPy (seeded with ``numpy.random.default_rng``), never with anything module-specific.
"""
import numpy as np

SEED = 20241008
C2_WAVELENGTHS = (0.7065, 0.855, 1.015)
C5_WAVELENGTHS = (0.405, 0.465, 0.488, 0.532, 0.561, 0.635, 0.785)


def unit(v):
    v = np.asarray(v, dtype=float)
    return v / np.linalg.norm(v)


# ------------------------------------------------------------------ C1
def c1_plano_convex(rt, mat, nrays=1001):
    """scripts/2022_10_27_plano_convex_lens.py:15-31 (1 sphere between 2 flats, n=1.3)."""
    aperture_radius = 25.4
    t0 = 2.679486355
    t1 = 1
    rad_curv = 100
    n = 1.3
    dz = 5
    singlet = rt.System([rt.FlatSurface([0, 0, 0], [0, 0, 1], aperture_radius),
                         rt.SphericalSurface.get_on_axis(-rad_curv, t0 + t1, aperture_radius),
                         rt.FlatSurface([0, 0, t0 + t1], [0, 0, 1], aperture_radius)],
                        [mat.Constant(n), mat.Vacuum()])
    rays = rt.get_collimated_rays([0, 0, -dz], aperture_radius, nrays, 0.5)
    return singlet, rays, mat.Vacuum(), mat.Vacuum()


# ------------------------------------------------------------------ C2
def c2_system(rt, mat):
    """AC508-100-B after a flat at z=0, plus a flat at the paraxial focus for 0.855 um."""
    radius = 25.4
    doublet = rt.Doublet(mat.Nlak22(), mat.Nsf6ht(),
                         radius_crown=65.8, radius_flint=-280.6, radius_interface=-56,
                         thickness_crown=13.0, thickness_flint=2.0,
                         aperture_radius=radius, input_collimated=True, names="AC508-100-B")
    system = rt.System([rt.FlatSurface([0, 0, 0], [0, 0, 1], radius)], [])
    system = system.concatenate(doublet, mat.Vacuum(), distance=10)
    _, f2, _, _, _, _, _, _ = system.get_cardinal_points(0.855, mat.Vacuum(), mat.Vacuum())
    system = system.concatenate(rt.System([rt.FlatSurface(f2, [0, 0, 1], radius)], []),
                                mat.Vacuum(), distance=None)
    return system


def c2_rays(nrays, seed=SEED, disk_radius=10.0, z0=-5.0):
    """Collimated rays, positions uniform in a disk, wavelength = C2_WAVELENGTHS[i % 3]."""
    rng = np.random.default_rng(seed)
    r = disk_radius * np.sqrt(rng.random(nrays))
    phi = 2 * np.pi * rng.random(nrays)
    rays = np.zeros((nrays, 8))
    rays[:, 0] = r * np.cos(phi)
    rays[:, 1] = r * np.sin(phi)
    rays[:, 2] = z0
    rays[:, 5] = 1.0
    rays[:, 7] = np.asarray(C2_WAVELENGTHS)[np.arange(nrays) % 3]
    return rays


def c2_achromat(rt, mat, nrays=900):
    return c2_system(rt, mat), c2_rays(nrays), mat.Vacuum(), mat.Vacuum()


# ------------------------------------------------------------------ C3
def c3_system(rt, mat, wlen=0.635):
    """Two AC508-075 doublets in a 4f relay with object, pupil and image flats (9 surfaces)."""
    def ac508_075(collimated):
        return rt.Doublet(mat.Ebaf11(), mat.Nsf11(), radius_crown=50.8, radius_flint=-247.7,
                          radius_interface=-41.7, thickness_crown=20., thickness_flint=3.,
                          aperture_radius=25.4, input_collimated=collimated, names="AC508-075-A-ML")
    l1 = ac508_075(False)
    l2 = ac508_075(True)
    cp1 = l1.get_cardinal_points(wlen, mat.Vacuum(), mat.Vacuum())
    f1_left = cp1[0][-1]
    f1_right = cp1[1][-1]
    wd_right = f1_right - l1.surfaces[-1].paraxial_center[-1]
    system = rt.System([rt.FlatSurface([0, 0, 0], [0, 0, 1], 25.4)], [])
    system = system.concatenate(l1, mat.Vacuum(), -f1_left)
    d = l2.find_paraxial_collimated_distance(l2, wlen, mat.Vacuum(), mat.Vacuum(), mat.Vacuum())
    system = system.concatenate(rt.FlatSurface([0, 0, 0], [0, 0, 1], 25.4), mat.Vacuum(), wd_right)
    ind_pupil = len(system.surfaces) - 1
    system = system.concatenate(l2, mat.Vacuum(), d - wd_right)
    c2 = l2.get_cardinal_points(wlen, mat.Vacuum(), mat.Vacuum())
    wd2 = c2[1][2] - l2.surfaces[-1].paraxial_center[2]
    system = system.concatenate(rt.FlatSurface([0, 0, 0], [0, 0, 1], 25.4), mat.Vacuum(), wd2)
    system.set_aperture_stop(ind_pupil)
    return system


C3_FIELDS = (0., 4., 8., 12., 16.)


def c3_rays(rt, n_thetas, nphis, wlen=0.635, fields=C3_FIELDS):
    return np.concatenate([rt.get_ray_fan(np.array([h, 0, 0]), 1 * np.pi / 180, n_thetas, wlen, nphis=nphis)
                           for h in fields], axis=0)


def c3_relay(rt, mat, n_thetas=11, nphis=8):
    return c3_system(rt, mat), c3_rays(rt, n_thetas, nphis), mat.Vacuum(), mat.Vacuum()


# ------------------------------------------------------------------ C4
OPM_WAVELENGTH = 532e-6
OPM_N1 = 1.4


def c4_system(rt, mat):
    """scripts/2022_01_25_ray_trace_ideal_opm.py:9-80 (6 PerfectLens + 5 flats, one 30-deg tilt)."""
    n1, na1 = OPM_N1, 1.35
    alpha1 = np.arcsin(na1 / n1)
    f1 = 200 / 100
    n2, na2 = 1, 0.95
    alpha2 = np.arcsin(na2 / n2)
    f2 = 200 / 40
    r2 = na2 * f2
    theta = 30 * np.pi / 180
    n3, na3 = 1.51, 1
    alpha3 = np.arcsin(na3 / n3)
    f3 = 200 / 100
    o3_normal = np.array([-np.sin(theta), 0, np.cos(theta)])
    f_tube_lens_1 = 200
    f_tube_lens_2 = f_tube_lens_1 / f1 * f2 / n1
    f_tube_lens_3 = 200
    aperture_rad = 2
    p_o1 = n1 * f1
    p_pupil_o1 = p_o1 + f1
    p_t1 = p_o1 + f1 + f_tube_lens_1
    p_t2 = p_t1 + f_tube_lens_1 + f_tube_lens_2
    p_pupil_o2 = p_t2 + f_tube_lens_2
    p_o2 = p_t2 + f_tube_lens_2 + f2
    p_remote_focus = p_o2 + n2 * f2
    p_o3 = np.array([0, 0, p_remote_focus]) + n3 * f3 * o3_normal
    p_pupil_o3 = p_o3 + f3 * o3_normal
    p_t3 = p_o3 + (f3 + f_tube_lens_3) * o3_normal
    p_imag = p_t3 + f_tube_lens_3 * o3_normal
    return rt.System([rt.PerfectLens(f1, [0, 0, p_o1], [0, 0, 1], alpha1),
                      rt.FlatSurface([0, 0, p_pupil_o1], [0, 0, 1], n1 * f1),
                      rt.PerfectLens(f_tube_lens_1, [0, 0, p_t1], [0, 0, 1], alpha1),
                      rt.PerfectLens(f_tube_lens_2, [0, 0, p_t2], [0, 0, 1], alpha2),
                      rt.FlatSurface([0, 0, p_pupil_o2], [0, 0, 1], n2 * f2),
                      rt.PerfectLens(f2, [0, 0, p_o2], [0, 0, 1], alpha2),
                      rt.FlatSurface([0, 0, p_remote_focus], o3_normal, r2),
                      rt.PerfectLens(f3, p_o3, o3_normal, alpha3),
                      rt.FlatSurface(p_pupil_o3, o3_normal, f3 * n3),
                      rt.PerfectLens(f_tube_lens_3, p_t3, o3_normal, alpha3),
                      rt.FlatSurface(p_imag, o3_normal, aperture_rad)],
                     [mat.Vacuum(), mat.Vacuum(), mat.Vacuum(), mat.Vacuum(), mat.Vacuum(),
                      mat.Constant(n2), mat.Constant(n3), mat.Vacuum(), mat.Vacuum(), mat.Vacuum()])


def c4_rays(rt, n_thetas, nphis):
    theta = 30 * np.pi / 180
    dx = dy = 0.001
    return rt.get_ray_fan([dx, dy, dx * np.tan(theta)], np.arcsin(1.35 / OPM_N1), n_thetas,
                          OPM_WAVELENGTH, nphis=nphis)


def c4_opm(rt, mat, n_thetas=21, nphis=10):
    return c4_system(rt, mat), c4_rays(rt, n_thetas, nphis), mat.Constant(OPM_N1), mat.Vacuum()


def c4_mirror(rt, mat):
    """scripts/2021_07_25_mirror.py:9-18 (two plane mirrors + a flat)."""
    rays = rt.get_ray_fan([0, 0, 0], 5 * np.pi / 180, 25, 0.785, nphis=4)
    theta = np.pi / 4 - np.pi / 30
    system = rt.System([rt.PlaneMirror([0, 0, 30], [-np.sin(theta), 0, -np.cos(theta)], 25),
                        rt.PlaneMirror([-50, 0, 30], [1 / np.sqrt(2), 0, 1 / np.sqrt(2)], 25),
                        rt.FlatSurface([-50, 0, 60], [0, 0, 1], 25)],
                       [mat.Vacuum(), mat.Vacuum()])
    return system, rays, mat.Vacuum(), mat.Vacuum()


# ------------------------------------------------------------------ C5
def c5_system(rt, mat):
    """scripts/2021_10_06_ray_trace_system.py:9-145, excitation path only (14 surfaces)."""
    radius = 25
    t200c, t200f, r200f, r200i, r200c, bfl200 = 10.6, 6, 409.4, 92.1, -106.2, 190.6
    t100c, t100f, r100f, r100i, r100c, bfl100 = 16, 4, 363.1, 44.2, -71.1, 89
    t400c, t400f, r400f, r400i, r400c, bfl400 = 8, 8, 398.5, 148.9, -292.3, 396.1
    t300c, t300f, r300f, r300i, r300c, bfl300 = 6.0, 2.0, 580.8, 134, -161.5, 295.4
    d_dmd_lens = bfl200
    d_400_300 = bfl400 + bfl300 + 5
    d_300_obj = 300 + 1.8
    d_100_200 = 200 + bfl100
    d_100_400 = 100 + 400 - 6
    l1s = d_dmd_lens
    l1e = l1s + t200c + t200f
    l2s = l1e + d_100_200
    l2e = l2s + t100c + t100f
    l3s = l2e + d_100_400
    l3e = l3s + t400c + t400f
    l4s = l3e + d_400_300
    l4e = l4s + t300c + t300f
    l5s = l4e + d_300_obj
    focal_plane = l5s + 1.5 * 1.8
    on_axis = rt.SphericalSurface.get_on_axis
    return rt.System([on_axis(r200f, l1s, radius),
                      on_axis(r200i, l1s + t200f, radius),
                      on_axis(r200c, l1s + t200c + t200f, radius),
                      on_axis(r100f, l2s, radius),
                      on_axis(r100i, l2s + t100f, radius),
                      on_axis(r100c, l2s + t100c + t100f, radius),
                      on_axis(-r400c, l3s, radius),
                      on_axis(-r400i, l3s + t400c, radius),
                      on_axis(-r400f, l3s + t400c + t400f, radius),
                      on_axis(r300f, l4s, radius),
                      on_axis(r300i, l4s + t300f, radius),
                      on_axis(r300c, l4s + t300c + t300f, radius),
                      rt.PerfectLens(1.8, [0, 0, l5s], [0, 0, 1], 1.8 * 1.3),
                      rt.FlatSurface([0, 0, focal_plane], [0, 0, 1], 0.130)],
                     [mat.Sf2(), mat.Bk7(), mat.Constant(1),
                      mat.Sf10(), mat.Nbaf10(), mat.Constant(1),
                      mat.Bk7(), mat.Sf2(), mat.Constant(1),
                      mat.Sf2(), mat.Bk7(), mat.Constant(1),
                      mat.Constant(1.5)])


def c5_field_points(n_side=8):
    sep = 4 * 0.55 * (1.8 / 4 * 400 / 300 * 200 / 100)
    xs = np.linspace(-sep, sep, n_side)
    gx, gy = np.meshgrid(xs, xs)
    return np.stack((gx.ravel(), gy.ravel(), np.zeros(gx.size)), axis=1)


def c5_rays(rt, n_side, n_thetas, nphis, wavelengths=C5_WAVELENGTHS):
    max_angle = 0.5 * np.pi / 180
    return np.concatenate([rt.get_ray_fan(p, max_angle, n_thetas, wl, nphis=nphis)
                           for p in c5_field_points(n_side) for wl in wavelengths], axis=0)


def c5_odt(rt, mat, n_side=2, n_thetas=5, nphis=3):
    return c5_system(rt, mat), c5_rays(rt, n_side, n_thetas, nphis), mat.Constant(1), mat.Constant(1)


# ------------------------------------------------------------------ known-answer: perfect lens phase
def kat_perfect_lens_phase(rt, mat):
    """scripts/2021_10_28_test_perfect_lens_phase.py:12-38: a tilted plane wave focuses in phase."""
    wavelength, aperture, n1, n2, f, na = 0.785, 10, 1.1, 1.3, 4, 1
    alpha = np.arcsin(na / n1)
    system = rt.System([rt.FlatSurface([0, 0, 0], [0, 0, 1], aperture),
                        rt.PerfectLens(f, [0, 0, n1 * f], [0, 0, 1], alpha),
                        rt.FlatSurface([0, 0, n1 * f + n2 * f], [0, 0, 1], aperture)],
                       [mat.Constant(n1), mat.Constant(n2)])
    angle = 10 * np.pi / 180
    rays = rt.get_collimated_rays([0, 0, -1], 3, 7, wavelength, normal=[np.sin(angle), 0, np.cos(angle)])
    return system, rays, mat.Constant(n1), mat.Constant(n2)


# ------------------------------------------------------------------ edge cases (this repository)
def cauchy_class(mat):
    """A user Material subclass overriding ``n`` -- the reference's documented plugin point
    (materials.py:39-44).  The drop-in lowers it through a per-wavelength table."""
    class Cauchy(mat.Material):
        def __init__(self, a=1.5046, b=0.00420):
            self.a = a
            self.b = b

        def n(self, wavelength):
            return self.a + self.b / np.asarray(wavelength) ** 2
    return Cauchy


def stress_system(rt, mat):
    """Every surface kind, tilted/off-axis geometry, a back-reflecting mirror, huge radius (R=1e6
    tolerance quirk), Sellmeier / Constant / Vacuum / Ebaf11-polynomial / user-subclass materials."""
    Cauchy = cauchy_class(mat)
    surfaces = [rt.FlatSurface([0, 0, 0], [0, 0, 1], 20),
                rt.SphericalSurface.get_on_axis(30, 5, 15),
                rt.SphericalSurface.get_on_axis(-25, 12, 15),
                rt.FlatSurface([0, 0, 20], unit([0.1, 0, 1]), 25),
                rt.SphericalSurface(-50, [2, 1, 80], 20, input_axis=unit([0.05, 0, 1])),
                rt.SphericalSurface.get_on_axis(60, 40, 30),
                rt.PerfectLens(25, [0, 0, 100], [0, 0, 1], 1.1),
                rt.FlatSurface([0, 0, 112], [0, 0, 1], 1e6),
                rt.SphericalSurface.get_on_axis(1e6, 120, 30),
                rt.PlaneMirror([0, 0, 140], unit([0, 0.05, -1]), 50),
                rt.FlatSurface([0, 0, 100], [0, 0, -1], 60)]
    materials = [mat.Bk7(), mat.Vacuum(), mat.Sf10(), mat.Constant(1.33), mat.Ebaf11(),
                 mat.Vacuum(), mat.Vacuum(), Cauchy(), mat.Vacuum(), mat.Vacuum()]
    return rt.System(surfaces, materials)


def stress_rays(nrays, seed=SEED + 1):
    rng = np.random.default_rng(seed)
    rays = np.zeros((nrays, 8))
    rays[:, 0:2] = rng.normal(scale=3.0, size=(nrays, 2))
    rays[:, 2] = -10 + rng.normal(scale=1.0, size=nrays)
    theta = rng.uniform(0, 0.3, nrays)
    phi = rng.uniform(0, 2 * np.pi, nrays)
    d = np.stack((np.sin(theta) * np.cos(phi), np.sin(theta) * np.sin(phi), np.cos(theta)), axis=1)
    back = rng.random(nrays) < 0.05          # back-facing / backward propagating rays
    d[back, 2] *= -1
    rays[:, 3:6] = d
    rays[:, 6] = rng.uniform(0, 10, nrays)
    rays[:, 7] = np.array([0.5, 0.6328, 1.0, 0.405])[rng.integers(0, 4, nrays)]
    # a few hand-placed oddities: on-axis normal incidence, ray parallel to the first flat,
    # ray starting exactly on the first surface, zero direction, NaN wavelength, all-NaN row
    special = np.array([[0, 0, -10, 0, 0, 1, 0, 0.5],
                        [0, 0, -10, 1, 0, 0, 0, 0.5],
                        [1, 1, 0, 0, 0, 1, 0, 0.6328],
                        [0, 0, -10, 0, 0, 0, 0, 0.5],
                        [0, 0, -10, 0, 0, 1, 0, np.nan],
                        [np.nan] * 8,
                        [14.9, 0, -10, 0, 0, 1, 0, 0.5],
                        [0, 0, -10, 0, 0.7071067811865476, 0.7071067811865476, 0, 1.0]])
    rays[:len(special)] = special
    return rays


def stress(rt, mat, nrays=1500):
    return stress_system(rt, mat), stress_rays(nrays), mat.Vacuum(), mat.Vacuum()


def reversed_doublet(rt, mat, nrays=300):
    """Doublet built with input_collimated=False, then System.reverse(): rays enter from +z."""
    d = rt.Doublet(mat.Bk7(), mat.Sf2(), radius_crown=106.2, radius_flint=-409.4, radius_interface=-92.1,
                   thickness_crown=10.6, thickness_flint=6.0, aperture_radius=25.4, input_collimated=False)
    system = rt.System([rt.FlatSurface([0, 0, -5], [0, 0, 1], 25.4)], []).concatenate(d, mat.Vacuum(), 5)
    system = system.reverse()
    rays = rt.get_collimated_rays([0, 0, 40], 20, nrays // 6, 0.6328, nphis=6, phi_start=0.1,
                                  normal=[0, 0, -1])
    return system, rays, mat.Vacuum(), mat.Vacuum()


def tir_prism(rt, mat, nrays=400):
    """Rays entering glass at a flat and leaving through a steeply tilted flat: total internal
    reflection splits the bundle (TIR keeps phase and wavelength, RT:1218-1221)."""
    system = rt.System([rt.FlatSurface([0, 0, 0], [0, 0, 1], 30),
                        rt.FlatSurface([0, 0, 10], unit([0.8, 0, 1]), 40),
                        rt.FlatSurface([0, 0, 40], [0, 0, 1], 100)],
                       [mat.Sf10(), mat.Vacuum()])
    rays = rt.get_ray_fan([0, 0, -5], 0.5, nrays, 0.55)
    return system, rays, mat.Vacuum(), mat.Vacuum()


def astig_relay(rt, mat, nrays=19, offset=5.0):
    """scripts/2022_08_24_relay_astigmatism.py:9-86: three achromats, the first two displaced off axis
    by `offset` (the sphere aperture is measured about the ORIGIN-through axis, RT:1527-1535), traced
    with meridional, sagittal and 100-azimuth collimated bundles at 0.785 um."""
    wl = 0.785
    beam_rad = 20e-3 * np.sqrt(1 + (3 / (np.pi * 20e-3 ** 2 / (wl * 1e-3))) ** 2)
    t100c, r100c, r100i, t100f, r100f, bfl100 = 13.0, 65.8, -56., 2.0, -280.6, 91.5
    t180c, r180c, r180i, t180f, r180f, bfl180 = 9.5, 144.4, -115.4, 4.0, -328.2, 173.52
    t300c, r300c, r300i, t300f, bfl300, efl300 = 9.0, 167.7, -285.8, 4.0, 289.81, 300
    radius = 25.4
    z180 = 10
    z100 = (t180c + t180f) + bfl180 + 101.5
    z300 = z100 + (t100c + t100f) + bfl100 + efl300
    zend = z300 + (t300c + t300f) + bfl300
    surfaces = [rt.SphericalSurface(r180c, [offset, 0, z180 + np.abs(r180c)], radius),
                rt.SphericalSurface(r180i, [offset, 0, z180 + t180c - np.abs(r180i)], radius),
                rt.SphericalSurface(r180f, [offset, 0, z180 + t180c + t180f - np.abs(r180f)], radius),
                rt.SphericalSurface(-r100f, [offset, 0, z100 + np.abs(r100f)], radius),
                rt.SphericalSurface(-r100i, [offset, 0, z100 + t100f + np.abs(r100i)], radius),
                rt.SphericalSurface(-r100c, [offset, 0, z100 + t100f + t100c - np.abs(r100c)], radius),
                rt.SphericalSurface.get_on_axis(r300c, z300, radius),
                rt.SphericalSurface.get_on_axis(r300i, z300 + t300c, radius),
                rt.FlatSurface([0, 0, z300 + t300c + t300f], [0, 0, 1], radius),
                rt.FlatSurface([0, 0, zend], [0, 0, 1], radius)]
    materials = [mat.Nlak22(), mat.Nsf6(), mat.Constant(1), mat.Nsf6ht(), mat.Nlak22(), mat.Constant(1),
                 mat.Nlak22(), mat.Nsf6(), mat.Constant(1)]
    rays = np.concatenate((rt.get_collimated_rays([0, 0, 0], beam_rad, nrays, wl),
                           rt.get_collimated_rays([0, 0, 0], beam_rad, nrays, wl, phi_start=np.pi / 2),
                           rt.get_collimated_rays([0, 0, 0], beam_rad, nrays, wl, nphis=100)), axis=0)
    return rt.System(surfaces, materials), rays, mat.Vacuum(), mat.Vacuum()


def lightsheet(rt, mat, rad_curv, nrays=1001):
    """scripts/2024_04_01_lightsheet.py:23-36,72-133: electrically tunable lens (flat + sphere of
    radius `rad_curv`), two relay PerfectLenses, an objective PerfectLens and coverglass flats, built
    with System.concatenate (17 history planes)."""
    st = {"wavelength": 0.532, "aperture_radius_etl": 8, "aperture_radius": 50.8 / 2, "n_etl": 1.3,
          "t_edge": 5, "f1": 160, "f2": 120, "fobj": 20, "t_coverglass": 1.25, "n_coverglass": 1.4585,
          "dz_coverglass": 10, "n_immersion": 1.333}
    t_center = st["t_edge"] + rad_curv * (1 - np.sqrt(1 - (st["aperture_radius_etl"] / rad_curv) ** 2))
    rays = rt.get_collimated_rays([0, 0, -1], 8, nrays, st["wavelength"])
    etl = rt.System([rt.FlatSurface([0, 0, 0], [0, 0, 1], st["aperture_radius_etl"]),
                     rt.SphericalSurface.get_on_axis(-rad_curv, t_center, st["aperture_radius_etl"])],
                    materials=[mat.Constant(st["n_etl"])], names="etl")
    l1 = rt.System([rt.PerfectLens(st["f1"], [0, 0, 0], [0, 0, 1], alpha=np.arcsin(0.1))], [], names="l1")
    l2 = rt.System([rt.PerfectLens(st["f2"], [0, 0, 0], [0, 0, 1], alpha=np.arcsin(0.1))], [], names="l2")
    obj = rt.System([rt.PerfectLens(st["fobj"], [0, 0, 0], [0, 0, 1], alpha=np.arcsin(0.3))], [], names="obj")
    cglass = rt.System([rt.FlatSurface([0, 0, 0], [0, 0, 1], st["aperture_radius"]),
                        rt.FlatSurface([0, 0, st["t_coverglass"]], [0, 0, 1], st["aperture_radius"]),
                        rt.FlatSurface([0, 0, 30], [0, 0, 1], st["aperture_radius"])],
                       [mat.Constant(st["n_coverglass"]), mat.Constant(st["n_immersion"])], "coverglass")
    osys = etl.concatenate(l1, mat.Vacuum(), st["f1"] - (t_center - st["t_edge"]))
    osys = osys.concatenate(l2, mat.Vacuum(), st["f1"] + st["f2"])
    osys = osys.concatenate(obj, mat.Vacuum(), st["f2"] + st["fobj"])
    osys = osys.concatenate(cglass, mat.Vacuum(), st["dz_coverglass"])
    return osys, rays, mat.Vacuum(), mat.Vacuum()


# ------------------------------------------------------------------ randomised systems (fuzz)
FUZZ_GLASSES = ("Bk7", "Sf10", "Sf2", "Nsf11", "Nbaf10", "FusedSilica", "Nlak22", "Nsf6ht", "Nsk11")
N_FUZZ = 32


def _tilted(rng, axis, p, scale):
    axis = np.asarray(axis, dtype=float)
    if rng.random() >= p:
        return axis
    return unit(axis + np.array([1.0, 1.0, 0.0]) * rng.normal(scale=scale, size=3))


def fuzz(rt, mat, seed, nrays=160):
    """A seeded random system and bundle: 2-9 surfaces drawn from every kind (flats, spheres of either
    sign from R=4 to 2000 plus the occasional R=1e6, perfect lenses, plane mirrors that turn the
    bundle round), tilted and decentred at random, any medium between them (Vacuum, Constant,
    Sellmeier glasses, the Ebaf11 polynomial, a user n()), and a bundle that is a point-source fan,
    a tilted collimated beam or random rays -- with a few non-unit directions and the hand-placed
    oddities of ``stress_rays``.  The golden files hold the reference's answer for each seed."""
    rng = np.random.default_rng(SEED + 1000 + seed)
    Cauchy = cauchy_class(mat)

    def medium():
        u = rng.random()
        if u < 0.35:
            return mat.Vacuum()
        if u < 0.5:
            return mat.Constant(float(np.round(rng.uniform(1.0, 1.9), 4)))
        if u < 0.58:
            return mat.Ebaf11()
        if u < 0.64:
            return Cauchy(a=float(np.round(rng.uniform(1.4, 1.7), 4)), b=float(np.round(rng.uniform(0.002, 0.01), 5)))
        return getattr(mat, FUZZ_GLASSES[rng.integers(len(FUZZ_GLASSES))])()

    S = int(rng.integers(2, 10))
    sgn, z = 1.0, 0.0
    surfaces, materials = [], []
    for k in range(S):
        u = rng.random()
        ap = float(np.round(rng.uniform(3, 30), 3))
        shift = np.array([1.0, 1.0, 0.0]) * rng.normal(scale=1.0, size=3) if rng.random() < 0.3 else np.zeros(3)
        c = np.array([0.0, 0.0, z]) + shift
        if u < 0.3:
            surfaces.append(rt.FlatSurface(c, _tilted(rng, [0, 0, sgn], 0.3, 0.08), ap))
        elif u < 0.72:
            axis = _tilted(rng, [0, 0, sgn], 0.25, 0.05)
            R = float(rng.choice([-1.0, 1.0]) * np.round(np.exp(rng.uniform(np.log(4), np.log(2000))), 3))
            if rng.random() < 0.06:
                R = float(np.sign(R) * 1e6)
            surfaces.append(rt.SphericalSurface(R, c + R * axis, ap, input_axis=axis))
        elif u < 0.9:
            f = float(np.round(rng.uniform(5, 60), 3))
            surfaces.append(rt.PerfectLens(f, c, _tilted(rng, [0, 0, sgn], 0.2, 0.03),
                                           float(np.round(rng.uniform(0.2, 1.3), 3))))
        else:
            surfaces.append(rt.PlaneMirror(c, _tilted(rng, [0, 0, -sgn], 0.5, 0.05), 2 * ap))
            sgn = -sgn
        if k < S - 1:
            materials.append(medium())
        z += sgn * float(np.round(rng.uniform(3, 25), 3))

    mode = int(rng.integers(3))
    wl = float(rng.choice([0.405, 0.488, 0.532, 0.6328, 0.785, 1.0]))
    src = np.array([rng.normal(scale=0.5), rng.normal(scale=0.5), -float(rng.uniform(2, 20))])
    if mode == 0:
        center = np.array([0.0, 0.0, 1.0])
        for _ in range(8):                   # get_ray_fan demands norm(center_ray) == 1 exactly (RT:67-68)
            c = _tilted(rng, [0, 0, 1], 0.7, 0.05)
            if np.linalg.norm(c) == 1:
                center = c
                break
        rays = rt.get_ray_fan(src, float(rng.uniform(0.05, 0.6)), 20, wl, nphis=8, center_ray=tuple(center))
    elif mode == 1:
        rays = rt.get_collimated_rays(src, float(rng.uniform(1, 20)), 20, wl, nphis=8,
                                      normal=_tilted(rng, [0, 0, 1], 0.7, 0.05))
    else:
        rays = stress_rays(nrays, seed=SEED + 2000 + seed)
        rays[8:, 2] += src[2] + 10
    rays = np.array(rays[:nrays], dtype=np.float64)
    if mode != 2:
        rays[:, 6] = rng.uniform(0, 10, rays.shape[0])
        odd = rng.random(rays.shape[0]) < 0.05                  # non-unit directions
        rays[odd, 3:6] *= rng.uniform(0.5, 2.0, (int(odd.sum()), 1))
    return rt.System(surfaces, materials), rays, medium(), medium()


# name -> recipe; every recipe returns (system, rays, initial_material, final_material)
RECIPES = {
    "c1_plano_convex": c1_plano_convex,
    "c2_achromat": c2_achromat,
    "c3_relay": c3_relay,
    "c4_opm": c4_opm,
    "c4_mirror": c4_mirror,
    "c5_odt": c5_odt,
    "kat_perfect_lens_phase": kat_perfect_lens_phase,
    "stress": stress,
    "reversed_doublet": reversed_doublet,
    "tir_prism": tir_prism,
    "astig_relay": astig_relay,
    # the lightsheet script's first ETL radius (a hemisphere: sphere edge exactly at the aperture) and
    # its last (1e9 mm, where the absolute 1e-12 on-sphere tolerance rejects rays, SURVEY §7 hard part 2)
    "lightsheet_r8": lambda rt, mat: lightsheet(rt, mat, 8.0),
    "lightsheet_r120": lambda rt, mat: lightsheet(rt, mat, 120.0),
    "lightsheet_r1e9": lambda rt, mat: lightsheet(rt, mat, 1e9),
}
RECIPES.update({"fuzz_%02d" % k: (lambda rt, mat, k=k: fuzz(rt, mat, k)) for k in range(N_FUZZ)})

# recipes also recorded with their input rays rounded to float32 (<name>_f32in.npz): the reference's
# answer for float32 input, which the float32-input paths must reproduce
F32_INPUT_CASES = ("c2_achromat", "c3_relay", "c4_opm", "c5_odt", "stress", "fuzz_00", "fuzz_06", "fuzz_11",
                   "fuzz_14")


# ------------------------------------------------------------------ long systems (> RTPB_MAX_SURFACES)
def long_system(rt, mat, n_lenses=49):
    """A train of weak Bk7 / N-SF11 biconvex lenses (2 spheres each) with a pupil flat after every tenth
    lens, a PerfectLens in the middle and a final image flat: 2 * n_lenses + n_lenses // 10 + 2 surfaces
    (49 lenses: 104 surfaces, 209 history planes) -- beyond one fused launch's 63 surfaces."""
    surfaces, materials = [], []
    z = 0.0
    for k in range(n_lenses):
        glass = mat.Bk7() if k % 2 == 0 else mat.Nsf11()
        surfaces.append(rt.SphericalSurface.get_on_axis(400.0, z, 12.0))
        surfaces.append(rt.SphericalSurface.get_on_axis(-400.0, z + 2.0, 12.0))
        materials += [glass, mat.Vacuum()]
        z += 6.0
        if k % 10 == 9:
            surfaces.append(rt.FlatSurface([0, 0, z - 2.0], [0, 0, 1], 4.0))
            materials.append(mat.Vacuum())
        if k == n_lenses // 2:
            surfaces.append(rt.PerfectLens(50.0, [0, 0, z - 1.0], [0, 0, 1], 0.6))
            materials.append(mat.Vacuum())
    surfaces.append(rt.FlatSurface([0, 0, z + 5.0], [0, 0, 1], 30.0))
    return rt.System(surfaces, materials)


def long_rays(nrays=2000, seed=SEED + 3):
    """Collimated rays in a 6 mm disk at three wavelengths, a few tilted."""
    rng = np.random.default_rng(seed)
    r = 6.0 * np.sqrt(rng.uniform(0, 1, nrays))
    a = rng.uniform(0, 2 * np.pi, nrays)
    rays = np.zeros((nrays, 8))
    rays[:, 0], rays[:, 1], rays[:, 2] = r * np.cos(a), r * np.sin(a), -5.0
    d = np.stack((rng.normal(scale=0.01, size=nrays), rng.normal(scale=0.01, size=nrays), np.ones(nrays)), axis=1)
    rays[:, 3:6] = d / np.linalg.norm(d, axis=1)[:, None]
    rays[:, 7] = np.array([0.486, 0.5876, 0.6563])[np.arange(nrays) % 3]
    return rays
