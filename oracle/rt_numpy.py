"""NumPy ORACLE for the sequential ray trace -- TEST INFRASTRUCTURE ONLY.

This module restates the reference's ``System.ray_trace`` hot path (QI2lab/ray_trace_pb @ 2024_10_08,
src/raytrace/raytrace.py = "RT", src/raytrace/materials.py = "MAT") as plain NumPy over per-column
arrays.  It is the CHECKER used by ``tests/``, by ``__graft_entry__.smoke()`` and, as the CPU
baseline leg (kind "port"), by ``bench.py``.  The product path (``ray_trace_pb_amd``) never imports it.

Pinning: golden vectors produced by the reference itself (tests/golden/make_golden.py, run in this
container with /root/reference/src on the path) pin this restatement; tests/test_oracle_golden.py
requires it to reproduce every committed history BIT FOR BIT (NaN pattern included).

Arithmetic is written in exactly the order NumPy evaluates the reference expressions (left-to-right
products, ``np.linalg.norm`` = sqrt(((a*a + b*b) + c*c)), ``np.cross`` = a1*b2 - a2*b1 ...), so the
IEEE results agree with the reference to the last bit.

Input format: surfaces and materials as the JSON-able dicts of tests/golden/serialize.py.
"""
import numpy as np

TWO_PI = 2 * np.pi          # Python float, as in ``2 * np.pi`` of RT:1776-1777


# ----------------------------------------------------------------------------- materials
def refractive_index(m, wl):
    """n(wl) per ray.  MAT:48-51 (Sellmeier incl. Vacuum = zero coefficients MAT:54-56),
    MAT:72-79 (Constant), MAT:137-144 (Ebaf11 polynomial in wl^2 and wl^-2k), and the Cauchy user
    subclass of tests/golden/systems.py."""
    t = m["type"]
    wl = np.asarray(wl, dtype=np.float64)
    if t == "Constant":
        return np.ones(wl.shape) * m["n"]
    if t == "Cauchy":
        return m["a"] + m["b"] / wl ** 2
    if "params" in m:
        p = m["params"]
        w2 = wl * wl
        return np.sqrt(p[0] + p[1] * w2 + p[2] * wl ** -2 + p[3] * wl ** -4 + p[4] * wl ** -6 + p[5] * wl ** -8)
    b, c = np.float64(m["b"]), np.float64(m["c"])
    w2 = wl * wl
    acc = b[0] * w2 / (w2 - c[0]) + b[1] * w2 / (w2 - c[1]) + b[2] * w2 / (w2 - c[2])
    return np.sqrt(acc + 1)


# ----------------------------------------------------------------------------- small vector helpers
def _dot(a, b):
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]


def _norm(a):
    return np.sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2])


def _cross(a, b):
    return (a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0])


def _unit_or_zero(v):
    """v / |v| componentwise with NaN -> 0 (RT:1203-1209, RT:1271-1277)."""
    n = _norm(v)
    with np.errstate(invalid="ignore", divide="ignore"):
        out = [vi / n for vi in v]
    return tuple(np.where(np.isnan(o), 0.0, o) for o in out)


class Rays:
    """Column view of an (N, 8) ray block: p (3), d (3), phase, wavelength (RT:1-13)."""
    __slots__ = ("p", "d", "ph", "wl")

    def __init__(self, p, d, ph, wl):
        self.p, self.d, self.ph, self.wl = p, d, ph, wl

    @classmethod
    def from_array(cls, a):
        a = np.asarray(a, dtype=np.float64)
        return cls(tuple(a[:, i].copy() for i in range(3)), tuple(a[:, i].copy() for i in range(3, 6)),
                   a[:, 6].copy(), a[:, 7].copy())

    def to_array(self):
        return np.stack(list(self.p) + list(self.d) + [self.ph, self.wl], axis=1)

    def kill(self, mask):
        """Whole-row NaN where mask (RT:1192, 1226, 1294, 304, 1401, 1583, 1760)."""
        f = lambda c: np.where(mask, np.nan, c)
        return Rays(tuple(map(f, self.p)), tuple(map(f, self.d)), f(self.ph), f(self.wl))


def _bcast3(v, n):
    v = np.asarray(v, dtype=np.float64)
    if v.ndim == 1:
        return tuple(v[i] for i in range(3))
    return tuple(v[:, i] for i in range(3))


# ----------------------------------------------------------------------------- geometry kernels
def to_plane(r, normal, center, n_vals, exclude_backward):
    """RT:241-306 propagate_ray2plane: t = -((p-c).n)/(d.n); phase += |d t| * sign(t) * 2pi/wl * n."""
    nx, ny, nz = normal
    cx, cy, cz = center
    with np.errstate(all="ignore"):
        t = -((r.p[0] - cx) * nx + (r.p[1] - cy) * ny + (r.p[2] - cz) * nz) / \
            (r.d[0] * nx + r.d[1] * ny + r.d[2] * nz)
        sgn = np.where(t < 0, -1.0, 1.0)
        v = tuple(di * t for di in r.d)
        p = tuple(pi + vi for pi, vi in zip(r.p, v))
        ph = r.ph + _norm(v) * sgn * 2 * np.pi / r.wl * n_vals
    out = Rays(p, r.d, ph, r.wl)
    if exclude_backward:
        out = out.kill(sgn == -1)
    return out, t


def sphere_hit(r, center, radius, n_vals):
    """RT:1479-1516: nearest t > 0 root of |p + d t - c|^2 = R^2; miss -> p, phase NaN (d, wl kept)."""
    cx, cy, cz = center
    with np.errstate(all="ignore"):
        ox, oy, oz = r.p[0] - cx, r.p[1] - cy, r.p[2] - cz
        B = 2 * (r.d[0] * ox + r.d[1] * oy + r.d[2] * oz)
        C = ox ** 2 + oy ** 2 + oz ** 2 - radius ** 2
        root = np.sqrt(B ** 2 - 4 * C)
        t1 = 0.5 * (-B + root)
        t2 = 0.5 * (-B - root)
        t1 = np.where(t1 < 0, np.inf, t1)
        t2 = np.where(t2 < 0, np.inf, t2)
        t = np.minimum(t1, t2)                      # NaN-propagating like np.min(axis=1)
        t = np.where(t == np.inf, np.nan, t)
        p = tuple(pi + di * t for pi, di in zip(r.p, r.d))
        step = tuple(qi - pi for qi, pi in zip(p, r.p))
        ph = r.ph + _norm(step) * 2 * np.pi / r.wl * n_vals
    return Rays(p, r.d, ph, r.wl)


def on_flat(p, center, normal, aperture):
    """RT:1339-1347 (also PlaneMirror RT:1405-1412)."""
    with np.errstate(invalid="ignore"):
        rel = tuple(pi - ci for pi, ci in zip(p, center))
        return (np.abs(_dot(rel, normal)) < 1e-12) & (_norm(rel) <= aperture)


def on_sphere(p, center, radius, axis, aperture):
    """RT:1518-1535; the aperture is measured from the line through the ORIGIN along input_axis."""
    with np.errstate(invalid="ignore"):
        rel = tuple(pi - ci for pi, ci in zip(p, center))
        on = np.abs(_norm(rel) - abs(radius)) < 1e-12
        s = _dot(p, axis)
        ortho = tuple(pi - s * ai for pi, ai in zip(p, axis))
        return on & (_norm(ortho) <= aperture)


def snell(ri, normals, n1, n2):
    """RT:1197-1221: refract d about the surface normal; TIR -> position NaN only."""
    with np.errstate(all="ignore"):
        nb = _unit_or_zero(_cross(ri.d, normals))
        nc = _unit_or_zero(_cross(normals, nb))
        mag_nc = n1 / n2 * _dot(nc, ri.d)
        sgn = np.sign(_dot(normals, ri.d))
        tang = sgn * np.sqrt(1 - mag_nc ** 2)
        d_out = tuple(mag_nc * c + tang * n for c, n in zip(nc, normals))
    bad = np.isnan(d_out[0])
    p = tuple(np.where(bad, np.nan, pi) for pi in ri.p)
    return Rays(p, d_out, ri.ph.copy(), ri.wl.copy())


def mirror(ri, normals):
    """RT:1267-1289: reflect d (normal component flips)."""
    with np.errstate(all="ignore"):
        nb = _unit_or_zero(_cross(ri.d, normals))
        nc = _unit_or_zero(_cross(normals, nb))
        mag_na = -_dot(normals, ri.d)
        mag_nc = _dot(nc, ri.d)
        d_out = tuple(mag_na * n + mag_nc * c for n, c in zip(normals, nc))
    bad = np.isnan(d_out[0])
    p = tuple(np.where(bad, np.nan, pi) for pi in ri.p)
    return Rays(p, d_out, ri.ph.copy(), ri.wl.copy())


# ----------------------------------------------------------------------------- per-surface propagate
def propagate(s, r, m1, m2):
    """One surface: returns (plane at the surface, plane after the surface)."""
    t = s["type"]
    if t == "PerfectLens":
        return _perfect_lens(s, r, m1, m2)
    center = tuple(np.float64(s["center"]))
    if t in ("FlatSurface", "PlaneMirror"):
        normal = tuple(np.float64(s["normal"]))
        ri, ts = to_plane(r, normal, center, refractive_index(m1, r.wl), exclude_backward=(t == "FlatSurface"))
        if t == "PlaneMirror":
            ri = ri.kill(ts < 0)                                   # RT:1398-1403
        normals = tuple(np.full(r.wl.shape, v) for v in normal)   # RT:1323-1329
    elif t == "SphericalSurface":
        ri = sphere_hit(r, center, s["radius"], refractive_index(m1, r.wl))
        with np.errstate(all="ignore"):
            normals = tuple((pi - ci) / s["radius"] for pi, ci in zip(ri.p, center))   # RT:1476
    else:
        raise ValueError(f"unknown surface type {t}")

    if t == "PlaneMirror":                                          # ReflectingSurface RT:1238-1303
        ro = mirror(ri, normals)
        ok = on_flat(ri.p, center, normal, s["aperture_rad"])
        return ri, ro.kill(~ok)

    axis = tuple(np.float64(s["input_axis"]))                       # RefractingSurface RT:1160-1234
    with np.errstate(invalid="ignore"):
        incoming = _dot(r.d, axis) < 0
    ri = ri.kill(incoming)
    n1 = refractive_index(m1, ri.wl)
    n2 = refractive_index(m2, ri.wl)
    ro = snell(ri, normals, n1, n2)
    if t == "FlatSurface":
        ok = on_flat(ri.p, center, normal, s["aperture_rad"])
    else:
        ok = on_sphere(ri.p, center, s["radius"], axis, s["aperture_rad"])
    return ri, ro.kill(~ok)


def _perfect_lens(s, r, m1, m2):
    """RT:1601-1801: ideal lens mapping front focal plane (h, sin t1) -> back focal plane."""
    c = tuple(np.float64(s["center"]))
    nrm = tuple(np.float64(s["normal"]))
    f = s["focal_len"]
    sin_a = np.sin(s["alpha"])
    wl = r.wl
    n1 = refractive_index(m1, wl)
    n2 = refractive_index(m2, wl)
    with np.errstate(all="ignore"):
        ffp = tuple(ci - ni * f * n1 for ci, ni in zip(c, nrm))
        bfp = tuple(ci + ni * f * n2 for ci, ni in zip(c, nrm))
        rf, _ = to_plane(r, nrm, ffp, n1, exclude_backward=False)
        s1 = rf.d
        dn = _dot(s1, nrm)
        sp = tuple(si - dn * ni for si, ni in zip(s1, nrm))
        spn = _norm(sp)
        big = spn > 1e-12
        sp = tuple(np.where(big, si / spn, si) for si in sp)
        r1 = tuple(pi - fi for pi, fi in zip(rf.p, ffp))
        r1n = _norm(r1)
        nz = r1n != 0
        r1u = tuple(np.where(nz, ri / r1n, ri) for ri in r1)
        sin_t1 = _dot(sp, s1)
        p_out = tuple(n1 * f * sin_t1 * spi + bi for spi, bi in zip(sp, bfp))
        sin_t2 = -r1n / f / n2
        cos_t2 = np.sqrt(1 - sin_t2 ** 2)
        d_out = tuple(sin_t2 * ui + cos_t2 * ni for ui, ni in zip(r1u, nrm))
        steep = (np.abs(sin_t1) > sin_a) | (np.abs(sin_t2) > sin_a)
        out = Rays(p_out, d_out, np.zeros(wl.shape), wl.copy()).kill(steep)
        pw = _dot(r1, s1)
        out.ph = rf.ph - TWO_PI / wl * n1 * pw + TWO_PI / wl * (n1 ** 2 * f + n2 ** 2 * f)
        after, _ = to_plane(out, nrm, c, refractive_index(m2, out.wl), exclude_backward=False)
        before, _ = to_plane(r, nrm, c, n1, exclude_backward=False)
    return before, after


# ----------------------------------------------------------------------------- driver
def ray_trace(surfaces, materials, rays, reference_costs=False):
    """RT:641-661 + the rank handling of RT:1175-1178: (N,8) -> (1+2S, N, 8); (8,) -> (1+2S, 1, 8);
    (k, N, 8) -> (k+2S, N, 8).  ``materials`` has len(surfaces)+1 entries (initial ... final).

    ``reference_costs=True`` (used by bench.py's CPU-baseline leg) additionally reproduces the
    reference's data movement -- the history re-concatenated after every surface (RT:1229-1232,
    O(S^2 N)) and n(lambda) re-evaluated at each of its call sites (RT:297/1213/1512) -- so the timed
    CPU path costs what the reference's does.  The returned values are identical either way."""
    if len(materials) != len(surfaces) + 1:
        raise ValueError("length of materials should be len(surfaces) + 1")
    rays = np.asarray(rays, dtype=np.float64)
    if not surfaces:
        return rays
    if rays.ndim == 1:
        rays = rays[None, None, :]
    elif rays.ndim == 2:
        rays = rays[None]
    if reference_costs:
        hist = rays
        for ii, s in enumerate(surfaces):
            cur = Rays.from_array(hist[-1])
            for _ in range(2 if s["type"] != "PlaneMirror" else 0):   # the extra n(lambda) call sites
                refractive_index(materials[ii], cur.wl)
            at, after = propagate(s, cur, materials[ii], materials[ii + 1])
            hist = np.concatenate((hist, np.stack((at.to_array(), after.to_array()), axis=0)), axis=0)
        return hist
    planes = list(rays)
    cur = Rays.from_array(planes[-1])
    for ii, s in enumerate(surfaces):
        at, after = propagate(s, cur, materials[ii], materials[ii + 1])
        planes += [at.to_array(), after.to_array()]
        cur = after
    return np.stack(planes, axis=0)


# ----------------------------------------------------------------------------- ray generators (RT:45-161)
def ray_fan(pt, theta_max, n_thetas, wavelengths, nphis=1, center_ray=(0, 0, 1)):
    """RT:45-96: index = iphi * n_thetas + itheta; d = cos t c + cos p sin t ex + sin p sin t ey."""
    c = np.array(center_ray)
    thetas = np.linspace(-theta_max, theta_max, n_thetas)
    phis = np.arange(nphis) * 2 * np.pi / nphis
    tt, pp = np.meshgrid(thetas, phis)
    tt, pp = tt.ravel(), pp.ravel()
    ex = np.cross(np.array([0, 1, 0]), c)
    ex = ex / np.linalg.norm(ex)
    ey = np.cross(c, ex)
    out = np.zeros((n_thetas * nphis, 8))
    out[:, 0:3] = np.array(pt, dtype=float).squeeze()
    for k in range(3):
        out[:, 3 + k] = c[k] * np.cos(tt) + ex[k] * np.cos(pp) * np.sin(tt) + ey[k] * np.sin(pp) * np.sin(tt)
    out[:, 7] = wavelengths
    return out


def ray_fan_rows(pt, theta_max, n_thetas, wavelengths, nphis, row0, row1, center_ray=(0, 0, 1)):
    """Rays [row0 * n_thetas, row1 * n_thetas) of ``ray_fan(pt, theta_max, n_thetas, wavelengths, nphis)``
    (whole phi rows; RT:45-96): the same operations on the same operands per ray, so the rows are
    bit-identical to the corresponding slice of the whole fan -- for tracing a large fan in pieces."""
    c = np.array(center_ray)
    thetas = np.linspace(-theta_max, theta_max, n_thetas)
    phis = np.arange(row0, row1) * 2 * np.pi / nphis
    tt, pp = np.meshgrid(thetas, phis)
    tt, pp = tt.ravel(), pp.ravel()
    ex = np.cross(np.array([0, 1, 0]), c)
    ex = ex / np.linalg.norm(ex)
    ey = np.cross(c, ex)
    out = np.zeros((n_thetas * (row1 - row0), 8))
    out[:, 0:3] = np.array(pt, dtype=float).squeeze()
    for k in range(3):
        out[:, 3 + k] = c[k] * np.cos(tt) + ex[k] * np.cos(pp) * np.sin(tt) + ey[k] * np.sin(pp) * np.sin(tt)
    out[:, 7] = wavelengths
    return out
