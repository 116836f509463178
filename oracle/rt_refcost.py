"""CPU BASELINE restatement of the reference's hot path with the reference's own data flow -- TEST AND
BENCHMARK INFRASTRUCTURE ONLY (bench.py's ``cpu_baseline`` leg, tests/).  The product never imports it.

``oracle/rt_numpy.py`` is the checker: a column-array restatement that reproduces the golden histories
bit for bit but runs ~2x faster than the reference, because it skips the reference's array plumbing.
This module is the same arithmetic, in the same IEEE order, organised the way the reference moves data
(QI2lab/ray_trace_pb @ 2024_10_08, src/raytrace/raytrace.py = RT, materials.py = MAT), so that timing it
on the GPU box's host measures what the reference costs there:

* rays travel as (N, 8) AoS blocks; positions and directions are rebuilt with ``np.stack`` into (N, 3)
  arrays, dot products are ``np.sum(a * b, axis=1)``, norms ``np.linalg.norm(axis=1)``, tangent vectors
  ``np.cross`` (RT:1197-1209, RT:1262-1277, RT:287-297);
* per-ray failures are written with boolean fancy indexing into the (N, 8) blocks (RT:1192, 1221, 1226,
  1289, 1294, 304, 1401, 1760);
* ``n(lambda)`` is evaluated at every call site the reference evaluates it (RT:297, 1213, 1512,
  1682-1687, 1741, 1750, 1776-1777);
* the history is re-concatenated after every surface (RT:1229-1232, RT:1296-1301, RT:1799).

tests/test_cpu_baseline.py pins it to the golden vectors (bit for bit) and to the oracle;
tests/golden/calibrate_cpu.py times it against the reference itself in this container.  Surfaces and
materials are the JSON dicts of tests/golden/serialize.py, as for rt_numpy.
"""
import numpy as np

from .rt_numpy import refractive_index


def _n(m, wl):
    """Material.n at a call site, with the reference's per-call costs: Sellmeier squares the wavelength
    at each of its three terms (MAT:48-51), Constant builds ones * n (MAT:72-79); other kinds as the
    oracle.  Values identical to rt_numpy.refractive_index (wl ** 2 is wl * wl)."""
    if "c" in m:                                                  # Sellmeier (and Vacuum)
        (b1, b2, b3), (c1, c2, c3) = np.float64(m["b"]), np.float64(m["c"])
        val = b1 * wl ** 2 / (wl ** 2 - c1) + b2 * wl ** 2 / (wl ** 2 - c2) + b3 * wl ** 2 / (wl ** 2 - c3)
        return np.sqrt(val + 1)
    if m["type"] == "Constant":
        return np.ones(np.atleast_1d(np.array(wl)).shape) * float(m["n"])
    return refractive_index(m, wl)


def _rows(v, n):
    v = np.asarray(v, dtype=np.float64).squeeze()
    return v[None, :] if v.ndim == 1 else v


def plane_step(rays, normal, center, m, backward_nan=False):
    """propagate_ray2plane (RT:241-306) on an (N, 8) block; returns (block, ts)."""
    rays = np.atleast_2d(np.array(rays, copy=True))
    nv, cv = _rows(normal, len(rays)), _rows(center, len(rays))
    x, y, z, dx, dy, dz, ph, wl = (rays[:, k] for k in range(8))
    ts = -((x - cv[:, 0]) * nv[:, 0] + (y - cv[:, 1]) * nv[:, 1] + (z - cv[:, 2]) * nv[:, 2]) / \
        (dx * nv[:, 0] + dy * nv[:, 1] + dz * nv[:, 2])
    with np.errstate(invalid="ignore"):
        sgn = np.ones(len(rays), dtype=int)
        sgn[ts < 0] = -1
    step = np.stack((dx, dy, dz), axis=1) * ts[:, None]
    pos = np.stack((x, y, z), axis=1) + step
    dphi = np.linalg.norm(step, axis=1) * sgn * 2 * np.pi / wl * _n(m, wl)
    out = np.concatenate((pos, np.stack((dx, dy, dz, ph + dphi, wl), axis=1)), axis=1)
    if backward_nan:
        out[sgn == -1, :] = np.nan
    return out, ts


def sphere_step(rays, s, m):
    """SphericalSurface.get_intersect (RT:1479-1516)."""
    rays = np.atleast_2d(rays)
    x, y, z, dx, dy, dz, ph, wl = (rays[:, k] for k in range(8))
    cx, cy, cz = np.asarray(s["center"], dtype=np.float64)
    R = s["radius"]
    B = 2 * (dx * (x - cx) + dy * (y - cy) + dz * (z - cz))
    C = (x - cx) ** 2 + (y - cy) ** 2 + (z - cz) ** 2 - R ** 2
    with np.errstate(invalid="ignore"):
        t = np.stack((0.5 * (-B + np.sqrt(B ** 2 - 4 * 1 * C)), 0.5 * (-B - np.sqrt(B ** 2 - 4 * 1 * C))), axis=1)
        t[t < 0] = np.inf
    t = np.min(t, axis=1)
    t[t == np.inf] = np.nan
    p0 = np.stack((x, y, z), axis=1)
    pos = p0 + np.stack((dx, dy, dz), axis=1) * t[:, None]
    dphi = np.linalg.norm(pos - np.stack((x, y, z), axis=1), axis=1) * 2 * np.pi / wl * _n(m, wl)
    return np.concatenate((pos, np.stack((dx, dy, dz, ph + dphi, wl), axis=1)), axis=1)


def _tangent(ds, normals):
    """nc: the unit tangent in the plane of d and N (RT:1203-1209 / RT:1271-1277)."""
    with np.errstate(invalid="ignore", divide="ignore"):
        nb = np.cross(ds, normals)
        nb = nb / np.linalg.norm(nb, axis=1)[:, None]
        nb[np.isnan(nb)] = 0
        nc = np.cross(normals, nb)
        nc = nc / np.linalg.norm(nc, axis=1)[:, None]
        nc[np.isnan(nc)] = 0
    return nc


def _on_flat(pts, s):
    c, nrm = np.asarray(s["center"], dtype=np.float64), np.asarray(s["normal"], dtype=np.float64)
    pts = np.atleast_2d(pts)
    a = np.abs(np.sum((pts[..., 0:3] - c) * nrm, axis=-1)) < 1e-12
    b = np.linalg.norm(pts[..., 0:3] - c, axis=-1) <= s["aperture_rad"]
    return np.logical_and(a, b)


def _on_sphere(pts, s):
    c, ax = np.asarray(s["center"], dtype=np.float64), np.asarray(s["input_axis"], dtype=np.float64)
    pts = np.atleast_2d(pts)
    on = np.abs(np.linalg.norm(pts[..., 0:3] - c, axis=-1) - abs(s["radius"])) < 1e-12
    ortho = pts[..., :3] - np.sum(pts[..., :3] * ax, axis=-1)[..., None] * ax
    return np.logical_and(on, np.linalg.norm(ortho, axis=-1) <= s["aperture_rad"])


def refract_step(hist, s, m1, m2):
    """RefractingSurface.propagate (RT:1160-1234) for FlatSurface / SphericalSurface."""
    rays = hist[-1]
    if s["type"] == "FlatSurface":
        hit, _ = plane_step(rays, s["normal"], s["center"], m1, backward_nan=True)
        normals = np.tile(np.atleast_2d(np.asarray(s["normal"], dtype=np.float64)), (hit.shape[0], 1))
    else:
        hit = sphere_step(rays, s, m1)
        normals = (np.atleast_2d(hit)[:, :3] - np.asarray(s["center"], dtype=np.float64)[None, :]) / s["radius"]
    with np.errstate(invalid="ignore"):
        back = np.sum(rays[:, 3:6] * np.asarray(s["input_axis"], dtype=np.float64), axis=1) < 0
    hit[back] = np.nan
    ds = hit[:, 3:6]
    wls = hit[:, 7][:, None]
    nc = _tangent(ds, normals)
    with np.errstate(invalid="ignore"):
        mag = _n(m1, wls) / _n(m2, wls) * np.sum(nc * ds, axis=1)[:, None]
        sgn = np.sign(np.sum(normals * ds, axis=1))[:, None]
        d_out = mag * nc + sgn * np.sqrt(1 - mag ** 2) * normals
        out = np.concatenate((hit[:, :3], d_out, hit[:, 6:]), axis=1)
        out[np.isnan(d_out[:, 0]), :3] = np.nan
    ok = _on_flat(hit, s) if s["type"] == "FlatSurface" else _on_sphere(hit, s)
    out[np.logical_not(ok)] = np.nan
    return np.concatenate((hist, np.stack((hit, out), axis=0)), axis=0)


def mirror_step(hist, s, m1):
    """ReflectingSurface.propagate (RT:1238-1303) for PlaneMirror (RT:1398-1412)."""
    hit, ts = plane_step(hist[-1], s["normal"], s["center"], m1)
    hit[ts < 0] = np.nan
    normals = np.tile(np.atleast_2d(np.asarray(s["normal"], dtype=np.float64)), (hit.shape[0], 1))
    ds = hit[:, 3:6]
    nc = _tangent(ds, normals)
    d_out = -np.sum(normals * ds, axis=1)[:, None] * normals + np.sum(nc * ds, axis=1)[:, None] * nc
    out = np.concatenate((hit[:, :3], d_out, hit[:, 6:]), axis=1)
    out[np.isnan(d_out[:, 0]), :3] = np.nan
    out[np.logical_not(_on_flat(hit, s))] = np.nan
    return np.concatenate((hist, np.stack((hit, out), axis=0)), axis=0)


def lens_step(hist, s, m1, m2):
    """PerfectLens.propagate (RT:1601-1801)."""
    c, nrm, f = np.asarray(s["center"], dtype=np.float64), np.asarray(s["normal"], dtype=np.float64), s["focal_len"]
    rays = hist[-1]
    wl = rays[:, 7]
    ffp = c[None, :] - nrm[None, :] * f * _n(m1, wl)[:, None]
    bfp = c[None, :] + nrm[None, :] * f * _n(m2, wl)[:, None]
    rf, _ = plane_step(rays, nrm, ffp, m1)
    s1 = rf[:, 3:6]
    sp = s1 - np.sum(s1 * nrm[None, :], axis=1)[:, None] * nrm[None, :]
    with np.errstate(invalid="ignore"):
        spn = np.linalg.norm(sp, axis=1)
        big = spn > 1e-12
        sp[big] = sp[big] / spn[big][:, None]
    r1 = rf[:, 0:3] - ffp
    r1n = np.linalg.norm(r1, axis=1)
    nz = r1n != 0
    r1u = np.array(r1, copy=True)
    r1u[nz] = r1u[nz] / np.linalg.norm(r1u[nz], axis=1)[:, None]
    sin1 = np.sum(sp * s1, axis=1)
    out = np.zeros(rf.shape)
    out[:, 7] = wl
    out[:, :3] = _n(m1, wl)[:, None] * f * sin1[:, None] * sp + bfp[None, :]
    with np.errstate(invalid="ignore"):
        sin2 = -r1n / f / _n(m2, wl)
        out[:, 3:6] = sin2[:, None] * r1u + np.sqrt(1 - sin2 ** 2)[:, None] * nrm[None, :]
        clip = np.logical_or(np.abs(sin1) > np.sin(s["alpha"]), np.abs(sin2) > np.sin(s["alpha"]))
        out[clip] = np.nan
    pw = np.sum(r1 * s1, axis=1)
    out[:, 6] = rf[:, 6] - 2 * np.pi / wl * _n(m1, wl) * pw + \
        2 * np.pi / wl * (_n(m1, wl) ** 2 * f + _n(m2, wl) ** 2 * f)
    after, _ = plane_step(out, nrm, c, m2)
    before, _ = plane_step(rays, nrm, c, m1)
    return np.concatenate((hist, np.stack((before, after), axis=0)), axis=0)


def ray_trace(surfaces, materials, rays):
    """System.ray_trace (RT:641-661): (N, 8) -> (2S+1, N, 8), (8,) -> (2S+1, 1, 8), (k, N, 8) appended."""
    if len(materials) != len(surfaces) + 1:
        raise ValueError("length of materials should be len(surfaces) + 1")
    hist = np.asarray(rays, dtype=np.float64)
    if hist.ndim == 1:
        hist = hist[None, None, :]
    elif hist.ndim == 2:
        hist = hist[None]
    for ii, s in enumerate(surfaces):
        m1, m2 = materials[ii], materials[ii + 1]
        t = s["type"]
        if t == "PerfectLens":
            hist = lens_step(hist, s, m1, m2)
        elif t == "PlaneMirror":
            hist = mirror_step(hist, s, m1)
        elif t in ("FlatSurface", "SphericalSurface"):
            hist = refract_step(hist, s, m1, m2)
        else:
            raise ValueError(f"unknown surface type {t}")
    return hist
