"""Sequential optical ray tracing on MI355X -- drop-in for ``raytrace.raytrace``.

A ray is the 8-vector (x, y, z, dx, dy, dz, phase, wavelength): a point on the ray, its unit
direction, the accumulated phase 2*pi/wavelength * optical path length, and the wavelength
(QI2lab/ray_trace_pb @ 2024_10_08, src/raytrace/raytrace.py = RT, lines 1-13).  z is the optical
axis; x points up and y out of the page (right-handed).

The public API mirrors the reference: ``System``, ``Doublet``, ``Surface``, ``RefractingSurface``,
``ReflectingSurface``, ``FlatSurface``, ``PlaneMirror``, ``SphericalSurface``, ``PerfectLens``, the ray
generators and the ray utilities, with the same signatures and return conventions.

What runs where
---------------
* ``System.ray_trace`` and ``Surface.propagate`` -- the hot path -- lower the system to the C ABI of
  include/rtpb.h and run ONE fused HIP kernel on gfx950 per trace (ray record in VGPRs, descriptors in
  SGPRs, each history plane written once).  NumPy input returns NumPy output (through
  ``rtpb_trace_host``, optionally sharded over several GPUs); torch CUDA tensors stay on the device.
  There is no CPU fallback: without librtpb.so these calls raise.
* Object construction, ray generators, paraxial (ABCD) analysis, ``intersect_rays`` and plotting are
  host-side NumPy/Matplotlib, as in the reference (they are O(S) or set-up work, SURVEY.md §2 rows
  7-9, 11-12).
"""
import functools
import threading
from collections.abc import Sequence
from copy import deepcopy
from typing import Optional

import numpy as np

from . import _capi as C
from . import _engine as E
from .materials import Material, Vacuum

array = np.ndarray


def _is_torch_cuda(x):
    t = type(x)
    return t.__module__.startswith("torch") and t.__name__ == "Tensor" and x.is_cuda


def get_free_space_abcd(d: float, n: float = 1.) -> np.ndarray:
    """Ray-transfer (ABCD) matrix of free propagation over distance d in index n (RT:32-41)."""
    return np.array([[1, d / n], [0, 1]])


# =============================================================================== ray generators
def get_ray_fan(pt, theta_max: float, n_thetas: int, wavelengths, nphis: int = 1, center_ray=(0, 0, 1),
                *, device=None, dtype=None, devices=None):
    """Fan of rays leaving the point ``pt`` (RT:45-96).

    Ray (iphi, itheta) -> index iphi*n_thetas + itheta; direction
    cos(theta) c + cos(phi) sin(theta) ex + sin(phi) sin(theta) ey with ex = y x c / |.|, ey = c x ex,
    theta in linspace(-theta_max, theta_max, n_thetas), phi = k 2 pi / nphis.  Phase 0.

    ``wavelengths``: one value, or one per ray (an array of n_thetas*nphis values, NumPy or torch), as
    ``rays[:, 7] = wavelengths`` assigns it (RT:94).

    With ``device`` (a torch CUDA device), the fan is generated directly in HBM by the ``rtpb_ray_fan_tables``
    kernel (``rtpb_ray_fan_tables_wl`` for per-ray wavelengths) and returned as a torch tensor.  With ``devices`` (GPU
    indices) it is generated as contiguous ray-index shards, one per GPU (whole phi rows, as even as the
    row count allows), and returned as the list of per-device tensors -- the input of a multi-GPU
    ``System.ray_trace`` that never gathers (e.g. the C4 configuration, 100M rays over 8 GPUs)."""
    center_ray = np.array(center_ray)
    if np.linalg.norm(center_ray) != 1:
        raise ValueError("center_ray must be a unit vector")
    if devices is not None:
        import torch
        out = []
        if not _is_torch_cuda(wavelengths) and np.ndim(wavelengths) > 0 and np.size(wavelengths) > 1:
            wavelengths = _wavelength_column(wavelengths, int(n_thetas) * int(nphis))   # host column, once
        for (p0, p1), d in zip(shard_bounds(int(nphis), len(devices)), devices):
            buf = torch.empty(((p1 - p0) * n_thetas, 8), device=torch.device("cuda", int(d)),
                              dtype=torch.float32 if dtype in ("float32", np.float32, torch.float32) else torch.float64)
            out.append(fan_into(buf, pt, theta_max, n_thetas, wavelengths, nphis, center_ray, phi_rows=(p0, p1)))
        return out
    if device is not None:
        return _ray_fan_device(pt, theta_max, n_thetas, wavelengths, nphis, center_ray, device, dtype)
    thetas = np.linspace(-theta_max, theta_max, n_thetas)
    phis = np.arange(nphis) * 2 * np.pi / nphis
    tt, pp = np.meshgrid(thetas, phis)
    tt, pp = tt.ravel(), pp.ravel()
    ex = np.cross(np.array([0, 1, 0]), center_ray)
    ex = ex / np.linalg.norm(ex)
    ey = np.cross(center_ray, ex)
    rays = np.zeros((n_thetas * nphis, 8))
    rays[:, 0:3] = np.array(pt).squeeze()
    ct, st, cp, sp = np.cos(tt), np.sin(tt), np.cos(pp), np.sin(pp)
    for k in range(3):
        rays[:, 3 + k] = center_ray[k] * ct + ex[k] * cp * st + ey[k] * sp * st
    rays[:, 7] = wavelengths
    return rays


def _ray_fan_device(pt, theta_max, n_thetas, wavelength, nphis, center_ray, device, dtype):
    import torch
    dev = torch.device(device)
    tdt = torch.float32 if dtype in ("float32", np.float32, torch.float32) else torch.float64
    out = torch.empty((n_thetas * nphis, 8), dtype=tdt, device=dev)
    fan_into(out, pt, theta_max, n_thetas, wavelength, nphis, center_ray)
    return out


@functools.lru_cache(maxsize=16)
def _fan_tables(theta_max, n_thetas, nphis, center_ray, center_dtype):
    """Host-side values of RT:71-81 (cached: a sweep reuses one fan shape for every field point)."""
    center_ray = np.array(center_ray, dtype=center_dtype)
    thetas = np.linspace(-theta_max, theta_max, n_thetas)
    phis = np.arange(nphis) * 2 * np.pi / nphis
    enx = np.cross(np.array([0, 1, 0]), center_ray)
    enx = enx / np.linalg.norm(enx)
    eny = np.cross(center_ray, enx)
    tcs = np.ascontiguousarray(np.stack((np.cos(thetas), np.sin(thetas)), axis=1), dtype=np.float64)
    pcs = np.ascontiguousarray(np.stack((np.cos(phis), np.sin(phis)), axis=1), dtype=np.float64)
    for a in (enx, eny, tcs, pcs):
        a.setflags(write=False)
    return enx, eny, tcs, pcs


def _wavelength_column(wavelengths, n, device=None):
    """``rays[:, 7] = wavelengths`` for n rays (RT:94, RT:159) as a float64 column: None for one wavelength
    (a scalar or a one-element array: the kernel's constant), else the n per-ray values -- NumPy (host) or, for
    a torch tensor or with ``device``, a contiguous CUDA tensor.  Shapes NumPy's assignment rejects raise."""
    import torch
    if isinstance(wavelengths, torch.Tensor):
        if wavelengths.numel() == 1:
            return None
        dev = device if device is not None else (wavelengths.device if wavelengths.is_cuda else None)
        col = torch.empty(n, dtype=torch.float64, device=dev if dev is not None else "cpu")
        col[:] = wavelengths.to(device=col.device, dtype=torch.float64)
        return col
    w = np.asarray(wavelengths)
    if w.ndim == 0 or w.size == 1:
        return None
    if w.shape == (n,) and w.dtype == np.float64 and w.flags.c_contiguous:
        col = w
    else:
        col = np.empty(n)
        col[:] = w                       # the reference's assignment: same broadcasting, same errors
    if device is not None:
        return torch.from_numpy(col).to(device)
    return col


def _wavelength_args(wavelength, n_total, lo, hi, device):
    """(scalar wavelength, per-ray CUDA column of rays lo..hi or None) for a generator launch."""
    col = _wavelength_column(wavelength, n_total)
    if col is None:
        return float(np.asarray(wavelength.cpu() if hasattr(wavelength, "cpu") else wavelength).ravel()[0]), None
    import torch
    part = col[lo:hi]
    part = part.to(device) if isinstance(part, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(part)).to(device)
    return 0.0, part.contiguous()


def fan_into(buf, pt, theta_max, n_thetas, wavelength, nphis=1, center_ray=(0, 0, 1), phi_rows=None):
    """Write get_ray_fan(pt, theta_max, n_thetas, wavelength, nphis, center_ray) into the torch CUDA
    buffer ``buf`` ((n_thetas*nphis, 8), float64 or float32) on its current stream.  ``phi_rows=(p0, p1)``
    writes only rays p0*n_thetas .. p1*n_thetas - 1 (a contiguous shard; ``buf`` then has
    (p1-p0)*n_thetas rows).  ``wavelength``: a scalar or the whole fan's n_thetas*nphis per-ray values
    (NumPy or torch; a shard reads its own slice).

    Every host-side value of RT:71-81 -- the linspace thetas, the phis, their np.cos / np.sin, and the
    enx / eny basis -- is evaluated here with NumPy exactly as the reference does (n_thetas + nphis
    trig evaluations instead of n_thetas * nphis); the kernel does the per-ray products in the
    reference's order, so the device fan is bit-identical to the reference's."""
    import torch
    center_ray = np.array(center_ray)
    enx, eny, tcs, pcs = _fan_tables(float(theta_max), int(n_thetas), int(nphis), tuple(center_ray.tolist()),
                                     center_ray.dtype.str)
    vec = [np.ascontiguousarray(np.asarray(v, dtype=np.float64).ravel()) for v in (pt, center_ray, enx, eny)]
    code = C.RTPB_F64 if buf.dtype == torch.float64 else C.RTPB_F32
    p0, p1 = (0, int(nphis)) if phi_rows is None else (int(phi_rows[0]), int(phi_rows[1]))
    if not 0 <= p0 <= p1 <= nphis or buf.shape != (int(n_thetas) * (p1 - p0), 8) or not buf.is_contiguous():
        raise ValueError("fan_into: buffer shape does not match the fan (or its phi rows)")
    if p1 == p0:
        return buf
    pcs = np.ascontiguousarray(pcs[p0:p1])
    nt = int(n_thetas)
    wl, col = _wavelength_args(wavelength, nt * int(nphis), p0 * nt, p1 * nt, buf.device)
    stream = torch.cuda.current_stream(buf.device).cuda_stream
    if col is None:
        C.check(C.lib().rtpb_ray_fan_tables(buf.device.index or 0, code, buf.data_ptr(), vec[0].ctypes.data,
                                            nt, p1 - p0, vec[1].ctypes.data, vec[2].ctypes.data,
                                            vec[3].ctypes.data, tcs.ctypes.data, pcs.ctypes.data, wl, stream))
    else:
        # col is read by the kernel on this stream; torch's allocator reuses its memory only in stream order
        C.check(C.lib().rtpb_ray_fan_tables_wl(buf.device.index or 0, code, buf.data_ptr(), vec[0].ctypes.data,
                                               nt, p1 - p0, vec[1].ctypes.data, vec[2].ctypes.data,
                                               vec[3].ctypes.data, tcs.ctypes.data, pcs.ctypes.data, col.data_ptr(),
                                               stream))
    return buf


def get_collimated_rays(pt, displacement_max, n_disps: int, wavelengths, nphis: int = 1, phi_start: float = 0.,
                        normal=(0, 0, 1), *, device=None, dtype=None):
    """Parallel rays along ``normal`` through a disk of points around ``pt`` (RT:99-161).

    index = idisp*nphis + iphi; position pt + off (n1 cos phi + n2 sin phi) with n1 = y x normal
    (or normal x x when normal is along y), n2 = normal x n1; offsets linspace(-dmax, dmax, n_disps).
    ``wavelengths``: one value or one per ray (n_disps*nphis), "either floating point or an array the same size
    as n_disps * nphis" (RT:115).  With ``device`` the bundle is generated in HBM by
    ``rtpb_collimated_rays_tables`` (``rtpb_collimated_rays_tables_wl`` for per-ray wavelengths)."""
    if np.abs(np.linalg.norm(normal) - 1) > 1e-12:
        raise ValueError("normal must be a normalized vector")
    if device is not None:
        return _collimated_device(pt, displacement_max, n_disps, wavelengths, nphis, phi_start, normal, device,
                                  dtype)
    phis = np.arange(nphis) * 2 * np.pi / nphis + phi_start
    offs = np.linspace(-displacement_max, displacement_max, n_disps)
    pp, oo = np.meshgrid(phis, offs)
    pp, oo = pp.ravel(), oo.ravel()
    pt = np.array(pt).squeeze()
    normal = np.array(normal).squeeze()
    n1 = np.cross(np.array([0, 1, 0]), normal)
    if np.linalg.norm(n1) == 0:
        n1 = np.cross(normal, np.array([1, 0, 0]))
    n1 = n1 / np.linalg.norm(n1)
    n2 = np.cross(normal, n1)
    n2 = n2 / np.linalg.norm(n2)
    rays = np.zeros((n_disps * nphis, 8))
    rays[:, 0:3] = pt[None, :] + n1[None, :] * (oo * np.cos(pp))[:, None] + n2[None, :] * (oo * np.sin(pp))[:, None]
    rays[:, 3:6] = normal
    rays[:, 7] = wavelengths
    return rays


def _collimated_device(pt, displacement_max, n_disps, wavelength, nphis, phi_start, normal, device, dtype):
    """get_collimated_rays in HBM: the host-side values of RT:128-144 (phis, offsets, their cos/sin,
    the n1/n2 basis) come from NumPy exactly as in the reference, the per-ray products from
    ``rtpb_collimated_rays_tables`` -- bit-identical to the reference's rays."""
    import torch
    dev = torch.device(device)
    tdt = torch.float32 if dtype in ("float32", np.float32, torch.float32) else torch.float64
    out = torch.empty((n_disps * nphis, 8), dtype=tdt, device=dev)
    phis = np.arange(nphis) * 2 * np.pi / nphis + phi_start
    offs = np.ascontiguousarray(np.linspace(-displacement_max, displacement_max, n_disps), dtype=np.float64)
    normal = np.array(normal).squeeze()
    n1 = np.cross(np.array([0, 1, 0]), normal)
    if np.linalg.norm(n1) == 0:
        n1 = np.cross(normal, np.array([1, 0, 0]))
    n1 = n1 / np.linalg.norm(n1)
    n2 = np.cross(normal, n1)
    n2 = n2 / np.linalg.norm(n2)
    pcs = np.ascontiguousarray(np.stack((np.cos(phis), np.sin(phis)), axis=1), dtype=np.float64)
    vec = [np.ascontiguousarray(np.asarray(v, dtype=np.float64).ravel()) for v in (pt, normal, n1, n2)]
    n = int(n_disps) * int(nphis)
    wl, col = _wavelength_args(wavelength, n, 0, n, dev)
    code = C.RTPB_F64 if tdt == torch.float64 else C.RTPB_F32
    stream = torch.cuda.current_stream(dev).cuda_stream
    if col is None:
        C.check(C.lib().rtpb_collimated_rays_tables(dev.index or 0, code, out.data_ptr(), vec[0].ctypes.data,
                                                    int(n_disps), int(nphis), vec[1].ctypes.data, vec[2].ctypes.data,
                                                    vec[3].ctypes.data, offs.ctypes.data, pcs.ctypes.data, wl, stream))
    else:
        C.check(C.lib().rtpb_collimated_rays_tables_wl(dev.index or 0, code, out.data_ptr(), vec[0].ctypes.data,
                                                       int(n_disps), int(nphis), vec[1].ctypes.data,
                                                       vec[2].ctypes.data, vec[3].ctypes.data, offs.ctypes.data,
                                                       pcs.ctypes.data, col.data_ptr(), stream))
    return out


# =============================================================================== ray utilities
def intersect_rays(ray1, ray2):
    """Intersection point of pairs of rays (NaN when they do not meet within 1e-12) (RT:164-238).
    torch CUDA inputs are solved on the GPU (``rtpb_intersect_rays``) and return a CUDA tensor."""
    if _is_torch_cuda(ray1) or _is_torch_cuda(ray2):
        return _intersect_rays_device(ray1, ray2)
    ray1 = np.atleast_2d(ray1)
    ray2 = np.atleast_2d(ray2)
    if len(ray1) == 1 and len(ray2) > 1:
        ray1 = np.tile(ray1, (len(ray2), 1))
    if len(ray2) == 1 and len(ray1) > 1:
        ray2 = np.tile(ray2, (len(ray1), 1))
    if len(ray1) != len(ray2):
        raise ValueError("ray1 and ray2 must be the same length")
    p1, d1 = ray1[:, 0:3], ray1[:, 3:6]
    p2, d2 = ray2[:, 0:3], ray2[:, 3:6]
    x1, y1, z1 = p1.T
    dx1, dy1, dz1 = d1.T
    x2, y2, z2 = p2.T
    dx2, dy2, dz2 = d2.T
    # distance s along ray2 from whichever 2x2 sub-system is non-singular (xz, then xy, then yz)
    s = np.full(len(ray1), np.nan)
    with np.errstate(invalid="ignore", divide="ignore"):
        det_xz = dx2 * dz1 - dz2 * dx1
        det_xy = dx2 * dy1 - dy2 * dx1
        det_yz = dz2 * dy1 - dy2 * dz1
        use_xz = det_xz != 0
        use_xy = ~use_xz & (det_xy != 0)
        use_yz = ~use_xz & ~use_xy & (det_yz != 0)
        s[use_xz] = (((z2 - z1) * dx1 - (x2 - x1) * dz1) / det_xz)[use_xz]
        s[use_xy] = (((y2 - y1) * dx1 - (x2 - x1) * dy1) / det_xy)[use_xy]
        s[use_yz] = (((y2 - y1) * dz1 - (z2 - z1) * dy1) / det_yz)[use_yz]
    t = np.full(len(ray1), np.nan)
    with np.errstate(all="ignore"):
        use_z = dz1 != 0
        use_y = ~use_z & (dy1 != 0)
        use_x = ~(use_z | use_y)
        t[use_z] = ((z2 + s * dz2 - z1) / dz1)[use_z]
        t[use_y] = ((y2 + s * dy2 - y1) / dy1)[use_y]
        t[use_x] = ((x2 + s * dx2 - x1) / dx1)[use_x]
    on1 = np.stack((x1, y1, z1), axis=1) + t[:, None] * np.stack((dx1, dy1, dz1), axis=1)
    on2 = np.stack((x2, y2, z2), axis=1) + s[:, None] * np.stack((dx2, dy2, dz2), axis=1)
    with np.errstate(invalid="ignore"):
        miss = np.max(np.abs(on1 - on2), axis=1) > 1e-12
        on1[miss] = np.nan
    return on1


def _intersect_rays_device(ray1, ray2):
    import torch
    dev = ray1.device if _is_torch_cuda(ray1) else ray2.device
    tdt = ray1.dtype if _is_torch_cuda(ray1) else ray2.dtype
    r1 = torch.as_tensor(ray1, device=dev).to(tdt).reshape(-1, 8).contiguous()
    r2 = torch.as_tensor(ray2, device=dev).to(tdt).reshape(-1, 8).contiguous()
    n1, n2 = r1.shape[0], r2.shape[0]
    if n1 != n2 and n1 != 1 and n2 != 1:
        raise ValueError("ray1 and ray2 must be the same length")
    out = torch.empty((max(n1, n2), 3), dtype=tdt, device=dev)
    C.check(C.lib().rtpb_intersect_rays(dev.index or 0, C.RTPB_F64 if tdt == torch.float64 else C.RTPB_F32,
                                        r1.data_ptr(), n1, r2.data_ptr(), n2, out.data_ptr(),
                                        torch.cuda.current_stream(dev).cuda_stream))
    return out


def propagate_ray2plane(rays, normal, center, material: Material, exclude_backward_propagation: bool = False):
    """Move rays onto the plane {(p - center).normal = 0} (RT:241-306).

    Returns ``(rays_out, ts)``; the phase grows by |d t| sign(t) 2 pi / wavelength n(wavelength); rays
    that must travel backwards become NaN when ``exclude_backward_propagation``.  ``normal`` and
    ``center`` broadcast against (N, 3).  Runs on the GPU (``rtpb_propagate_plane``, the same
    arithmetic as the fused trace kernel): NumPy in -> NumPy out (float64), torch CUDA in -> torch out."""
    import torch
    on_device = _is_torch_cuda(rays)
    dev = rays.device if on_device else torch.device("cuda", torch.cuda.current_device())
    r = (rays if on_device else torch.from_numpy(np.atleast_2d(np.asarray(rays, dtype=np.float64)))).to(
        dev, dtype=torch.float64)
    r = r.reshape(-1, 8).contiguous()
    n = r.shape[0]

    def plane_vec(v):
        a = np.asarray(v.cpu() if _is_torch_cuda(v) else v, dtype=np.float64).squeeze()
        if a.ndim == 1 and a.size == 3:
            return torch.from_numpy(a.copy()).to(dev), 0
        a = a.reshape(-1, 3)
        if a.shape[0] != n:
            raise ValueError("normal and center must broadcast to (N, 3)")
        return torch.from_numpy(np.ascontiguousarray(a)).to(dev), 1

    nv, n_per = plane_vec(normal)
    cv, c_per = plane_vec(center)
    low = E.lower_material(material, lambda: E.distinct_wavelengths(r[:, 7]))
    ws = torch.empty(256 + 16 * max(low.table_len, 1), dtype=torch.uint8, device=dev)
    out = torch.empty_like(r)
    ts = torch.empty(n, dtype=torch.float64, device=dev)
    C.check(C.lib().rtpb_propagate_plane(dev.index or 0, C.RTPB_F64, r.data_ptr(), n, nv.data_ptr(), n_per,
                                         cv.data_ptr(), c_per, C.ctypes.byref(low), int(bool(exclude_backward_propagation)),
                                         out.data_ptr(), ts.data_ptr(), ws.data_ptr(), ws.numel(),
                                         torch.cuda.current_stream(dev).cuda_stream))
    if on_device:
        return out, ts
    return out.cpu().numpy(), ts.cpu().numpy()


def ray_angle_about_axis(rays, reference_axis):
    """Angle of each ray to ``reference_axis`` and the unit direction of its transverse part (RT:309-328)."""
    rays = np.atleast_2d(rays)
    reference_axis = np.asarray(reference_axis)
    cosines = np.sum(rays[:, 3:6] * reference_axis[None, :], axis=1)
    angles = np.arccos(cosines)
    na = rays[:, 3:6] - cosines[:, None] * reference_axis[None, :]
    na = na / np.linalg.norm(na, axis=1)[:, None]
    return angles, na


def dist_pt2plane(pts, normal, center):
    """Distance from points to a plane and the nearest points on it (RT:331-353)."""
    pts = np.atleast_2d(pts)
    npts = pts.shape[0]
    rays = np.concatenate((pts, np.tile(normal, (npts, 1)), np.zeros((npts, 2))), axis=1)
    rays_int, _ = propagate_ray2plane(rays, normal, center, Vacuum())
    return np.linalg.norm(rays_int[:, :3] - pts, axis=1), rays_int[:, :3]


# =============================================================================== systems
def _dtype_code(dtype, rays):
    if dtype is None:
        return C.RTPB_F64               # the reference always computes in float64
    name = getattr(dtype, "__name__", None) or str(dtype)
    name = name.replace("torch.", "")
    if name in ("float64", "double", "f64"):
        return C.RTPB_F64
    if name in ("float32", "float", "f32"):
        return C.RTPB_F32
    raise ValueError(f"dtype must be float64 or float32, got {dtype!r}")


def _is_shard_list(rays):
    return isinstance(rays, (list, tuple)) and len(rays) > 0 and all(_is_torch_cuda(r) for r in rays)


def shard_bounds(n, n_shards):
    """Contiguous ray-index shards [lo, hi) of n rays over n_shards devices -- the split rtpb_trace_host and
    ray_trace_pb_amd.distributed use."""
    return [(n * g // n_shards, n * (g + 1) // n_shards) for g in range(n_shards)]


def history_buffer(shape, dtype, device):
    """A preallocated history for ``ray_trace(..., out=)``: a C-contiguous torch CUDA tensor of ``shape``
    ((P, N, 8), P stored planes) and ``dtype`` (torch.float32 / torch.float64) on ``device``, whose device
    memory is mapped in shuffled 64 MiB chunks so that the history's many-plane writes run at their fast rate
    wherever the memory lies.  It is an ordinary torch allocation (the device's history pool, a
    torch.cuda.MemPool whose segments librtpb maps): Tensor.record_stream and torch's memory statistics apply."""
    return E.history_buffer(shape, dtype, device)


def record_stream(tensor, stream):
    """Mark a use of ``tensor`` on ``stream`` before it is freed: torch's ``Tensor.record_stream`` (enough for
    every history this package allocates), plus the library's record for a buffer of its own C-ABI pool."""
    E.record_stream(tensor, stream)


def trim_history_buffers():
    """Release the device memory the history pools cache (``torch.cuda.empty_cache()`` releases torch's default
    pool; a history pool keeps its unused segments until this call or until another allocation needs them)."""
    E.trim_history_buffers()


def history_buffers_held(device=-1):
    """(bytes, segments) of history memory cached but not in use on ``device`` (-1: all devices)."""
    return E.history_buffers_held(device)


def trace_surfaces(surfaces, materials, rays, *, planes="all", dtype=None, devices=None, layout="aos", gather=True,
                   out=None):
    """Trace ``rays`` through ``surfaces`` with ``materials`` (len(surfaces)+1 entries) on the GPU.

    ``rays`` follows the reference's rank convention (RT:1175-1178): (8,) -> one ray, (N, 8) -> a
    bundle (history plane 0 = the input), (k, N, 8) -> an existing history whose last plane is traced
    and which is extended.  ``planes`` = 'all' (reference output), 'final', or a list of plane indices
    of the new trace (0 = input, 2i+1 at surface i, 2i+2 after it).

    Multi-GPU in one process: a NumPy bundle with ``devices`` is split by ray index inside the library
    (one host thread per GPU); a torch CUDA bundle with ``devices`` is scattered by ray index to the
    listed GPUs, traced there concurrently, and gathered back onto its own device (``gather=False``:
    the list of per-device histories instead); a list of torch CUDA shards (one per device, e.g. from
    ``get_ray_fan(..., devices=)``) is traced where it lives and returns the list of per-device
    histories.  Systems longer than RTPB_MAX_SURFACES run as consecutive fused segments.

    ``out``: a torch CUDA (N, 8) bundle on one device may be traced into a caller-provided history --
    a C-contiguous tensor of exactly the result's shape, type and device (for example a
    :func:`history_buffer`, whose placement keeps the many-plane writes at their fast rate); the
    result is ``out`` itself."""
    if len(materials) != len(surfaces) + 1:
        raise ValueError("length of materials should be len(surfaces) + 1")
    if out is not None and (not _is_torch_cuda(rays) or rays.ndim == 3 or devices is not None
                            or len(surfaces) > C.RTPB_MAX_SURFACES):
        raise ValueError("out= is for a torch CUDA (N, 8) or (8,) bundle on one device, up to "
                         f"{C.RTPB_MAX_SURFACES} surfaces")
    if not surfaces:
        return rays
    if _is_shard_list(rays):
        # each shard on its own device: launches are asynchronous, so the devices trace concurrently
        return [trace_surfaces(surfaces, materials, r, planes=planes, dtype=dtype, layout=layout) for r in rays]
    on_device = _is_torch_cuda(rays)
    if on_device and devices is not None:
        devs = _resolve_devices(devices)
        if devs and (len(devs) > 1 or devs[0] != rays.device.index):
            return _trace_scattered(surfaces, materials, rays, devs, planes=planes, dtype=dtype, layout=layout,
                                    gather=gather)
    if len(surfaces) > C.RTPB_MAX_SURFACES:
        return _trace_segmented(surfaces, materials, rays, planes=planes, dtype=dtype, devices=devices, layout=layout)
    if not on_device:
        rays = np.asarray(rays)
    nd = rays.ndim
    if nd == 2:
        last = rays                     # the common (N, 8) bundle: no views (a torch view costs microseconds)
    elif nd == 1:
        rays = rays[None, None, :]
        last = rays[-1]
    elif nd == 3:
        last = rays[-1]
    if nd not in (1, 2, 3) or rays.shape[-1] != 8:
        raise ValueError(f"rays must have shape (8,), (N, 8) or (k, N, 8); got {tuple(rays.shape)}")
    k = rays.shape[0] if nd == 3 else 1
    n = last.shape[0]
    code = _dtype_code(dtype, rays)
    sel = E.resolve_planes(planes, len(surfaces))
    full = planes == "all" if isinstance(planes, str) else False

    layout_code = C.RTPB_AOS if layout == "aos" else C.RTPB_SOA
    if on_device:
        return _trace_device_tables(surfaces, materials, rays, last, code, sel, full and k > 1, layout_code, out)

    def wavelengths():
        return E.distinct_wavelengths(last[:, 7])

    low = E.lower(surfaces, materials, wavelengths, code)
    if layout != "aos":
        raise ValueError("layout='soa' is only available for device (torch CUDA) inputs")
    devs = _resolve_devices(devices)
    if full and k > 1:
        out = E.host_empty((k - 1 + len(sel), n, 8), np.float64 if code == C.RTPB_F64 else np.float32)
        out[:k] = rays
        E.trace_host(low, last, sel[1:], devs, out=out[k:])
        return out
    return E.trace_host(low, last, sel, devs)


# histories at least this large are allocated in the history pool (shuffled-chunk placement).  From
# the one-process sweep of profiles/r05/b/history_threshold.log (the same trace into torch.empty and into
# history-pool histories, 4 of each): equal up to 256 MiB, the pool 2 % faster at 512 MiB, 11 % faster at C2's
# 671 MiB history (1M rays, float64) and 8 % faster for a quarter-size C3 history; smaller histories are single
# chunks, where the shuffle has nothing to place.  Both are torch allocations with torch's stream rules.
POOLED_HISTORY_BYTES = 512 << 20


def _default_history(code, last, sel, layout_code):
    """The result buffer of a trace without out=: a history-pool tensor for large histories, else None
    (trace_device then allocates with torch's default pool)."""
    import torch
    n = last.shape[0]
    elem = 8 if code == C.RTPB_F64 else 4
    if len(sel) * n * 8 * elem < POOLED_HISTORY_BYTES:
        return None
    shape = (len(sel), n, 8) if layout_code == C.RTPB_AOS else (len(sel), 8, n)
    return E.pool_empty(shape, torch.float64 if elem == 8 else torch.float32, last.device)


_MISS_FLAGS = threading.local()


def _miss_flag(device):
    """The table-miss flag of rtpb_trace_checked for this thread and device: one int32 in pinned host memory,
    which the kernel writes directly (a miss is rare) and the host reads after synchronising the launch
    stream -- no device allocation, fill or device-to-host copy per call."""
    import torch
    flags = getattr(_MISS_FLAGS, "flags", None)
    if flags is None:
        flags = _MISS_FLAGS.flags = {}
    f = flags.get(device)
    if f is None:
        f = flags[device] = torch.zeros(1, dtype=torch.int32, pin_memory=True)
    return f


def _trace_device_tables(surfaces, materials, rays, last, code, sel, extend, layout_code, out=None):
    """The torch-CUDA trace of trace_surfaces.  Tabulated materials (user n() overrides, Ebaf11) are
    lowered with the key set of the previous bundle traced through them when there is one, and the kernel
    flags any ray whose wavelength is not among those keys (rtpb_trace_checked); only then is the bundle's
    wavelength column scanned (rtpb_distinct_keys) and the bundle re-traced with its own keys.  Either
    way every ray reads n() of its own wavelength: bit-identical to lowering with the bundle's keys.
    ``extend``: ``rays`` is a (k > 1, N, 8) history that the full trace extends (RT:1175-1178)."""
    import torch
    if out is not None:
        n = last.shape[0]
        shape = (len(sel), n, 8) if layout_code == C.RTPB_AOS else (len(sel), 8, n)
        E.check_out(out, shape, torch.float64 if code == C.RTPB_F64 else torch.float32, last.device)

    def run(low, miss=None):
        if extend:
            new = E.trace_device(low, last, sel[1:], miss=miss)
            return torch.cat((rays.to(new.dtype), new), dim=0)
        if out is not None:
            return E.trace_device(low, last, sel, layout_out=layout_code, miss=miss, out=out)
        dst = _default_history(code, last, sel, layout_code)
        return E.trace_device(low, last, sel, layout_out=layout_code, miss=miss, out=dst, own_out=dst is not None)

    def run_checked(low):
        """The launch with the table-miss flag; None when some ray's wavelength is not a key of the tables."""
        miss = _miss_flag(last.device)
        miss[0] = 0
        res = run(low, miss)
        torch.cuda.current_stream(last.device).synchronize()       # the launch has set the flag or not
        return res if int(miss[0]) == 0 else None

    memo = E.memo_lookup(surfaces, materials, code)
    missed = False
    if memo is not None:
        low, with_keys = memo
        if not with_keys:
            return run(low)
        res = run_checked(low)                 # the previous bundle's keys, memoised with the lowering
        if res is not None:
            return res
        del res
        missed = True                          # those keys miss a ray: straight to the bundle's own keys
    tab = E.tabulated(materials)
    if not tab:
        low = E.lower(surfaces, materials, None, code, tab=tab)
        E.memo_store(surfaces, materials, code, low)
        return run(low)
    fp = E.table_fingerprint(tab)
    prev = None if missed else E.previous_keys(fp)
    if prev is not None:
        low = E.lower(surfaces, materials, lambda: prev, code)
        res = run_checked(low)
        if res is not None:
            E.memo_store(surfaces, materials, code, low, tabulated=True)
            return res
        del res
    keys = E.distinct_wavelengths(last[:, 7])
    E.remember_keys(fp, keys)
    return run(E.lower(surfaces, materials, lambda: keys, code))


def _trace_scattered(surfaces, materials, rays, devs, *, planes, dtype, layout, gather):
    """A torch CUDA bundle split by ray index over ``devs``: each shard is copied to its
    GPU (device-to-device), traced there on that device's current stream, and -- with ``gather`` --
    copied back into one history on the bundle's own device.  Rays are independent, so the result is
    bit-identical to a single-device trace."""
    import torch
    if rays.ndim == 1:
        rays = rays[None, None, :]
    elif rays.ndim == 2:
        rays = rays[None]
    n = rays.shape[1]
    shards = []
    for (a, b), d in zip(shard_bounds(n, len(devs)), devs):
        dev = torch.device("cuda", d)
        shards.append(rays[:, a:b] if dev == rays.device else rays[:, a:b].to(dev, non_blocking=True))
    outs = [trace_surfaces(surfaces, materials, r if r.shape[0] > 1 else r[0], planes=planes, dtype=dtype,
                           layout=layout) for r in shards]
    if not gather:
        return outs
    axis = 2 if layout == "soa" else 1
    shape = list(outs[0].shape)
    shape[axis] = n
    out = E.device_empty(shape, outs[0].dtype, rays.device)
    for (a, b), o in zip(shard_bounds(n, len(devs)), outs):
        out.narrow(axis, a, b - a).copy_(o, non_blocking=True)
    return out


def _trace_segmented(surfaces, materials, rays, *, planes, dtype, devices, layout):
    """A system longer than RTPB_MAX_SURFACES (the 128-bit plane mask of one fused launch) runs as
    consecutive fused segments of at most RTPB_MAX_SURFACES surfaces, each continuing from the previous
    segment's last plane exactly as the reference's surface loop continues (RT:658-659, 3-D histories
    RT:1175-1178).  Segments are traced with float64 storage -- the continuation must not be rounded --
    and the requested planes are assembled (and rounded once, for float32 storage) at the end."""
    on_device = _is_torch_cuda(rays)
    if on_device:
        import torch
        xp_stack, xp_cat = torch.stack, torch.cat
    else:
        rays = np.asarray(rays)
        xp_stack, xp_cat = np.stack, np.concatenate
    if rays.ndim == 1:
        rays = rays[None, None, :]
    elif rays.ndim == 2:
        rays = rays[None]
    if rays.ndim != 3 or rays.shape[-1] != 8:
        raise ValueError(f"rays must have shape (8,), (N, 8) or (k, N, 8); got {tuple(rays.shape)}")
    S = len(surfaces)
    code = _dtype_code(dtype, rays)
    sel = E.resolve_planes(planes, S)
    want = set(sel)
    full = isinstance(planes, str) and planes == "all"
    pieces = {}
    cur = rays[-1]
    if 0 in want:
        pieces[0] = cur.double() if on_device else np.asarray(cur, dtype=np.float64)
    M = C.RTPB_MAX_SURFACES
    for s0 in range(0, S, M):
        s1 = min(S, s0 + M)
        last = 2 * (s1 - s0)
        req = sorted({p - 2 * s0 for p in want if 2 * s0 < p <= 2 * s1} | {last})
        res = trace_surfaces(surfaces[s0:s1], materials[s0:s1 + 1], cur, planes=req, dtype="float64", devices=devices)
        for p, arr in zip(req, res):
            if 2 * s0 + p in want:
                pieces[2 * s0 + p] = arr
        cur = res[-1]
    out = xp_stack([pieces[p] for p in sel])
    if code == C.RTPB_F32:
        out = out.float() if on_device else out.astype(np.float32)
    if full and rays.shape[0] > 1:
        head = rays.to(out.dtype) if on_device else rays.astype(out.dtype)
        out = xp_cat((head, out[1:]))
    if layout == "soa":
        if not on_device:
            raise ValueError("layout='soa' is only available for device (torch CUDA) inputs")
        out = out.transpose(1, 2).contiguous()
    return out


def _resolve_devices(devices):
    if devices is None:
        return None
    if isinstance(devices, str):
        if devices != "all":
            raise ValueError("devices must be None, 'all' or a list of device indices")
        n = C.device_count()
        if n <= 0:
            raise RuntimeError("no GPU visible")
        return list(range(n))
    return [int(d) for d in devices]


class _AxisOnly:
    """Lowering stand-in for a user-geometry surface: the hook kernels read only input_axis."""

    def __init__(self, input_axis):
        self.input_axis = input_axis
        self.normal = input_axis
        self.center = (0.0, 0.0, 0.0)
        self.aperture_rad = np.inf

    @staticmethod
    def _rtpb_kind():
        return C.RTPB_FLAT


def propagate_user_geometry(surface, ray_array, material1, material2, *, devices=None):
    """RefractingSurface.propagate (RT:1160-1234) / ReflectingSurface.propagate (RT:1238-1303) for a
    user Surface subclass that supplies its own get_intersect / get_normal / is_pt_on_surface.

    The three hooks run exactly as the user wrote them (on the history's own array type, NumPy or
    torch); the rest of propagate -- the front-side test, the Snell / reflection step and the NaN
    rules -- runs on the GPU (``rtpb_front_side`` / ``rtpb_interact``).  Hook order and arguments
    follow the reference: get_intersect(last plane, material1), get_normal(unmasked hits),
    is_pt_on_surface(front-side-masked hits)."""
    import torch
    on_device = _is_torch_cuda(ray_array)
    hist = ray_array if on_device else np.asarray(ray_array)
    if hist.ndim == 1:
        hist = hist[None, None, :]
    elif hist.ndim == 2:
        hist = hist[None]
    if hist.ndim != 3 or hist.shape[-1] != 8:
        raise ValueError(f"rays must have shape (8,), (N, 8) or (k, N, 8); got {tuple(hist.shape)}")
    rays = hist[-1]
    n = rays.shape[0]
    if on_device:
        dev = rays.device
    else:
        devs = _resolve_devices(devices)
        dev = torch.device("cuda", devs[0] if devs else torch.cuda.current_device())
    tdt = rays.dtype if (on_device and rays.dtype == torch.float32) else torch.float64
    code = C.RTPB_F32 if tdt == torch.float32 else C.RTPB_F64

    def to_dev(a, cols):
        t = torch.as_tensor(np.asarray(a) if not torch.is_tensor(a) else a)
        t = t.to(device=dev, dtype=tdt).reshape(-1, cols)
        if t.shape[0] != n:
            t = t.expand(n, cols)
        return t.contiguous()

    hits = surface.get_intersect(rays, material1)              # user hook (RT:1181)
    normals = surface.get_normal(hits)                          # user hook (RT:1182), on unmasked hits
    h_d = to_dev(hits, 8)
    n_d = to_dev(normals, 3)
    reflect = isinstance(surface, ReflectingSurface)
    axis = getattr(surface, "input_axis", (0.0, 0.0, 1.0))
    low = E.lower([_AxisOnly(axis)], [material1, material2 if material2 is not None else material1],
                  lambda: E.distinct_wavelengths(h_d[:, 7]), code)
    lib = C.lib()
    stream = torch.cuda.current_stream(dev).cuda_stream
    with E.plan_ref(low) as plan:
        if not reflect:                                         # front-side test (RT:1184-1192)
            r_d = to_dev(rays, 8)
            C.check(lib.rtpb_front_side(plan, dev.index, r_d.data_ptr(), h_d.data_ptr(), n, h_d.data_ptr(),
                                        stream))
        hits_user = h_d if on_device else h_d.cpu().numpy()
        on = surface.is_pt_on_surface(hits_user)                # user hook (RT:1225, 1293)
        on_t = torch.as_tensor(on if torch.is_tensor(on) else np.asarray(on)).to(dev)
        on_d = torch.broadcast_to(on_t.reshape(-1) != 0, (n,)).to(torch.uint8).contiguous()
        out_d = torch.empty_like(h_d)
        C.check(lib.rtpb_interact(plan, dev.index, C.RTPB_REFLECT if reflect else C.RTPB_REFRACT,
                                  h_d.data_ptr(), n_d.data_ptr(), on_d.data_ptr(), n, out_d.data_ptr(), stream))
    new = torch.stack((h_d, out_d))
    if on_device:
        return torch.cat((hist.to(new.dtype), new), dim=0)
    return np.concatenate((hist, new.cpu().numpy()), axis=0)


_CUSTOM = {}       # tuple of surface classes -> per surface: runs its own propagate / geometry hooks (class properties)


class System:
    """An ordered collection of optical surfaces with the materials between them (RT:359-932).

    ``materials`` has len(surfaces) - 1 entries (the media between consecutive surfaces); the
    initial and final media are given to each call (``ray_trace``, paraxial methods)."""

    def __init__(self, surfaces: list, materials: list, names: list = None, surfaces_by_name=None,
                 aperture_stop: Optional[int] = None):
        if len(materials) > 1 and len(materials) != len(surfaces) - 1:
            raise ValueError(f"len(materials) = {len(materials):d} != len(surfaces) - 1 = {len(surfaces) - 1:d}")
        self.surfaces = surfaces
        self.materials = materials
        self.aperture_stop = aperture_stop
        if names is None:
            self.names = [""]
        else:
            self.names = names if isinstance(names, list) else [names]
        if surfaces_by_name is None:
            self.surfaces_by_name = np.zeros(len(surfaces), dtype=int)
        else:
            if len(surfaces_by_name) != len(surfaces):
                raise ValueError("len(surfaces_by_name) must equal len(surfaces)")
            self.surfaces_by_name = np.array(surfaces_by_name).astype(int)

    # ------------------------------------------------------------------ composition (RT:402-482)
    def reverse(self):
        """The same optic traversed the other way (rays typically enter from +z)."""
        flipped = [deepcopy(s) for s in reversed(self.surfaces)]
        for s in flipped:
            s.input_axis *= -1
            s.output_axis *= -1
        return System(flipped, list(reversed(self.materials)))

    def concatenate(self, other, material: Material, distance: Optional[float] = None,
                    axis: Sequence = (0., 0., 1.)):
        """Append a System or Surface after this one, separated by ``material``; with ``distance`` the
        new surfaces are shifted so the first paraxial center sits ``distance`` along ``axis`` after the
        current last one (RT:417-478)."""
        if isinstance(other, System):
            extra = [deepcopy(s) for s in other.surfaces]
            extra_mats = other.materials
            other_stop = other.aperture_stop
            extra_by_name = other.surfaces_by_name
            extra_names = other.names
        elif isinstance(other, Surface):
            extra = [deepcopy(other)]
            extra_mats = []
            other_stop = None
            extra_by_name = np.array([0])
            extra_names = [""]
        else:
            raise TypeError(f"other should be of type System or Surface, but was {type(other)}")
        if distance is not None:
            for ii, s in enumerate(extra):
                if ii == 0:
                    shift = self.surfaces[-1].paraxial_center + distance * np.array(axis) - s.paraxial_center
                else:
                    shift = extra[ii - 1].paraxial_center - other.surfaces[ii - 1].paraxial_center
                s.center += shift
                s.paraxial_center += shift
        by_name = np.concatenate((self.surfaces_by_name, extra_by_name + np.max(self.surfaces_by_name) + 1))
        if self.aperture_stop is not None:
            stop = self.aperture_stop
        elif other_stop is not None:
            stop = other_stop + len(self.surfaces)
        else:
            stop = None
        return System(self.surfaces + extra, self.materials + [material] + extra_mats,
                      names=self.names + extra_names, surfaces_by_name=by_name, aperture_stop=stop)

    def set_aperture_stop(self, surface_index: int):
        self.aperture_stop = surface_index

    # ------------------------------------------------------------------ the hot path (RT:641-661)
    def ray_trace(self, rays, initial_material: Material, final_material: Material, *, planes="all",
                  dtype=None, devices=None, layout="aos", gather=True, out=None):
        """Trace rays through the system; returns the ray history.

        Same contract as the reference: (N, 8) rays -> (2S+1, N, 8) history (plane 0 = input, plane
        2i+1 at surface i, 2i+2 after it), (8,) -> (2S+1, 1, 8), (k, N, 8) -> (k+2S, N, 8).  Computed in
        float64 on the GPU by one fused kernel (systems longer than RTPB_MAX_SURFACES = 63 surfaces by
        consecutive fused segments).  Keyword-only extensions:

        planes   'all' (default) | 'final' | list of plane indices -- store only what is needed
        dtype    None/float64 (reference numerics) | float32 storage of the history (float64 arithmetic;
                 float64 rays are not rounded before the trace)
        devices  None (the bundle's GPU / GPU 0) | 'all' | list of GPU indices: ray-index shards, one per
                 GPU, traced concurrently (NumPy: host threads in the library; torch: device-to-device
                 scatter and gather)
        layout   'aos' (default) | 'soa' (torch inputs only: (planes, 8, N) output)
        gather   torch input with devices: False returns the list of per-device histories (no gather)
        out      torch input on one device: trace into this preallocated history (e.g. history_buffer(...),
                 for repeated traces) and return it

        torch CUDA tensors in -> torch CUDA tensors out (nothing leaves HBM); a list of per-device torch
        shards (e.g. ``get_ray_fan(..., devices=...)``) -> the list of per-device histories."""
        materials = [initial_material] + list(self.materials) + [final_material]
        if len(materials) != len(self.surfaces) + 1:
            raise ValueError("length of materials should be len(surfaces) + 1")
        classes = tuple(map(type, self.surfaces))
        custom = _CUSTOM.get(classes)
        if custom is None:
            if len(_CUSTOM) > 256:
                _CUSTOM.clear()
            custom = _CUSTOM[classes] = [s._rtpb_user_propagate() or s._rtpb_user_geometry() for s in self.surfaces]
        if not any(custom):
            return trace_surfaces(self.surfaces, materials, rays, planes=planes, dtype=dtype, devices=devices,
                                  layout=layout, gather=gather, out=out)
        if out is not None:
            raise ValueError("out= is not available for systems with user-defined surfaces")
        # user surfaces (own propagate, or own geometry hooks): run maximal runs of built-in surfaces
        # as fused GPU traces and hand the growing history to each user surface in between
        # (RT:658-659 order)
        if not (isinstance(planes, str) and planes == "all") or layout != "aos":
            raise ValueError("systems with user-defined surfaces support only planes='all', layout='aos'")
        if _is_shard_list(rays):
            return [self.ray_trace(r, initial_material, final_material, planes=planes, dtype=dtype, layout=layout)
                    for r in rays]
        hist, i, S = rays, 0, len(self.surfaces)
        while i < S:
            if custom[i]:
                s = self.surfaces[i]
                if s._rtpb_user_propagate():
                    hist = s.propagate(hist, materials[i], materials[i + 1])
                else:
                    hist = propagate_user_geometry(s, hist, materials[i], materials[i + 1], devices=devices)
                i += 1
                continue
            j = i
            while j < S and not custom[j]:
                j += 1
            hist = trace_surfaces(self.surfaces[i:j], materials[i:j + 1], hist, dtype=dtype, devices=devices)
            i = j
        return hist

    # ------------------------------------------------------------------ paraxial analysis (RT:484-855)
    def _indices(self, wavelength, initial_material, final_material):
        mats = [initial_material] + list(self.materials) + [final_material]
        return np.array([m.n(wavelength) for m in mats])

    def get_ray_transfer_matrix(self, wavelength: float, initial_material: Material, final_material: Material,
                                axis=None):
        """ABCD matrices: [k] maps the ray at surface 0 to just before surface k (k < S), and [S] to just
        after the last surface (RT:719-752)."""
        ns = self._indices(wavelength, initial_material, final_material)
        S = len(self.surfaces)
        mats = np.zeros((S + 1, 2, 2))
        mats[0] = get_free_space_abcd(0, ns[0])
        for ii in range(1, S + 1):
            surf = self.surfaces[ii - 1].get_ray_transfer_matrix(ns[ii - 1], ns[ii])
            if ii < S:
                gap = np.linalg.norm(self.surfaces[ii].paraxial_center - self.surfaces[ii - 1].paraxial_center)
                step = get_free_space_abcd(gap, ns[ii]).dot(surf)
            else:
                step = surf
            mats[ii] = step.dot(mats[ii - 1])
        return mats

    def get_cardinal_points(self, wavelength: float, initial_material: Material, final_material: Material,
                            axis=None):
        """Focal points, principal points, nodal points and effective focal lengths
        (fp1, fp2, pp1, pp2, np1, np2, efl1, efl2) (RT:754-813)."""
        fwd = self.get_ray_transfer_matrix(wavelength, initial_material, final_material)[-1]
        bwd = self.reverse().get_ray_transfer_matrix(wavelength, final_material, initial_material)[-1]
        n_obj = initial_material.n(wavelength)
        n_img = final_material.n(wavelength)
        first, last = self.surfaces[0], self.surfaces[-1]
        d2 = -fwd[0, 0] / fwd[1, 0] * n_img
        efl2 = -n_img / fwd[1, 0]
        fp2 = last.paraxial_center + d2 * last.output_axis
        pp2 = fp2 - efl2 * last.output_axis
        np2 = last.paraxial_center + (n_img - n_obj * bwd[1, 1]) / bwd[1, 0] * last.output_axis
        d1 = -bwd[0, 0] / bwd[1, 0] * n_obj
        efl1 = -n_obj / bwd[1, 0]
        fp1 = first.paraxial_center - d1 * first.input_axis
        pp1 = fp1 + efl1 * first.input_axis
        np1 = first.paraxial_center - (n_obj - n_img * fwd[1, 1]) / fwd[1, 0] * first.output_axis
        return fp1, fp2, pp1, pp2, np1, np2, efl1, efl2

    def find_paraxial_collimated_distance(self, other, wavelength: float, initial_material: Material,
                                          intermediate_material: Material, final_material: Material, axis=None):
        """Gap to insert between this system and ``other`` so collimated light stays collimated (RT:615-639)."""
        m1 = self.get_ray_transfer_matrix(wavelength, initial_material, intermediate_material)[-1]
        m2 = other.get_ray_transfer_matrix(wavelength, intermediate_material, final_material)[-1]
        return -(m1[0, 0] / m1[1, 0] + m2[1, 1] / m2[1, 0]) * intermediate_material.n(wavelength)

    def seidel_third_order(self, wavelength: float, initial_material: Material, final_material: Material,
                           print_results: bool = False, object_distance: float = 0., object_height: float = 0.,
                           object_angle: float = 0.):
        """Per-surface Seidel sums (spherical, coma, astigmatism, field curvature, distortion) from the
        paraxial marginal and chief rays, Kidger "Fundamentals of Optical Design" eqs. 6.27-6.37
        (RT:484-613).  Requires an aperture stop."""
        if self.aperture_stop is None:
            raise ValueError("aperture_stop was None, but aperture_stop must be provided to "
                             "compute Seidel aberrations")
        ns = self._indices(wavelength, initial_material, final_material)
        rtm = self.get_ray_transfer_matrix(wavelength, initial_material, final_material)
        stop = rtm[self.aperture_stop]
        stop_rad = self.surfaces[self.aperture_stop].aperture_rad
        if np.isinf(object_distance):
            h_chief, u_chief = 0., object_angle
            h_marg, u_marg = stop_rad / stop[0, 0], 0.
        else:
            o2s = stop.dot(get_free_space_abcd(object_distance, ns[0]))
            h_start = 0.
            u_start = stop_rad / o2s[0, 1] / ns[0]
            h_marg = o2s[0, 0] * h_start + o2s[0, 1] * ns[0] * u_start
            u_marg = o2s[1, 0] * h_start + o2s[1, 1] * ns[0] * u_start
            uc_start = -o2s[0, 0] / o2s[0, 1] / ns[0] * object_height
            h_chief = o2s[0, 0] * object_height + o2s[0, 1] * ns[0] * uc_start
            u_chief = o2s[1, 0] * object_height + o2s[1, 1] * ns[0] * uc_start
        start = np.array([[h_marg, h_chief], [ns[0] * u_marg, ns[0] * u_chief]])
        tr = rtm.dot(start)              # (S+1, 2, 2): [surface, (h, n u), (marginal, chief)]
        h, nu = tr[:-1, 0, 0], tr[:-1, 1, 0]
        hb, nub = tr[:-1, 0, 1], tr[:-1, 1, 1]
        n_in, n_out = ns[:-1], ns[1:]
        curv = np.array([1 / s.radius if isinstance(s, SphericalSurface) else 0 for s in self.surfaces])
        A = n_in * h * curv + nu
        Ab = n_in * hb * curv + nub
        d_un = tr[1:, 1, 0] / n_out / n_out - nu / n_in / n_in
        lag = n_in * (hb * nu / n_in - h * nub / n_in)
        ab = np.full((len(self.surfaces), 5), np.nan)
        ab[:, 0] = -A ** 2 * h * d_un
        ab[:, 1] = -A * Ab * h * d_un
        ab[:, 2] = -Ab ** 2 * h * d_un
        ab[:, 3] = -lag ** 2 * curv * (1 / n_out - 1 / n_in)
        ab[:, 4] = (-Ab ** 3 * h * (1 / n_out ** 2 - 1 / n_in ** 2) +
                    hb * Ab * curv * (2 * h * Ab - hb * A) * (1 / n_out - 1 / n_in))
        if print_results:
            print("surface,          h,          u,       hbar,       ubar,   delta(u/n)          A,"
                  "       Abar,   Lag. inv.")
            for ii in range(len(self.surfaces)):
                print(f"{ii:02d}:      {h[ii]:10.6g}, {nu[ii] / ns[ii]:10.6g}, {hb[ii]:10.6g}, "
                      f"{nub[ii] / ns[ii]:10.6g}, {d_un[ii]:10.6g}, {A[ii]:10.6g}, {Ab[ii]:10.6g}, {lag[ii]:10.6g}")
            print("surfaces, spherical,       coma,     astig.,   field curv.,   distortion")
            for ii in range(len(self.surfaces)):
                print(f"{ii:02d}:      " + ", ".join(f"{v:10.6g}" for v in ab[ii]))
            print("sum:     " + ", ".join(f"{v:10.6g}" for v in ab.sum(axis=0)))
        return ab

    def gaussian_paraxial(self, q_in: complex, wavelength: float, initial_material: Material,
                          final_material: Material, print_results: bool = False):
        """Propagate a Gaussian-beam q parameter through the paraxial system (RT:663-717)."""
        S = len(self.surfaces)
        qs = np.zeros(S + 1, dtype=complex)
        qs[0] = q_in
        for ii, s in enumerate(self.surfaces):
            n1 = initial_material.n(wavelength) if ii == 0 else self.materials[ii - 1].n(wavelength)
            if ii < S - 1:
                n2 = self.materials[ii].n(wavelength)
                d = np.linalg.norm(self.surfaces[ii + 1].paraxial_center - s.paraxial_center)
            else:
                n2 = final_material.n(wavelength)
                d = 0.
            abcd = get_free_space_abcd(d, n2).dot(s.get_ray_transfer_matrix(n1, n2))
            qs[ii + 1] = (qs[ii] * abcd[0, 0] + abcd[0, 1]) / (qs[ii] * abcd[1, 0] + abcd[1, 1])
        if print_results:
            for ii, q in enumerate(qs):
                print(f"{ii:02d}: q = {q:.6g}")
        return qs

    def auto_focus(self, wavelength: float, initial_material: Material, final_material: Material,
                   mode: str = "ray-fan"):
        """Focus position: by tracing a tiny fan ('ray-fan') or collimated bundle ('collimated') through
        the system on the GPU and intersecting the outer rays, or paraxially (RT:815-855)."""
        if mode in ("ray-fan", "collimated"):
            if mode == "ray-fan":
                rays = get_ray_fan([0, 0, 0], 1e-9, 3, wavelength)
            else:
                rays = get_collimated_rays([0, 0, 0], 1e-9, 3, wavelength)
            rays = self.ray_trace(rays, initial_material, final_material)
            return intersect_rays(rays[-1, 1], rays[-1, 2])[0]
        if mode == "paraxial-focused":
            return self.get_cardinal_points(wavelength, initial_material, final_material)[1]
        if mode == "paraxial-collimated":
            abcd = self.get_ray_transfer_matrix(wavelength, initial_material, final_material)[-1]
            dx = -abcd[0, 0] / abcd[1, 0] * self.materials[-1].n(wavelength)
            return self.surfaces[-1].paraxial_center[2] + dx * np.sign(self.surfaces[-1].input_axis[2])
        raise ValueError(f"mode must be 'ray-fan', or 'collimated' 'paraxial-focused',"
                         f" or paraxial-collimated' but was '{mode:s}'")

    # ------------------------------------------------------------------ plotting (RT:857-932)
    def plot(self, ray_array=None, phi: float = 0, colors: Optional[list] = None, label: str = None, ax=None,
             show_names: bool = True, fontsize: float = 16, **kwargs):
        """Draw rays (history array (planes, N, 8)) and surfaces in the plane at azimuth ``phi``."""
        import matplotlib.pyplot as plt
        if ax is None:
            figh = plt.figure(**kwargs)
            ax = plt.subplot(1, 1, 1)
        else:
            figh = ax.get_figure()
        if ray_array is not None:
            ray_array = np.asarray(ray_array.cpu() if _is_torch_cuda(ray_array) else ray_array)
            h = ray_array[:, :, 0] * np.cos(phi) + ray_array[:, :, 1] * np.sin(phi)
            label = "" if label is None else label
            if colors is None:
                ax.plot(ray_array[:, :, 2], h, label=label)
            else:
                if len(colors) == 1 and not isinstance(colors, list):
                    colors = [colors] * ray_array.shape[1]
                if len(colors) != ray_array.shape[1]:
                    raise ValueError("len(colors) must equal ray_array.shape[1]")
                for ii in range(ray_array.shape[1]):
                    ax.plot(ray_array[:, ii, 2], h[:, ii], color=colors[ii], label=label if ii == 0 else None)
            ax.set_xlabel("z-position (mm)", fontsize=fontsize)
            ax.set_ylabel("height (mm)", fontsize=fontsize)
        ax.tick_params(axis="x", labelsize=fontsize)
        ax.tick_params(axis="y", labelsize=fontsize)
        for ii, s in enumerate(self.surfaces or []):
            s.draw(ax)
            if show_names and (ii == 0 or self.surfaces_by_name[ii] != self.surfaces_by_name[ii - 1]):
                ax.text(s.paraxial_center[2], s.paraxial_center[0] + 1.1 * s.aperture_rad,
                        self.names[self.surfaces_by_name[ii]], horizontalalignment="center", fontsize=fontsize)
        return figh, ax


class Doublet(System):
    """Cemented achromatic doublet (RT:935-1025).  Radii are given for the crown side facing -z; with
    ``input_collimated=False`` the lens is built flint side first (radii negated)."""

    def __init__(self, material_crown: Optional[Material] = None, material_flint: Optional[Material] = None,
                 radius_crown: Optional[float] = None, radius_flint: Optional[float] = None,
                 radius_interface: Optional[float] = None, thickness_crown: Optional[float] = None,
                 thickness_flint: Optional[float] = None, aperture_radius: float = 25.4,
                 input_collimated: bool = True, names: str = ""):
        if input_collimated:
            mats = [material_crown, material_flint]
            radii = [radius_crown, radius_interface, radius_flint]
            zs = [0, thickness_crown, thickness_crown + thickness_flint]
        else:
            mats = [material_flint, material_crown]
            radii = [-radius_flint, -radius_interface, -radius_crown]
            zs = [0, thickness_flint, thickness_flint + thickness_crown]
        surfs = [FlatSurface([0, 0, z], [0, 0, 1], aperture_rad=aperture_radius) if np.isinf(r)
                 else SphericalSurface.get_on_axis(r, z, aperture_radius) for r, z in zip(radii, zs)]
        self.radius_crown = float(radius_crown)
        self.radius_flint = float(radius_flint)
        self.radius_interface = float(radius_interface)
        self.thickness_crown = float(thickness_crown)
        self.thickness_flint = float(thickness_flint)
        super().__init__(surfs, mats, names=names, surfaces_by_name=None)


# =============================================================================== surfaces
_SURFACE_CLASS_INFO = {}


def _surface_class_info(cls):
    """(own propagate, own geometry hooks, fused-kernel kind class or None) of a Surface class -- class
    properties, computed once per class (they are queried on every trace)."""
    info = _SURFACE_CLASS_INFO.get(cls)
    if info is None:
        owner = cls._rtpb_owner
        user_prop = owner("propagate").__module__ != __name__
        kind_cls = next((c for c in cls.__mro__ if "_RTPB_KIND" in c.__dict__ and c._RTPB_KIND is not None), None)
        if user_prop or not issubclass(cls, (RefractingSurface, ReflectingSurface)) or kind_cls is PerfectLens:
            user_geom = False
        else:
            user_geom = kind_cls is None or any(owner(m).__module__ != __name__ for m in Surface._GEOMETRY[1:])
        info = (user_prop, user_geom, kind_cls)
        _SURFACE_CLASS_INFO[cls] = info
    return info


class Surface:
    """Base optical surface: input/output axes, center, paraxial center, aperture radius (RT:1031-1156)."""

    # every assignment / deletion of an attribute is counted: the drop-in call's lowering memo is valid only while
    # the count is unchanged (_engine.memo_lookup)
    def __setattr__(self, name, value):
        object.__setattr__(self, name, value)
        E.MUTATIONS[0] += 1

    def __delattr__(self, name):
        object.__delattr__(self, name)
        E.MUTATIONS[0] += 1

    def __init__(self, input_axis, output_axis, center, paraxial_center, aperture_rad: float):
        self.input_axis = np.array(input_axis).squeeze().astype(float)
        self.output_axis = np.array(output_axis).squeeze().astype(float)
        self.center = np.array(center).squeeze().astype(float)
        self.paraxial_center = np.array(paraxial_center).squeeze().astype(float)
        self.aperture_rad = aperture_rad

    # lowering hook: the rtpb surface kind, or None for user subclasses the kernel cannot run
    _RTPB_KIND = None
    _GEOMETRY = ("propagate", "get_intersect", "get_normal", "is_pt_on_surface")

    def _rtpb_kind_class(self):
        return _surface_class_info(type(self))[2]

    @classmethod
    def _rtpb_owner(cls, name):
        return next(c for c in cls.__mro__ if name in c.__dict__)

    def _rtpb_user_propagate(self):
        """True for a user subclass that supplies its own ``propagate`` (the reference's plugin point,
        RT:1092-1104, as PerfectLens does): System.ray_trace then runs that code for this surface."""
        return _surface_class_info(type(self))[0]

    def _rtpb_user_geometry(self):
        """True for a user RefractingSurface / ReflectingSurface subclass that keeps the base propagate
        but supplies its own get_intersect / get_normal / is_pt_on_surface (RT:1071-1156): traced by
        propagate_user_geometry (user hooks + GPU Snell/reflection).  PerfectLens subclasses keep the
        lens kernel: PerfectLens.propagate never calls the hooks (RT:1680-1801)."""
        return _surface_class_info(type(self))[1]

    def _rtpb_kind(self):
        kind_cls = self._rtpb_kind_class()
        if kind_cls is None or self._rtpb_user_geometry():
            raise NotImplementedError(
                f"{type(self).__name__} is not one of the fused-kernel surface kinds (FlatSurface, "
                "PlaneMirror, SphericalSurface, PerfectLens); System.ray_trace / propagate trace it "
                "through its own geometry hooks or propagate instead.")
        return kind_cls._RTPB_KIND

    def get_normal(self, pts):
        pass

    def get_intersect(self, rays, material: Material):
        pass

    def propagate(self, ray_array, material1: Material, material2: Material):
        """Propagate rays through this surface alone: appends (at, after) planes to the history
        (RT:1092-1104).  Runs the same fused GPU kernel as System.ray_trace with one surface (user
        geometry hooks: propagate_user_geometry)."""
        if self._rtpb_user_geometry():
            return propagate_user_geometry(self, ray_array, material1, material2)
        return trace_surfaces([self], [material1, material2], ray_array)

    def get_ray_transfer_matrix(self, n1: float, n2: float):
        pass

    def solve_img_eqn(self, s, n1: float, n2: float):
        """Image distance for object distance ``s`` (same sign convention, RT:1115-1138)."""
        mat = self.get_ray_transfer_matrix(n1, n2)
        with np.errstate(divide="ignore"):
            if np.abs(s) > 1e12:
                return np.atleast_1d(-n2 * mat[0, 0] / mat[1, 0])
            return np.atleast_1d(-n2 * (-mat[0, 0] * s / n1 + mat[0, 1]) / np.array(-mat[1, 0] * s / n1 + mat[1, 1]))

    def is_pt_on_surface(self, pts):
        pass

    def draw(self, ax):
        pass


class RefractingSurface(Surface):
    """Surface that refracts by Snell's law (RT:1159-1234); ``propagate`` runs on the GPU."""


class ReflectingSurface(Surface):
    """Surface that reflects (RT:1237-1303); ``propagate`` runs on the GPU."""

    def propagate(self, ray_array, material1: Material, material2: Optional[Material] = None):
        if self._rtpb_user_geometry():
            return propagate_user_geometry(self, ray_array, material1, material2)
        return trace_surfaces([self], [material1, material2 if material2 is not None else material1], ray_array)


def _draw_plane(ax, center, normal, aperture_rad):
    y_hat = np.array([0, 1, 0])
    proj = normal - normal.dot(y_hat) * y_hat
    proj = proj / np.linalg.norm(proj)
    dv = np.cross(proj, y_hat)
    if np.isinf(aperture_rad):
        pts = center[None, :] + np.array([0, 1])[:, None] * dv[None, :]
        ax.axline(pts[0, (2, 0)], xy2=pts[1, (2, 0)], color="k")
        return
    ts = np.linspace(-aperture_rad, aperture_rad, 101)
    pts = center[None, :] + ts[:, None] * dv[None, :]
    ax.plot(pts[:, 2], pts[:, 0], "k")


def _on_plane(pts, center, normal, aperture_rad):
    pts = np.atleast_2d(pts)
    rel = pts[..., 0:3] - center
    return (np.abs(np.sum(rel * normal, axis=-1)) < 1e-12) & (np.linalg.norm(rel, axis=-1) <= aperture_rad)


class FlatSurface(RefractingSurface):
    """Plane {(p - center).normal = 0}; the normal points along the direction of travel (RT:1306-1374)."""
    _RTPB_KIND = C.RTPB_FLAT

    def __init__(self, center, normal, aperture_rad: float):
        self.normal = np.array(normal).squeeze()
        super().__init__(normal, normal, center, center, aperture_rad)

    def get_normal(self, pts):
        return np.tile(np.atleast_2d(self.normal), (np.atleast_2d(pts).shape[0], 1))

    def get_intersect(self, rays, material: Material):
        return propagate_ray2plane(rays, self.normal, self.center, material, exclude_backward_propagation=True)[0]

    def is_pt_on_surface(self, pts):
        return _on_plane(pts, self.center, self.normal, self.aperture_rad)

    def get_ray_transfer_matrix(self, n1=None, n2=None):
        return np.array([[1, 0], [0, 1]])

    def draw(self, ax):
        _draw_plane(ax, self.center, self.normal, self.aperture_rad)


class PlaneMirror(ReflectingSurface):
    """Plane mirror; the normal points along the direction of travel (RT:1377-1432)."""
    _RTPB_KIND = C.RTPB_PLANE_MIRROR

    def __init__(self, center, normal, aperture_rad):
        self.normal = np.array(normal).squeeze()
        super().__init__(normal, normal, center, center, aperture_rad)

    def get_normal(self, pts):
        return np.tile(np.atleast_2d(self.normal), (np.atleast_2d(pts).shape[0], 1))

    def get_intersect(self, rays, material: Material):
        out, ts = propagate_ray2plane(rays, self.normal, self.center, material)
        out[ts < 0] = np.nan
        return out

    def is_pt_on_surface(self, pts):
        return _on_plane(pts, self.center, self.normal, self.aperture_rad)

    def get_ray_transfer_matrix(self, n1: float, n2: float):
        return np.array([[1, 0], [0, -1]])

    def draw(self, ax):
        _draw_plane(ax, self.center, self.normal, self.aperture_rad)


class SphericalSurface(RefractingSurface):
    """Sphere of signed radius ``radius`` about ``center`` (RT:1435-1555).  Positive radius = convex as
    seen from -z; the aperture is measured from the line through the origin along ``input_axis``."""
    _RTPB_KIND = C.RTPB_SPHERE

    def __init__(self, radius, center, aperture_rad, input_axis=(0, 0, 1)):
        self.radius = radius
        paraxial_center = np.array(center).squeeze() - self.radius * np.array(input_axis).squeeze()
        super().__init__(input_axis, input_axis, center, paraxial_center, aperture_rad)

    @classmethod
    def get_on_axis(cls, radius: float, surface_z_position: float, aperture_rad: float):
        """Sphere whose vertex sits on the z axis at ``surface_z_position``."""
        return cls(radius, [0, 0, surface_z_position + radius], aperture_rad, (0, 0, 1))

    def get_normal(self, pts):
        """Outward normal for radius > 0, inward for radius < 0."""
        return (np.atleast_2d(pts)[:, :3] - self.center[None, :]) / self.radius

    def get_intersect(self, rays, material: Material):
        rays = np.atleast_2d(rays)
        p, d = rays[:, 0:3], rays[:, 3:6]
        rel = p - self.center
        B = 2 * np.sum(d * rel, axis=1)
        Cq = np.sum(rel ** 2, axis=1) - self.radius ** 2
        with np.errstate(invalid="ignore"):
            roots = np.stack((0.5 * (-B + np.sqrt(B ** 2 - 4 * Cq)), 0.5 * (-B - np.sqrt(B ** 2 - 4 * Cq))), axis=1)
            roots[roots < 0] = np.inf
        t = np.min(roots, axis=1)
        t[t == np.inf] = np.nan
        pts = p + d * t[:, None]
        out = np.concatenate((pts, d, rays[:, 6:8]), axis=1)
        out[:, 6] = rays[:, 6] + np.linalg.norm(pts - p, axis=1) * 2 * np.pi / rays[:, 7] * material.n(rays[:, 7])
        return out

    def is_pt_on_surface(self, pts):
        pts = np.atleast_2d(pts)
        dist = np.linalg.norm(pts[..., 0:3] - self.center, axis=-1)
        ortho = pts[..., :3] - np.sum(pts[..., :3] * self.input_axis, axis=-1)[..., None] * self.input_axis
        return (np.abs(dist - abs(self.radius)) < 1e-12) & (np.linalg.norm(ortho, axis=-1) <= self.aperture_rad)

    def get_ray_transfer_matrix(self, n1: float, n2: float):
        sgn = np.sign(np.dot(self.center - self.paraxial_center, self.input_axis))
        with np.errstate(divide="ignore"):
            f = sgn * np.abs(self.radius) / np.array(n2 - n1)
        return np.array([[1, 0], [-1 / f, 1]])

    def draw(self, ax):
        theta_max = np.arcsin(self.aperture_rad / np.abs(self.radius))
        th = np.linspace(-theta_max, theta_max, 101)
        ax.plot(self.center[2] - self.radius * np.cos(th), self.center[0] - self.radius * np.sin(th), "k")


class PerfectLens(RefractingSurface):
    """Ideal (aberration-free, Abbe-sine) lens of focal length f at ``center`` (RT:1558-1821).

    Front/back focal planes sit n1 f before and n2 f after the lens; a ray (h, sin t1) in the front
    focal plane maps to (n1 f sin t1, -h / (f n2)) in the back focal plane; rays steeper than
    ``alpha`` on either side are clipped (NaN).  The output planes are the rays just before and just
    after the lens plane; phases make a plane wave focus in phase."""
    _RTPB_KIND = C.RTPB_PERFECT_LENS

    def __init__(self, focal_len: float, center, normal, alpha: float):
        self.focal_len = focal_len
        self.alpha = alpha
        self.normal = np.array(normal).squeeze()
        super().__init__(normal, normal, center, center, focal_len * np.sin(self.alpha))

    def get_intersect(self, rays, material: Material):
        out, ts = propagate_ray2plane(rays, self.normal, self.center, material)
        with np.errstate(invalid="ignore"):
            out[ts < 0] = np.nan
        return out

    def is_pt_on_surface(self, pts):
        pts = np.atleast_2d(pts)
        return np.abs(np.sum((pts[:, :3] - self.center) * self.normal, axis=1)) < 1e-12

    def propagate(self, rays, material1: Material, material2: Material):
        return trace_surfaces([self], [material1, material2], rays)

    def get_ray_transfer_matrix(self, n1: float, n2: float):
        return np.array([[1, 0], [-1 / self.focal_len, 1]])

    def draw(self, ax):
        _draw_plane(ax, self.center, self.normal, self.aperture_rad)
