"""Device-side analysis of traced bundles: spot statistics per (field, wavelength)
group and a chunked spot-diagram sweep that never leaves HBM (BASELINE configs[4] / C5 scale).

The reference computes spot diagrams in user scripts with NumPy on the full host history; here the
fans are generated on the GPU (``rtpb_ray_fan_tables``), traced with only the final plane stored, and reduced
on the GPU with a deterministic fixed-order reduction (``rtpb_spot_stats``).
"""
import time

import numpy as np

from . import _capi as C
from . import _engine as E

STAT_NAMES = ("count", "sum_x", "sum_y", "sum_z", "sum_xx", "sum_yy", "sum_xy")


def spot_stats_raw(plane, group_size, stream=None):
    """Per-group sums (n_groups, 7) of a torch CUDA (N, 8) plane, N = n_groups * group_size."""
    import torch
    n = plane.shape[0]
    if n % group_size:
        raise ValueError("plane length must be a multiple of group_size")
    ngroups = n // group_size
    plane = plane.contiguous()
    tiles = -(-group_size // 256)
    ws = torch.empty(ngroups * tiles * 7, dtype=torch.float64, device=plane.device)
    stats = torch.empty((ngroups, 7), dtype=torch.float64, device=plane.device)
    if stream is None:
        stream = torch.cuda.current_stream(plane.device).cuda_stream
    C.check(C.lib().rtpb_spot_stats(plane.device.index or 0,
                                    C.RTPB_F64 if plane.dtype == torch.float64 else C.RTPB_F32,
                                    plane.data_ptr(), group_size, ngroups, ws.data_ptr(), ws.numel(),
                                    stats.data_ptr(), stream))
    return stats


def summarize(raw):
    """count, centroid (x, y, z) and RMS spot radius about the centroid from the raw sums (kept as
    "raw": count, sum x, y, z, x^2, y^2, xy per group, reduced in the kernels' fixed order)."""
    raw = np.asarray(raw, dtype=np.float64)
    n = raw[..., 0]
    with np.errstate(invalid="ignore", divide="ignore"):
        cx, cy, cz = raw[..., 1] / n, raw[..., 2] / n, raw[..., 3] / n
        var = raw[..., 4] / n - cx * cx + raw[..., 5] / n - cy * cy
    return {"count": n, "centroid": np.stack((cx, cy, cz), axis=-1), "rms_radius": np.sqrt(np.maximum(var, 0.0)),
            "raw": raw}


def spot_stats(plane, group_size):
    """Spot summary per contiguous group of ``group_size`` rays of a torch CUDA (N, 8) plane."""
    return summarize(spot_stats_raw(plane, group_size).cpu().numpy())


def spot_sweep(system, initial_material, final_material, field_points, wavelengths, theta_max, n_thetas, nphis=1,
               center_ray=(0, 0, 1), device="cuda:0", dtype="float64", groups_per_batch=None, fused=True,
               devices=None):
    """Spot diagrams for every (field point, wavelength): a ``get_ray_fan(field, theta_max, n_thetas,
    wavelength, nphis)`` bundle per group, generated, traced (final plane only) and reduced on the GPU.

    ``fused=True`` (default) runs generation, trace and reduction as ONE kernel per batch of groups
    (``rtpb_spot_sweep``: no rays touch HBM); ``fused=False`` runs the three steps separately through
    HBM buffers (``rtpb_ray_fan_tables`` -> ``rtpb_trace`` planes='final' -> ``rtpb_spot_stats``).  Both
    give bit-identical statistics.  ``devices`` (fused only): the (field, wavelength) groups are split into
    contiguous ranges, one per GPU, swept concurrently from this thread (per-device kernel times in the
    timing dict).  Returns (summary dict with arrays shaped (n_fields, n_wavelengths, ...), timing dict)."""
    import torch
    dev = torch.device(device)
    tdt = torch.float64 if dtype in ("float64", np.float64) else torch.float32
    code = C.RTPB_F64 if tdt == torch.float64 else C.RTPB_F32
    if np.linalg.norm(np.asarray(center_ray, dtype=float)) != 1:
        raise ValueError("center_ray must be a unit vector")
    field_points = np.atleast_2d(np.asarray(field_points, dtype=float))
    wavelengths = np.atleast_1d(np.asarray(wavelengths, dtype=float))
    G = field_points.shape[0] * wavelengths.size
    per = n_thetas * nphis
    mats = [initial_material] + list(system.materials) + [final_material]
    # tabulated materials are lowered at the wavelengths the kernels see: the group's wavelength rounded to the
    # storage type (a float32 sweep's rays carry float32 wavelengths, and the table lookup matches exactly)
    keys = wavelengths if tdt == torch.float64 else wavelengths.astype(np.float32).astype(np.float64)
    low = E.lower(system.surfaces, mats, lambda: np.unique(keys), code)
    S = len(system.surfaces)
    if fused:
        devs = [dev] if devices is None else [torch.device("cuda", int(d)) for d in devices]
        return _spot_sweep_fused(low, S, field_points, wavelengths, theta_max, n_thetas, nphis, center_ray, devs,
                                 groups_per_batch)
    if devices is not None:
        raise ValueError("devices= needs the fused sweep")
    if groups_per_batch is None:
        groups_per_batch = max(1, min(G, (1 << 27) // per))     # ~128M rays in flight
    sel = E.resolve_planes("final", len(system.surfaces))
    rays = torch.empty((groups_per_batch * per, 8), dtype=tdt, device=dev)
    out = torch.empty((1, groups_per_batch * per, 8), dtype=tdt, device=dev)
    raw = np.zeros((G, 7))
    jobs = [(f, w) for f in range(field_points.shape[0]) for w in range(wavelengths.size)]
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for b0 in range(0, G, groups_per_batch):
        batch = jobs[b0:b0 + groups_per_batch]
        for k, (f, w) in enumerate(batch):       # generate each fan in place in the batch buffer
            _fan_into(rays[k * per:(k + 1) * per], field_points[f], theta_max, n_thetas, wavelengths[w], nphis,
                      center_ray, code)
        m = len(batch) * per
        E.trace_device(low, rays[:m], sel, out=out[:, :m])
        raw[b0:b0 + len(batch)] = spot_stats_raw(out[0, :m], per).cpu().numpy()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    summ = summarize(raw.reshape(field_points.shape[0], wavelengths.size, 7))
    return summ, {"seconds": dt, "rays": G * per, "ray_surface_per_s": G * per * S / dt}


def _spot_sweep_fused(low, S, field_points, wavelengths, theta_max, n_thetas, nphis, center_ray, devs,
                      groups_per_batch):
    import torch
    from .raytrace import _fan_tables, shard_bounds
    c = np.array(center_ray)
    enx, eny, tcs, pcs = _fan_tables(float(theta_max), int(n_thetas), int(nphis), tuple(c.tolist()), c.dtype.str)
    nf, nw = field_points.shape[0], wavelengths.size
    params = np.empty((nf * nw, 4))
    params[:, 0:3] = np.repeat(field_points, nw, axis=0)          # group = field * nw + wavelength
    params[:, 3] = np.tile(wavelengths, nf)
    G = params.shape[0]
    per = n_thetas * nphis
    tiles = -(-per // 256)
    if groups_per_batch is None:
        groups_per_batch = max(1, min(G, 65535, (1 << 26) // (tiles * 7)))   # workspace <= 512 MB
        # whole field points per batch: a field point's groups share each ray's generation and first surface
        # (the kernel's bundle rows), so batches do not split them
        if groups_per_batch >= nw:
            groups_per_batch -= groups_per_batch % nw
    vec = [np.ascontiguousarray(np.asarray(v, dtype=np.float64).ravel()) for v in (c, enx, eny)]
    # one contiguous range of groups per device -- whole field points when there are enough of them (see
    # groups_per_batch); per device: workspace, statistics, its current stream
    if nf >= len(devs):
        bounds = [(f0 * nw, f1 * nw) for f0, f1 in shard_bounds(nf, len(devs))]
    else:
        bounds = shard_bounds(G, len(devs))
    work = []
    for (g0, g1), dev in zip(bounds, devs):
        ws = torch.empty(groups_per_batch * tiles * 7, dtype=torch.float64, device=dev)
        stats = torch.empty((max(g1 - g0, 1), 7), dtype=torch.float64, device=dev)
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        work.append((dev, g0, g1, ws, stats, ev, torch.cuda.current_stream(dev)))
    for dev in devs:
        torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    with E.plan_ref(low) as plan:
        for dev, g0, g1, ws, stats, ev, st in work:
            ev[0].record(st)
        # batches issued round-robin over the devices: every launch is asynchronous, so they run concurrently
        nb = max(-(-(g1 - g0) // groups_per_batch) for _, g0, g1, *_ in work)
        for k in range(nb):
            for dev, g0, g1, ws, stats, ev, st in work:
                b0 = g0 + k * groups_per_batch
                b1 = min(g1, b0 + groups_per_batch)
                if b0 >= b1:
                    continue
                gp = np.ascontiguousarray(params[b0:b1])
                C.check(C.lib().rtpb_spot_sweep(plan, dev.index or 0, b1 - b0, gp.ctypes.data, int(n_thetas),
                                                int(nphis), vec[0].ctypes.data, vec[1].ctypes.data,
                                                vec[2].ctypes.data, tcs.ctypes.data, pcs.ctypes.data, ws.data_ptr(),
                                                ws.numel(), stats[b0 - g0:b1 - g0].data_ptr(), st.cuda_stream))
        for dev, g0, g1, ws, stats, ev, st in work:
            ev[1].record(st)
        raw = np.concatenate([stats[:g1 - g0].cpu().numpy() for _, g0, g1, _, stats, _, _ in work])
    dt = time.perf_counter() - t0
    per_dev = []
    for dev, g0, g1, ws, stats, ev, st in work:
        ms = ev[0].elapsed_time(ev[1])
        # HBM bytes of the fused sweep: the per-tile partial sums written and read back (the rays never
        # leave the registers)
        nbytes = (g1 - g0) * tiles * 7 * 8 * 2 + (g1 - g0) * 7 * 8
        per_dev.append({"device": dev.index or 0, "groups": g1 - g0, "rays": (g1 - g0) * per, "kernel_ms": ms,
                        "ray_surface_per_s": (g1 - g0) * per * S / (ms * 1e-3) if ms > 0 else None,
                        "hbm_bytes": nbytes, "hbm_GBps": nbytes / (ms * 1e-3) / 1e9 if ms > 0 else None})
    summ = summarize(raw.reshape(nf, nw, 7))
    return summ, {"seconds": dt, "rays": G * per, "ray_surface_per_s": G * per * S / dt, "per_device": per_dev}


def _fan_into(buf, pt, theta_max, n_thetas, wavelength, nphis, center_ray, code):
    from .raytrace import fan_into
    fan_into(buf, pt, theta_max, n_thetas, wavelength, nphis, center_ray)


class GridInterpolator:
    """``scipy.interpolate.griddata(points, values, grid, method='linear')`` evaluated on the GPU.

    The Delaunay triangulation is scipy's own (``scipy.spatial.Delaunay``, host, the same call
    LinearNDInterpolator makes); a uniform cell index of triangle bounding boxes is built once, and
    ``rtpb_grid_interpolate`` locates and interpolates every grid point with scipy's barycentric
    arithmetic.  Values for points strictly inside a triangle are bit-identical to scipy's; on a shared
    edge (within scipy's eps) the first listed triangle is used, which can differ from scipy's walk by a
    rounding.  ``set_values`` swaps the vertex values (the PSF loop re-uses one triangulation while
    only the phases change)."""

    def __init__(self, points, device="cuda:0"):
        import torch
        from scipy.spatial import Delaunay
        self.dev = torch.device(device)
        self.points = np.ascontiguousarray(points, dtype=np.float64)
        tri = Delaunay(self.points)
        simp = np.ascontiguousarray(tri.simplices, dtype=np.int32)
        v = self.points[simp]                                       # (n_tri, 3, 2)
        lo, hi = v.min(axis=1), v.max(axis=1)
        span = float(max(np.ptp(self.points[:, 0]), np.ptp(self.points[:, 1]), 1e-300))
        lo, hi = lo - 1e-9 * span, hi + 1e-9 * span                 # scipy accepts points within eps
        x0, y0 = lo.min(axis=0)
        nt = simp.shape[0]
        ncell = max(1, int(np.sqrt(2 * nt)))
        cw = max((hi[:, 0].max() - x0) / ncell, 1e-300) * (1 + 1e-12)
        ch = max((hi[:, 1].max() - y0) / ncell, 1e-300) * (1 + 1e-12)
        cx0 = np.clip(((lo[:, 0] - x0) / cw).astype(np.int64), 0, ncell - 1)
        cx1 = np.clip(((hi[:, 0] - x0) / cw).astype(np.int64), 0, ncell - 1)
        cy0 = np.clip(((lo[:, 1] - y0) / ch).astype(np.int64), 0, ncell - 1)
        cy1 = np.clip(((hi[:, 1] - y0) / ch).astype(np.int64), 0, ncell - 1)
        nxs, nys = cx1 - cx0 + 1, cy1 - cy0 + 1
        cnt = nxs * nys
        tri_id = np.repeat(np.arange(nt, dtype=np.int64), cnt)
        local = np.arange(cnt.sum()) - np.repeat(np.cumsum(cnt) - cnt, cnt)
        cx = np.repeat(cx0, cnt) + local % np.repeat(nxs, cnt)
        cy = np.repeat(cy0, cnt) + local // np.repeat(nxs, cnt)
        cell = cy * ncell + cx
        order = np.lexsort((tri_id, cell))                        # by cell, then triangle index
        cell, tri_id = cell[order], tri_id[order]
        start = np.searchsorted(cell, np.arange(ncell * ncell + 1)).astype(np.int32)
        t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(self.dev, dtype=dt)  # noqa: E731
        self._transform = t(tri.transform.reshape(nt, 6), torch.float64)
        self._simplices = t(simp, torch.int32)
        self._start = t(start, torch.int32)
        self._cells = t(tri_id.astype(np.int32), torch.int32)
        self._values = torch.zeros(self.points.shape[0], dtype=torch.float64, device=self.dev)
        self.desc = C.Triangulation(nt, self._transform.data_ptr(), self._simplices.data_ptr(),
                                    self._values.data_ptr(), ncell, ncell, float(x0), float(y0), float(cw),
                                    float(ch), self._start.data_ptr(), self._cells.data_ptr())

    def set_values(self, values):
        import torch
        self._values.copy_(torch.as_tensor(np.ascontiguousarray(values, dtype=np.float64)))
        return self

    def __call__(self, xs, ys, radius=None, phase=True):
        """Interpolate on meshgrid(xs, ys) -> torch (len(ys), len(xs)) phase (NaN outside the hull);
        with ``radius``, also the pupil field exp(i*phase) (0 outside ``radius`` or where undefined)."""
        import torch
        gx = torch.as_tensor(np.ascontiguousarray(xs, dtype=np.float64)).to(self.dev)
        gy = torch.as_tensor(np.ascontiguousarray(ys, dtype=np.float64)).to(self.dev)
        nx, ny = gx.numel(), gy.numel()
        ph = torch.empty((ny, nx), dtype=torch.float64, device=self.dev) if phase else None
        fld = torch.empty((ny, nx), dtype=torch.complex128, device=self.dev) if radius is not None else None
        C.check(C.lib().rtpb_grid_interpolate(self.dev.index or 0, C.ctypes.byref(self.desc), gx.data_ptr(), nx,
                                              gy.data_ptr(), ny, float(radius) if radius is not None else 0.0,
                                              ph.data_ptr() if ph is not None else None,
                                              fld.data_ptr() if fld is not None else None,
                                              torch.cuda.current_stream(self.dev).cuda_stream))
        return ph, fld


def griddata_linear(points, values, xs, ys, device="cuda:0"):
    """scipy.interpolate.griddata(points, values, meshgrid(xs, ys), method='linear') on the GPU
    (torch (len(ys), len(xs)); see :class:`GridInterpolator`)."""
    return GridInterpolator(points, device).set_values(values)(xs, ys)[0]


def pupil_psf(system, initial_material, final_material, source_points, wavelength, theta_max, n_thetas, nphis,
              pupil_plane, pupil_radius, grid_step, grid_extent=3.0, device="cuda:0", interp="gpu", as_numpy=True):
    """Point-spread functions from pupil phases (the pipeline of
    scripts/2022_02_06_perfect_imaging_system_psf.py:73-105).

    For every source point: a ``get_ray_fan(src, theta_max, n_thetas, wavelength, nphis)`` is generated
    and traced on the GPU (only history plane ``pupil_plane`` is stored); the pupil phase (column 6)
    is interpolated onto a square grid of pitch ``grid_step`` spanning +-grid_extent*pupil_radius with
    ``scipy.interpolate.griddata`` (linear, Delaunay -- as the script; host), masked outside
    ``pupil_radius`` and where undefined, and Fourier transformed on the GPU (torch.fft = hipFFT):
    E_out = fftshift(fft2(ifftshift(exp(i phi)))).  Returns (psf |E_out|^2 normalised to the stack
    maximum, pupil field, grid coordinates).

    ``interp='gpu'`` (default) interpolates and forms the pupil field on the GPU
    (:class:`GridInterpolator`, scipy's triangulation and arithmetic; the triangulation is re-used while
    the pupil positions stay the same); ``interp='host'`` calls scipy's griddata as the script does.
    ``as_numpy=False`` returns the psf and pupil stacks as torch CUDA tensors (no host copies)."""
    import torch
    from scipy.interpolate import griddata
    from .raytrace import get_ray_fan
    dev = torch.device(device)
    src = np.atleast_2d(np.asarray(source_points, dtype=float))
    nxy = int(2 * (grid_extent * pupil_radius // grid_step) + 1)
    xs = grid_step * np.arange(nxy)
    xs -= np.mean(xs)
    xx, yy = np.meshgrid(xs, xs)
    interp_pts = np.stack((xx.ravel(), yy.ravel()), axis=1)
    outside = np.sqrt(xx ** 2 + yy ** 2) > pupil_radius
    if interp == "gpu":
        pt = torch.empty((len(src), nxy, nxy), dtype=torch.complex128, device=dev)
        gi, key = None, None
        for ii, p in enumerate(src):
            rays = get_ray_fan(p, theta_max, n_thetas, wavelength, nphis=nphis, device=dev)
            plane = system.ray_trace(rays, initial_material, final_material, planes=[pupil_plane])[0]
            h = plane.cpu().numpy()
            ok = ~np.isnan(h[:, 0]) & ~np.isnan(h[:, 1])
            pts = np.ascontiguousarray(h[ok, :2])
            if gi is None or key != pts.tobytes():                  # same pupil positions: same triangulation
                gi, key = GridInterpolator(pts, dev), pts.tobytes()
            _, pt[ii] = gi.set_values(h[ok, 6])(xs, xs, radius=pupil_radius, phase=False)
        pupil = pt.cpu().numpy() if as_numpy else pt
    else:
        pupil = np.zeros((len(src), nxy, nxy), dtype=complex)
        for ii, p in enumerate(src):
            rays = get_ray_fan(p, theta_max, n_thetas, wavelength, nphis=nphis, device=dev)
            plane = system.ray_trace(rays, initial_material, final_material, planes=[pupil_plane])[0]
            h = plane.cpu().numpy()
            ok = ~np.isnan(h[:, 0]) & ~np.isnan(h[:, 1])
            phis = griddata(h[ok, :2], h[ok, 6], interp_pts).reshape(xx.shape)
            e = np.exp(1j * phis)
            e[outside] = 0
            e[np.isnan(phis)] = 0
            pupil[ii] = e
        pt = torch.from_numpy(pupil).to(dev)
    out = torch.fft.fftshift(torch.fft.fft2(torch.fft.ifftshift(pt, dim=(-2, -1))), dim=(-2, -1))
    psf = out.abs() ** 2
    psf = psf / psf.max()
    return (psf.cpu().numpy() if as_numpy else psf), pupil, xs
