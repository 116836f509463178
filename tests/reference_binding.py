"""The reference-side binding a maintainer of QI2lab/ray_trace_pb would add, as a
tested file.  It uses nothing of this repository but librtpb.so and its C ABI (include/rtpb.h): it
lowers the reference's own objects -- duck-typed on the reference's class names and attributes, so it
runs on the reference's ``raytrace`` package and on this repository's drop-in alike -- and replaces the
surface loop of ``System.ray_trace`` (RT:641-661, the loop at RT:658-659).

    import reference_binding
    ray_trace_gpu = reference_binding.make_ray_trace(raytrace.raytrace, raytrace.materials, "librtpb.so")
    raytrace.raytrace.System.ray_trace = ray_trace_gpu          # the one-line switch

Semantics kept from the reference:
  * input ranks (RT:1175-1178): (8,) -> (1, 1, 8), (N, 8) -> (1, N, 8), (k, N, 8) is an existing history
    that is extended by 2S planes; the return is always float64;
  * Surface subclasses: a subclass that overrides none of get_intersect / get_normal / is_pt_on_surface /
    propagate lowers as its built-in base class; anything else (a user geometry or propagate) runs through
    the reference's own Python loop for the whole call;
  * Material subclasses: Constant and Sellmeier (Material.n, incl. Vacuum) are evaluated by the kernel;
    any other n() (Ebaf11, user classes) is evaluated by the material itself at the bundle's distinct
    wavelengths and handed over as a (wavelength, n) table;
  * systems longer than RTPB_MAX_SURFACES run as chained launches, each extending the history exactly as
    the reference's loop would.
This file is TEST INFRASTRUCTURE of this repository: tests/test_gpu_binding.py runs it on the GPU
against the reference's golden histories.
"""
import ctypes

import numpy as np

RTPB_MAX_SURFACES = 63
_KINDS = (("PerfectLens", 3), ("PlaneMirror", 2), ("SphericalSurface", 1), ("FlatSurface", 0))
_HOOKS = ("get_intersect", "get_normal", "is_pt_on_surface", "propagate")


class _Surf(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("center", ctypes.c_double * 3), ("normal", ctypes.c_double * 3),
                ("input_axis", ctypes.c_double * 3), ("radius", ctypes.c_double),
                ("radius_sq", ctypes.c_double), ("aperture", ctypes.c_double),
                ("focal_len", ctypes.c_double), ("sin_alpha", ctypes.c_double), ("on_tol", ctypes.c_double)]


class _Mat(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("table_len", ctypes.c_int32), ("c", ctypes.c_double * 6),
                ("table", ctypes.POINTER(ctypes.c_double))]


def _builtin_kind(rt, s):
    """Surface kind code, or None when the class (or a subclass) brings its own geometry/propagate."""
    for name, code in _KINDS:
        base = getattr(rt, name)
        if isinstance(s, base):
            own = any(getattr(type(s), h) is not getattr(base, h) for h in _HOOKS)
            return None if own else code
    return None


def lower_surface(s, kind):
    """rtpb_surface of a reference surface object of built-in ``kind`` (RT:1035-1069 attributes)."""
    d = _Surf()
    d.kind = kind
    d.center[:] = np.asarray(s.center, dtype=float).ravel()
    d.input_axis[:] = np.asarray(s.input_axis, dtype=float).ravel()
    d.normal[:] = np.asarray(getattr(s, "normal", s.input_axis), dtype=float).ravel()
    d.aperture = float(s.aperture_rad)
    d.on_tol = 1e-12                                    # RT:1343, 1408, 1528
    if kind == 1:
        d.radius, d.radius_sq = float(s.radius), float(s.radius ** 2)          # RT:1499
    if kind == 3:
        d.focal_len, d.sin_alpha = float(s.focal_len), float(np.sin(s.alpha))  # RT:1758
    return d


def lower_material(mat, m, wl):
    """rtpb_material of a reference material (``mat``: raytrace.materials); ``wl``: the bundle's distinct
    wavelengths, the keys of a table for any n() the kernel does not evaluate itself."""
    d = _Mat()
    if type(m).n is mat.Constant.n:
        d.kind, d.c[0] = 0, float(m._n)
    elif type(m).n is mat.Material.n:                   # Sellmeier (MAT:39-51), Vacuum
        d.kind = 1
        d.c[:] = [float(v) for v in (m.b1, m.b2, m.b3, m.c1, m.c2, m.c3)]
    else:                                               # Ebaf11 or a user n(): its own values
        d._tab = np.ascontiguousarray(np.stack((wl, np.broadcast_to(np.asarray(m.n(wl), dtype=float), wl.shape)),
                                               axis=1))
        d.kind, d.table_len = 3, wl.size
        d.table = d._tab.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    return d


def lower_system(rt, mat, surfaces, materials, wl):
    """(rtpb_surface array, rtpb_material array, keep-alive list) of built-in surfaces and their S+1 materials."""
    kinds = [_builtin_kind(rt, s) for s in surfaces]
    if any(k is None for k in kinds):
        raise ValueError("user surface geometry: not lowerable")
    S = len(surfaces)
    surf = (_Surf * max(S, 1))(*[lower_surface(s, k) for s, k in zip(surfaces, kinds)])
    keep = [lower_material(mat, m, wl) for m in materials]   # keeps the table arrays alive
    return surf, (_Mat * (S + 1))(*keep), keep


def make_ray_trace(rt, mat, lib_path):
    """System.ray_trace replacement bound to librtpb.so at ``lib_path`` (``rt`` / ``mat``: the
    reference's raytrace.raytrace / raytrace.materials modules)."""
    lib = ctypes.CDLL(lib_path)
    lib.rtpb_last_error.restype = ctypes.c_char_p
    lib.rtpb_plan_create.argtypes = [ctypes.POINTER(_Surf), ctypes.c_int32, ctypes.POINTER(_Mat), ctypes.c_int32,
                                     ctypes.c_int32, ctypes.POINTER(ctypes.c_void_p)]
    lib.rtpb_plan_destroy.argtypes = [ctypes.c_void_p]
    lib.rtpb_trace_host.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p,
                                    ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(ctypes.c_int32), ctypes.c_int32]
    python_loop = rt.System.ray_trace

    def trace_segment(surfaces, kinds, materials, rays2d):
        S = len(surfaces)
        wl = np.unique(rays2d[:, 7])
        surf = (_Surf * S)(*[lower_surface(s, k) for s, k in zip(surfaces, kinds)])
        keep = [lower_material(mat, m, wl) for m in materials]   # keeps the table arrays alive
        mats = (_Mat * (S + 1))(*keep)
        plan = ctypes.c_void_p()
        if lib.rtpb_plan_create(surf, S, mats, S + 1, 0, ctypes.byref(plan)) != 0:
            raise RuntimeError(lib.rtpb_last_error().decode())
        out = np.empty((2 * S + 1, rays2d.shape[0], 8))
        mask = (1 << (2 * S + 1)) - 1
        rc = lib.rtpb_trace_host(plan, rays2d.ctypes.data, 0, rays2d.shape[0], out.ctypes.data, mask & (2 ** 64 - 1),
                                 mask >> 64, None, 0)
        lib.rtpb_plan_destroy(plan)
        if rc != 0:
            raise RuntimeError(lib.rtpb_last_error().decode())
        return out

    def ray_trace(self, rays, initial_material, final_material):
        materials = [initial_material] + list(self.materials) + [final_material]
        if len(materials) != len(self.surfaces) + 1:                        # RT:655-656
            raise ValueError("length of materials should be len(surfaces) + 1")
        kinds = [_builtin_kind(rt, s) for s in self.surfaces]
        if any(k is None for k in kinds):
            return python_loop(self, rays, initial_material, final_material)
        hist = np.asarray(rays, dtype=np.float64)
        if hist.ndim == 1:
            hist = hist[None, None, :]
        elif hist.ndim == 2:
            hist = hist[None]
        S = len(self.surfaces)
        for s0 in range(0, S, RTPB_MAX_SURFACES):
            s1 = min(S, s0 + RTPB_MAX_SURFACES)
            new = trace_segment(self.surfaces[s0:s1], kinds[s0:s1], materials[s0:s1 + 1],
                                np.ascontiguousarray(hist[-1]))
            hist = np.concatenate((hist, new[1:]), axis=0)                  # RT:1229-1232
        return hist

    return ray_trace


def bind_oneshot(lib_path):
    """The one-shot entry points (ABI 8) with their argument types: rtpb_trace_f64 /
    rtpb_trace_f32(surfaces, nsurf, materials, nmat, rays_in, n, out, plane_mask_flags, device, hip_stream) on
    device pointers -- e.g. CuPy's / torch's ``data_ptr()`` -- for a caller that keeps its rays on the GPU."""
    lib = ctypes.CDLL(lib_path)
    lib.rtpb_last_error.restype = ctypes.c_char_p
    for name in ("rtpb_trace_f64", "rtpb_trace_f32"):
        fn = getattr(lib, name)
        fn.restype = ctypes.c_int
        fn.argtypes = [ctypes.POINTER(_Surf), ctypes.c_int32, ctypes.POINTER(_Mat), ctypes.c_int32, ctypes.c_void_p,
                       ctypes.c_int64, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int32, ctypes.c_void_p]
    return lib
