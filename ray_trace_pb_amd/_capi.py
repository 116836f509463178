"""ctypes binding of the C ABI in include/rtpb.h (librtpb.so, built in-tree for gfx950).

The library is REQUIRED: there is no CPU fallback for the trace.  If librtpb.so is missing or cannot
be loaded, :func:`lib` raises ``RuntimeError`` telling how to build it.  ctypes releases the GIL for
the duration of every call, so the host multi-GPU path can run one Python thread per device.
"""
import ctypes
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "librtpb.so")

RTPB_ABI_VERSION = 9
RTPB_F64, RTPB_F32 = 0, 1
RTPB_AOS, RTPB_SOA = 0, 1
RTPB_REFRACT, RTPB_REFLECT = 0, 1
RTPB_FLAT, RTPB_SPHERE, RTPB_PLANE_MIRROR, RTPB_PERFECT_LENS = 0, 1, 2, 3
RTPB_CONSTANT, RTPB_SELLMEIER, RTPB_POLY6, RTPB_TABLE = 0, 1, 2, 3
RTPB_MAX_SURFACES = 63
RTPB_PLANES_FINAL, RTPB_OUT_SOA = 0x1, 0x2          # plane_mask_flags of rtpb_trace_f64 / _f32
RTPB_OK, RTPB_E_INVALID, RTPB_E_HIP, RTPB_E_NODEV, RTPB_E_LIMIT = 0, -1, -2, -3, -4

_c3 = ctypes.c_double * 3
_c6 = ctypes.c_double * 6


class Surface(ctypes.Structure):
    """struct rtpb_surface"""
    _fields_ = [("kind", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("center", _c3), ("normal", _c3), ("input_axis", _c3),
                ("radius", ctypes.c_double), ("radius_sq", ctypes.c_double), ("aperture", ctypes.c_double),
                ("focal_len", ctypes.c_double), ("sin_alpha", ctypes.c_double), ("on_tol", ctypes.c_double)]


class Triangulation(ctypes.Structure):
    _fields_ = [("n_tri", ctypes.c_int64), ("transform", ctypes.c_void_p), ("simplices", ctypes.c_void_p),
                ("values", ctypes.c_void_p), ("cells_x", ctypes.c_int32), ("cells_y", ctypes.c_int32),
                ("x0", ctypes.c_double), ("y0", ctypes.c_double), ("cell_w", ctypes.c_double),
                ("cell_h", ctypes.c_double), ("cell_start", ctypes.c_void_p), ("cell_tris", ctypes.c_void_p)]


class Material(ctypes.Structure):
    """struct rtpb_material"""
    _fields_ = [("kind", ctypes.c_int32), ("table_len", ctypes.c_int32), ("c", _c6),
                ("table", ctypes.POINTER(ctypes.c_double))]


class TraceCall(ctypes.Structure):
    """struct rtpb_trace_call (rtpb_trace_packed)"""
    _fields_ = [("plan", ctypes.c_void_p), ("rays_in", ctypes.c_void_p), ("out", ctypes.c_void_p),
                ("stream", ctypes.c_void_p), ("table_miss", ctypes.c_void_p), ("n_rays", ctypes.c_int64),
                ("in_field_stride", ctypes.c_int64), ("out_plane_stride", ctypes.c_int64),
                ("out_field_stride", ctypes.c_int64), ("plane_mask_lo", ctypes.c_uint64),
                ("plane_mask_hi", ctypes.c_uint64), ("device", ctypes.c_int32), ("in_dtype", ctypes.c_int32),
                ("in_layout", ctypes.c_int32), ("out_layout", ctypes.c_int32)]


# symbol -> (restype, argtypes); every symbol include/rtpb.h declares
_P = ctypes.c_void_p
_i32, _i64, _u64, _dbl = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_double
SIGNATURES = {
    "rtpb_abi_version": (ctypes.c_int, []),
    "rtpb_last_error": (ctypes.c_char_p, []),
    "rtpb_device_count": (ctypes.c_int, []),
    "rtpb_shutdown": (ctypes.c_int, []),
    "rtpb_buffer_alloc": (ctypes.c_int, [_i32, _u64, _u64, _u64, _P, ctypes.POINTER(_P), ctypes.POINTER(_P)]),
    "rtpb_buffer_free": (ctypes.c_int, [_P]),
    "rtpb_buffer_record_stream": (ctypes.c_int, [_P, _P]),
    "rtpb_buffer_trim": (ctypes.c_int, []),
    "rtpb_buffer_held": (ctypes.c_int, [_i32, ctypes.POINTER(_u64), ctypes.POINTER(_i32)]),
    "rtpb_buffer_dlpack": (ctypes.c_int, [_P, _i32, ctypes.POINTER(_i64), _i32, ctypes.POINTER(_P)]),
    "rtpb_buffer_dlpack_discard": (ctypes.c_int, [_P]),
    "rtpb_torch_alloc": (ctypes.c_void_p, [_i64, _i32, _P]),
    "rtpb_torch_free": (None, [_P, _i64, _i32, _P]),
    "rtpb_buffer_stats": (ctypes.c_int, [_i32, ctypes.POINTER(_u64), _i32]),
    "rtpb_plan_create": (ctypes.c_int, [ctypes.POINTER(Surface), _i32, ctypes.POINTER(Material), _i32, _i32,
                                        ctypes.POINTER(_P)]),
    "rtpb_plan_destroy": (ctypes.c_int, [_P]),
    "rtpb_trace": (ctypes.c_int, [_P, _i32, _P, _i32, _i64, _i32, _i64, _P, _i32, _i64, _i64, _u64, _u64, _P]),
    "rtpb_trace_packed": (ctypes.c_int, [ctypes.POINTER(TraceCall)]),
    "rtpb_trace_checked": (ctypes.c_int, [_P, _i32, _P, _i32, _i64, _i32, _i64, _P, _i32, _i64, _i64, _u64, _u64, _P,
                                          _P]),
    "rtpb_trace_f64": (ctypes.c_int, [ctypes.POINTER(Surface), _i32, ctypes.POINTER(Material), _i32, _P, _i64, _P,
                                      ctypes.c_uint32, _i32, _P]),
    "rtpb_trace_f32": (ctypes.c_int, [ctypes.POINTER(Surface), _i32, ctypes.POINTER(Material), _i32, _P, _i64, _P,
                                      ctypes.c_uint32, _i32, _P]),
    "rtpb_oneshot_plans": (ctypes.c_int, []),
    "rtpb_oneshot_clear": (None, []),
    "rtpb_trace_host": (ctypes.c_int, [_P, _P, _i32, _i64, _P, _u64, _u64, ctypes.POINTER(_i32), _i32]),
    "rtpb_ray_fan": (ctypes.c_int, [_i32, _i32, _P, ctypes.POINTER(_dbl), _dbl, _i64, _i64, ctypes.POINTER(_dbl),
                                    _dbl, _P]),
    "rtpb_collimated_rays": (ctypes.c_int, [_i32, _i32, _P, ctypes.POINTER(_dbl), _dbl, _i64, _i64, _dbl,
                                            ctypes.POINTER(_dbl), _dbl, _P]),
    "rtpb_intersect_rays": (ctypes.c_int, [_i32, _i32, _P, _i64, _P, _i64, _P, _P]),
    "rtpb_propagate_plane": (ctypes.c_int, [_i32, _i32, _P, _i64, _P, _i32, _P, _i32, ctypes.POINTER(Material), _i32,
                                            _P, _P, _P, _i64, _P]),
    "rtpb_ray_fan_tables": (ctypes.c_int, [_i32, _i32, _P, _P, _i64, _i64, _P, _P, _P, _P, _P, ctypes.c_double, _P]),
    "rtpb_collimated_rays_tables": (ctypes.c_int, [_i32, _i32, _P, _P, _i64, _i64, _P, _P, _P, _P, _P,
                                                   ctypes.c_double, _P]),
    "rtpb_ray_fan_tables_wl": (ctypes.c_int, [_i32, _i32, _P, _P, _i64, _i64, _P, _P, _P, _P, _P, _P, _P]),
    "rtpb_collimated_rays_tables_wl": (ctypes.c_int, [_i32, _i32, _P, _P, _i64, _i64, _P, _P, _P, _P, _P, _P, _P]),
    "rtpb_spot_sweep": (ctypes.c_int, [_P, _i32, _i64, _P, _i64, _i64, _P, _P, _P, _P, _P, _P, _i64, _P, _P]),
    "rtpb_grid_interpolate": (ctypes.c_int, [_i32, ctypes.POINTER(Triangulation), _P, _i64, _P, _i64,
                                             ctypes.c_double, _P, _P, _P]),
    "rtpb_distinct_keys": (ctypes.c_int, [_i32, _P, _i32, _i64, _i64, _P, _i32, _i32, _P, _P]),
    "rtpb_front_side": (ctypes.c_int, [_P, _i32, _P, _P, _i64, _P, _P]),
    "rtpb_interact": (ctypes.c_int, [_P, _i32, _i32, _P, _P, _P, _i64, _P, _P]),
    "rtpb_spot_stats": (ctypes.c_int, [_i32, _i32, _P, _i64, _i64, _P, _i64, _P, _P]),
    "rtpb_set_tuning": (ctypes.c_int, [ctypes.c_char_p, _i64]),
    "rtpb_timing_enable": (ctypes.c_int, [_i32]),
    "rtpb_timing_collect": (ctypes.c_int, [ctypes.POINTER(_dbl), ctypes.POINTER(_i64)]),
}

_lib = None
_lock = threading.Lock()


class RtpbError(RuntimeError):
    pass


def lib():
    """Load librtpb.so once; raise loudly when it is absent (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(f"{LIB_PATH} not found: the HIP extension is not built. "
                                   "Run `python -c 'import __graft_entry__ as g; g.build()'` or "
                                   "`python -m ray_trace_pb_amd._build`.")
            # One HIP runtime per process: PyTorch ships its own libamdhip64.so (same SONAME,
            # libamdhip64.so.7, as /opt/rocm's).  If librtpb.so were loaded first it would pull in
            # /opt/rocm's runtime and torch's copy, loaded later, would see no GPU.  Importing torch
            # first makes librtpb.so bind to the runtime torch already mapped.
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
            handle = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(handle, name)
                fn.restype = res
                fn.argtypes = args
            if handle.rtpb_abi_version() != RTPB_ABI_VERSION:
                raise RuntimeError("librtpb.so ABI version mismatch; rebuild it")
            _lib = handle
    return _lib


def check(rc):
    if rc != 0:
        msg = lib().rtpb_last_error().decode(errors="replace")
        raise RtpbError(f"rtpb error {rc}: {msg}")
    return rc


def device_count():
    return lib().rtpb_device_count()
