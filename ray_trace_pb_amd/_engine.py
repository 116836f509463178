"""Lowering of a System to C-ABI descriptors, the plan cache, and the two trace drivers.

* :func:`lower` turns surfaces + materials into ``rtpb_surface`` / ``rtpb_material`` arrays
  (include/rtpb.h).  Every constant the reference computes on the host side of its vector
  expressions is computed here exactly the same way (``radius**2`` RT:1499, ``np.sin(alpha)``
  RT:1758), so the kernel's f64 results are bit-identical to the reference.
* Plans (device-resident descriptors) are cached by the byte content of the lowered system.
* :func:`trace_host` -- NumPy in/out through ``rtpb_trace_host`` (H2D, kernel, D2H; optionally sharded
  over several GPUs by ray index, one host thread per device inside the library).
* :func:`trace_device` -- torch CUDA tensors in/out through ``rtpb_trace_packed`` (``rtpb_trace_checked``'s
  arguments in one per-thread block) on torch's current stream; nothing leaves HBM.
"""
import collections
import contextlib
import ctypes
import itertools
import os
import threading

import numpy as np

from . import _capi as C

# on-surface tolerance of the reference (RT:1343, 1408, 1528, 1597).  The kernel computes in float64
# for both storage types, so the reference's absolute tolerance applies unchanged.
ON_TOL = 1e-12


class Lowered:
    __slots__ = ("surfaces", "materials", "tables", "dtype", "nsurf", "key")


def _f3(v):
    a = np.asarray(v, dtype=np.float64).ravel()
    if a.size != 3:
        raise ValueError(f"expected a 3-vector, got {v!r}")
    return a


_LOWERED = collections.OrderedDict()
_LOWERED_MAX = 64
_memo_lock = threading.Lock()            # guards _LOWERED and _KEYS (traces may run on several threads)


def _vec_key(v):
    if type(v) is np.ndarray and v.dtype == np.float64:
        return v.tobytes()
    return np.asarray(v, dtype=np.float64).tobytes()


_KIND_OF_CLASS = {}                      # Surface class -> its fused-kernel kind (a class property)


def _kind_of(s):
    kind = _KIND_OF_CLASS.get(type(s))
    if kind is None:
        kind = _KIND_OF_CLASS[type(s)] = s._rtpb_kind()
    return kind


def _lower_key(surfaces, materials, wl, dtype):
    """Content key of a lowering: every surface / material value lower() reads (the host-side work of
    lower() is ~0.1-0.2 ms for a 9-surface system -- a few % of a C3 trace -- so repeated traces of the same
    system reuse the lowered descriptors), or None when some value has no cheap fingerprint."""
    try:
        parts = [dtype]
        for s in surfaces:
            kind = _kind_of(s)
            p = (kind, _vec_key(s.center), _vec_key(s.input_axis), _vec_key(getattr(s, "normal", s.input_axis)),
                 float(s.aperture_rad))
            if kind == C.RTPB_SPHERE:
                p += (float(s.radius),)
            elif kind == C.RTPB_PERFECT_LENS:
                p += (float(s.focal_len), float(s.alpha))
            parts.append(p)
        for m in materials:
            lowered = m._rtpb_lower() if hasattr(m, "_rtpb_lower") else None
            if lowered is not None:
                # (an immutable tuple of numbers is its own key)
                c = lowered[1]
                parts.append((lowered[0], c if type(c) is tuple else tuple(map(float, c))))
            else:
                # a tabulated material's n() values are memoised only when n() is known to depend on the
                # wavelength and the instance's attributes alone: the package's own (Ebaf11), or a user
                # subclass that declares it with ``rtpb_pure_n = True``.  Any other user n() -- which may
                # read class attributes, globals or other mutable state -- is evaluated on every trace.
                if not _pure_n(m):
                    return None
                fp = table_fingerprint([m])
                if fp is None:
                    return None
                parts.append(fp)
        if wl is not None:
            parts.append(wl.tobytes())
        return tuple(parts)
    except (TypeError, ValueError, AttributeError):
        return None


# ------------------------------------------------------------------------- drop-in call memo
# The content key above reads every lowered value on every trace (~10 us for the C2 system: a few % of a 1M-ray
# trace).  A repeated call with the SAME surface list and material objects skips it when nothing can have changed:
#   * MUTATIONS counts every attribute assignment or deletion on a Surface or a Material (their __setattr__ /
#     __delattr__), so a radius, an aperture, a material coefficient or a whole array rebound since the memo was
#     made invalidates it;
#   * the lists are compared by element identity (a surface or a medium swapped);
#   * arrays edited in place (s.center[2] = z) are caught by comparing the bytes of every array the lowering reads.
# Only systems whose lowered values live in the instances' __dict__ as plain numbers and numeric arrays get a memo.
MUTATIONS = [0]
_CALLS = collections.OrderedDict()       # id(surfaces list) -> _Call
_CALLS_MAX = 16


class _Call:
    __slots__ = ("surfaces", "items", "materials", "dtype", "gen", "arrays", "blob", "low", "lists", "keys_gen")


# bumped whenever remember_keys changes the key set of some tabulated materials: a memoised lowering of a tabulated
# system holds the keys of its time and is valid only while this is unchanged
KEYS_GEN = [0]


_SCALAR_ATTRS = ("aperture_rad", "radius", "focal_len", "alpha")
_NUMBER = (int, float, np.floating, np.integer)


def _call_arrays(surfaces):
    """The arrays the lowering reads (center, input_axis, normal), or None when some lowered value is not held in
    the instance's __dict__ as a numeric array or a plain number (properties, object arrays, lists)."""
    arrs = []
    for s in surfaces:
        d = getattr(s, "__dict__", None)
        if d is None:
            return None
        for name in ("center", "input_axis", "normal"):
            a = d.get(name)
            if a is None:
                if name == "normal" and not hasattr(s, "normal"):
                    continue
                return None
            if type(a) is not np.ndarray or a.dtype.kind not in "fiu":
                return None
            arrs.append(a)
        for name in _SCALAR_ATTRS:
            if name in d:
                if not isinstance(d[name], _NUMBER):
                    return None
            elif hasattr(s, name):
                return None
    return arrs


def memo_lookup(surfaces, materials, dtype):
    """(lowering, tabulated) of the previous call with these very surface and material objects, if provably
    unchanged -- a tabulated system's lowering holds the table keys of the previous bundle (valid while KEYS_GEN is
    unchanged; the caller still checks the bundle against them) -- or None."""
    e = _CALLS.get(id(surfaces))
    if e is None or e.surfaces is not surfaces or e.gen != MUTATIONS[0] or e.dtype != dtype:
        return None
    if e.keys_gen is not None and e.keys_gen != KEYS_GEN[0]:
        return None
    if e.items != surfaces or e.materials != materials:
        return None
    if b"".join([a.tobytes() for a in e.arrays]) != e.blob:
        return None
    for lst, snap in e.lists:
        if tuple(lst) != snap:
            return None
    return e.low, e.keys_gen is not None


def _material_lists(materials):
    """Snapshots of the list attributes (of plain numbers) of the materials (Ebaf11.params: editable in place), or None
    when some attribute is neither a number, a string, None nor such a list."""
    lists = []
    for m in materials:
        for v in vars(m).values():
            if v is None or isinstance(v, (str,) + _NUMBER):
                continue
            if isinstance(v, list) and all(isinstance(x, _NUMBER) for x in v):
                lists.append((v, tuple(v)))
                continue
            return None
    return lists


def memo_store(surfaces, materials, dtype, low, tabulated=False):
    """Remember ``low`` as the lowering of (surfaces, materials, dtype) for memo_lookup.  ``tabulated``: lowered with
    the previous bundle's table keys (valid while KEYS_GEN is unchanged); every tabulated material must have a pure
    n() (the package's own, or ``rtpb_pure_n``)."""
    if not isinstance(surfaces, list):
        return
    arrs = _call_arrays(surfaces)
    if arrs is None:
        return
    lists = _material_lists(materials)
    if lists is None:
        return
    if tabulated and not all(_pure_n(m) for m in tabulated_materials(materials)):
        return
    e = _Call()
    e.surfaces, e.items, e.materials, e.dtype = surfaces, list(surfaces), list(materials), dtype
    e.gen, e.arrays, e.blob, e.low = MUTATIONS[0], arrs, b"".join([a.tobytes() for a in arrs]), low
    e.lists, e.keys_gen = lists, (KEYS_GEN[0] if tabulated else None)
    with _memo_lock:
        _CALLS[id(surfaces)] = e
        _CALLS.move_to_end(id(surfaces))
        while len(_CALLS) > _CALLS_MAX:
            _CALLS.popitem(last=False)


def _pure_n(m):
    return type(m).n.__module__ == __package__ + ".materials" or getattr(type(m), "rtpb_pure_n", False) is True


def lower(surfaces, materials, wavelengths, dtype, tab=None):
    """Lower surfaces (len S) and materials (len S+1: initial, System.materials, final).
    ``wavelengths`` is a callable returning the distinct wavelengths of the bundle (used only for
    user Material subclasses, which lower to per-wavelength tables).  Results are memoised by content
    (_lower_key); the Lowered object is read-only once built.  ``tab``: tabulated(materials) when the caller has it."""
    if len(materials) != len(surfaces) + 1:
        raise ValueError("length of materials should be len(surfaces) + 1")
    wl = None
    if tabulated(materials) if tab is None else tab:
        wl = np.asarray(wavelengths(), dtype=np.float64)
    key = _lower_key(surfaces, materials, wl, dtype)
    if key is not None:
        with _memo_lock:
            low = _LOWERED.get(key)
            if low is not None:
                _LOWERED.move_to_end(key)
                return low
    low = _lower(surfaces, materials, (lambda: wl), dtype)
    if key is not None:
        with _memo_lock:
            _LOWERED[key] = low
            while len(_LOWERED) > _LOWERED_MAX:
                _LOWERED.popitem(last=False)
    return low


def _lower(surfaces, materials, wavelengths, dtype):
    S = len(surfaces)
    if len(materials) != S + 1:
        raise ValueError("length of materials should be len(surfaces) + 1")
    if S > C.RTPB_MAX_SURFACES:
        raise ValueError(f"at most {C.RTPB_MAX_SURFACES} surfaces per trace")
    low = Lowered()
    low.dtype = dtype
    low.nsurf = S
    low.surfaces = (C.Surface * max(S, 1))()
    for k, s in enumerate(surfaces):
        d = low.surfaces[k]
        kind = s._rtpb_kind()
        d.kind = kind
        d.center[:] = _f3(s.center)
        d.input_axis[:] = _f3(s.input_axis)
        d.normal[:] = _f3(getattr(s, "normal", s.input_axis))
        d.aperture = float(s.aperture_rad)
        d.on_tol = ON_TOL
        if kind == C.RTPB_SPHERE:
            d.radius = float(s.radius)
            d.radius_sq = float(s.radius ** 2)          # RT:1499 evaluates self.radius**2 on the host
        elif kind == C.RTPB_PERFECT_LENS:
            d.focal_len = float(s.focal_len)
            d.sin_alpha = float(np.sin(s.alpha))         # RT:1758 xp.sin(self.alpha)
    low.materials = (C.Material * (S + 1))()
    low.tables = []
    key_parts = [bytes(low.surfaces)]
    wl_cache = []
    for k, m in enumerate(materials):
        d = low.materials[k]
        lowered = m._rtpb_lower() if hasattr(m, "_rtpb_lower") else None
        if lowered is not None:
            d.kind, coeffs = lowered
            d.c[:] = [float(c) for c in coeffs]
            key_parts.append(bytes(d))
            continue
        # user Material subclass: tabulate its own n() at the bundle's distinct wavelengths
        if not wl_cache:
            wl_cache.append(np.asarray(wavelengths(), dtype=np.float64))
        wl = wl_cache[0]
        nv = np.broadcast_to(np.asarray(m.n(wl), dtype=np.float64), wl.shape)
        tab = np.ascontiguousarray(np.stack((wl, nv), axis=1).ravel())
        low.tables.append(tab)
        d.kind = C.RTPB_TABLE
        d.table_len = wl.size
        d.table = tab.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
        key_parts.append(bytes(memoryview(tab)) + b"T" + str(k).encode())
    low.key = (dtype, S, b"|".join(key_parts))
    return low


DISTINCT_SLOTS = 8192
DISTINCT_MAX_KEYS = 4096


def _distinct_device(col):
    """Distinct wavelengths of a torch CUDA column with rtpb_distinct_keys (one pass, hash set in HBM);
    None when there are more than DISTINCT_MAX_KEYS of them."""
    import torch
    if col.dtype not in (torch.float64, torch.float32):
        col = col.double()
    if col.shape[0] == 0:
        return np.empty(0)
    if col.stride(0) == 0:
        # a broadcast column (e.g. rays = ray.expand(N, 8)): every element is the one stored value
        return np.unique(col[:1].double().cpu().numpy())
    ws = torch.empty(DISTINCT_SLOTS + 1, dtype=torch.int64, device=col.device)
    lib = C.lib()
    C.check(lib.rtpb_distinct_keys(col.device.index, col.data_ptr(),
                                   C.RTPB_F32 if col.dtype == torch.float32 else C.RTPB_F64, col.shape[0],
                                   col.stride(0), ws.data_ptr(), DISTINCT_SLOTS, DISTINCT_MAX_KEYS,
                                   ws.data_ptr() + 8 * DISTINCT_SLOTS, torch.cuda.current_stream(col.device).cuda_stream))
    host = ws.cpu().numpy()
    if int(host[-1] & 0xFFFFFFFF) > DISTINCT_MAX_KEYS:
        return None
    keys = host[:DISTINCT_SLOTS].view(np.uint64)
    return np.unique(keys[keys != np.uint64(0xFFFFFFFFFFFFFFFF)].view(np.float64))


def distinct_wavelengths(col):
    """Sorted distinct values of a wavelength column (NumPy or torch CUDA), NaN last -- the keys of
    RTPB_TABLE materials.  Single-colour NumPy bundles (the common case) skip the sort; torch CUDA
    columns go through the rtpb_distinct_keys pass (a sort only beyond DISTINCT_MAX_KEYS colours)."""
    if type(col).__module__.startswith("torch"):
        import torch
        if col.is_cuda and col.dim() == 1:
            keys = _distinct_device(col)
            if keys is not None:
                return keys
        return np.unique(torch.unique(col.double()).cpu().numpy())
    w = np.asarray(col, dtype=np.float64)
    if w.size and (w == w[0]).all():
        return w[:1].copy()
    return np.unique(w)


# ------------------------------------------------------------------------- table keys of previous bundles
# Materials that lower to host-evaluated tables (user Material subclasses, Ebaf11) need the bundle's
# distinct wavelengths -- a pass over the whole wavelength column (rtpb_distinct_keys) before every trace.
# Torch-CUDA callers trace optimistically instead: with the key set of the previous bundle traced through
# the same tabulated materials, checked by the kernel (rtpb_trace_checked's table-miss flag), and only on a
# miss is the column scanned and the bundle re-traced with its own keys.  Exact either way: a table holds
# n() of the material at each key, and every ray's key is present or the trace is redone.  Assumes n()
# depends only on the wavelength and the material's attributes (the fingerprint below).
_KEYS = collections.OrderedDict()
_KEYS_MAX = 64


class _NoFingerprint(Exception):
    pass


def _fp(v, depth=0):
    if depth > 8:
        raise _NoFingerprint
    if v is None or isinstance(v, (bool, int, float, complex, str, bytes, np.generic)):
        return (type(v).__name__, v)
    if isinstance(v, np.ndarray):
        return ("nd", v.dtype.str, v.shape, v.tobytes())
    if isinstance(v, (list, tuple)):
        return (type(v).__name__,) + tuple(_fp(x, depth + 1) for x in v)
    if isinstance(v, dict):
        return ("dict",) + tuple(sorted((str(k), _fp(x, depth + 1)) for k, x in v.items()))
    raise _NoFingerprint


def tabulated(materials):
    """The materials that lower to host-evaluated (wavelength, n) tables."""
    return [m for m in materials if not (hasattr(m, "_rtpb_lower") and m._rtpb_lower() is not None)]


tabulated_materials = tabulated


def table_fingerprint(materials):
    """Hashable identity of the tabulated materials' n() (class + attribute values), or None.  A material
    may supply ``_rtpb_table_key()`` (a cheap hashable of everything its n() reads; Ebaf11 does)."""
    try:
        return tuple((type(m).__module__, type(m).__qualname__, id(type(m)),
                      m._rtpb_table_key() if hasattr(m, "_rtpb_table_key") else _fp(vars(m))) for m in materials)
    except (_NoFingerprint, TypeError):
        return None


def previous_keys(fp):
    if fp is None:
        return None
    with _memo_lock:
        keys = _KEYS.get(fp)
        if keys is not None:
            _KEYS.move_to_end(fp)
    return keys


def remember_keys(fp, keys):
    KEYS_GEN[0] += 1
    if fp is None:
        return
    with _memo_lock:
        _KEYS[fp] = keys
        _KEYS.move_to_end(fp)
        while len(_KEYS) > _KEYS_MAX:
            _KEYS.popitem(last=False)


def lower_material(m, wavelengths):
    """One ``rtpb_material`` (tables keep a reference on the returned struct as ``_keep``)."""
    d = C.Material()
    lowered = m._rtpb_lower() if hasattr(m, "_rtpb_lower") else None
    if lowered is not None:
        d.kind, coeffs = lowered
        d.c[:] = [float(c) for c in coeffs]
        return d
    wl = np.asarray(wavelengths(), dtype=np.float64)
    nv = np.broadcast_to(np.asarray(m.n(wl), dtype=np.float64), wl.shape)
    tab = np.ascontiguousarray(np.stack((wl, nv), axis=1).ravel())
    d.kind = C.RTPB_TABLE
    d.table_len = wl.size
    d.table = tab.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    d._keep = tab
    return d


# ------------------------------------------------------------------------- plan cache
# Plans (device-resident descriptors) cached by the lowered content, LRU-bounded.  A plan in use by a
# trace (plan_ref) is never destroyed under it: eviction only marks it, and the last user frees it.
# per-thread rtpb_trace_packed argument blocks of trace_device
_TLS = threading.local()


class _Plan:
    __slots__ = ("ptr", "lib", "users", "evicted")

    def __init__(self, ptr, lib):
        self.ptr, self.lib, self.users, self.evicted = ptr, lib, 0, False


_PLANS = collections.OrderedDict()
_PLANS_MAX = 32
_plans_lock = threading.Lock()


def _acquire(low):
    with _plans_lock:
        p = _PLANS.get(low.key)
        if p is not None:
            _PLANS.move_to_end(low.key)
        else:
            out = ctypes.c_void_p()
            lib = C.lib()
            C.check(lib.rtpb_plan_create(low.surfaces, low.nsurf, low.materials, low.nsurf + 1, low.dtype,
                                         ctypes.byref(out)))
            p = _Plan(out, lib)
            _PLANS[low.key] = p
            while len(_PLANS) > _PLANS_MAX:
                _, old = _PLANS.popitem(last=False)
                old.evicted = True
                if old.users == 0:
                    old.lib.rtpb_plan_destroy(old.ptr)
        p.users += 1
        return p


def _release(p):
    with _plans_lock:
        p.users -= 1
        if p.evicted and p.users == 0:
            p.lib.rtpb_plan_destroy(p.ptr)


@contextlib.contextmanager
def plan_ref(low):
    """The cached plan of a lowered system, held for the duration of the ``with`` block."""
    p = _acquire(low)
    try:
        yield p.ptr
    finally:
        _release(p)


def clear_plan_cache():
    """Drop every cached plan (plans in use are freed by their last user).  Plans read some knobs at
    creation (rtpb_set_tuning "indexed_materials"), so tests toggling them start from an empty cache."""
    with _plans_lock:
        while _PLANS:
            _, old = _PLANS.popitem(last=False)
            old.evicted = True
            if old.users == 0:
                old.lib.rtpb_plan_destroy(old.ptr)


def plan_for(low):
    """The cached plan's raw pointer (single-threaded tools; library paths use plan_ref)."""
    p = _acquire(low)
    _release(p)
    return p.ptr


def plane_mask(planes):
    """(lo, hi) 64-bit halves of the 128-bit plane mask of rtpb_trace (memoised per plane list)."""
    key = tuple(planes)
    m = _MASKS.get(key)
    if m is None:
        lo = hi = 0
        for p in key:
            if p < 64:
                lo |= 1 << p
            else:
                hi |= 1 << (p - 64)
        m = _MASKS[key] = (lo, hi)
        if len(_MASKS) > 256:
            _MASKS.clear()
            _MASKS[key] = m
    return m


_MASKS = {}


def resolve_planes(planes, nsurf):
    """'all' | 'final' | iterable of plane indices (0 = input, 2i+1 at surface i, 2i+2 after it)."""
    P = 2 * nsurf + 1
    if isinstance(planes, str):
        if planes == "all":
            return list(range(P))
        if planes == "final":
            return [P - 1]
        raise ValueError(f"planes must be 'all', 'final' or a list of plane indices, got {planes!r}")
    sel = sorted({int(p) if int(p) >= 0 else int(p) + P for p in planes})
    if not sel or sel[0] < 0 or sel[-1] >= P:
        raise ValueError(f"plane indices must lie in [0, {P - 1}]")
    return sel


# ------------------------------------------------------------------------- drivers
def _np_dtype(dtype):
    return np.float64 if dtype == C.RTPB_F64 else np.float32


PINNED_MIN_BYTES = 32 << 20


def host_empty(shape, dtype):
    """Output array for the NumPy path.  Large outputs come from PyTorch's pinned (page-locked)
    caching host allocator: the GPU DMAs straight into them, and a freed array's pages go back to
    the cache already faulted in -- a fresh np.empty of the C2 history (704 MB) costs ~60 ms of
    first-touch page faults, more than the whole trace.  The result is an ordinary ndarray."""
    nbytes = int(np.prod(shape)) * np.dtype(dtype).itemsize
    if nbytes >= PINNED_MIN_BYTES:
        try:
            import torch
            tdt = torch.float64 if np.dtype(dtype) == np.float64 else torch.float32
            return torch.empty(tuple(shape), dtype=tdt, pin_memory=True).numpy()
        except Exception:       # no torch / no pinned memory: fall back to pageable memory
            pass
    return np.empty(shape, dtype=dtype)


def input_code(dt):
    """Element type the kernel reads the input rays in: float32 rays as they are (widened exactly in
    the kernel, as NumPy promotes them in the reference), everything else as float64.  Independent of
    the storage type, so float64 rays are never rounded before the arithmetic."""
    code = _INPUT_CODES.get(dt)
    if code is None:
        name = str(dt).replace("torch.", "")
        code = _INPUT_CODES[dt] = C.RTPB_F32 if name == "float32" else C.RTPB_F64
    return code


_INPUT_CODES = {}


def trace_host(low, rays2d, planes, devices=None, out=None):
    """NumPy (N, 8) -> NumPy (len(planes), N, 8) of the plan's storage type."""
    rays2d = np.asarray(rays2d)
    in_code = input_code(rays2d.dtype)
    rays2d = np.ascontiguousarray(rays2d, dtype=_np_dtype(in_code))
    n = rays2d.shape[0]
    if out is None:
        out = host_empty((len(planes), n, 8), _np_dtype(low.dtype))
    lo, hi = plane_mask(planes)
    if devices is None:
        devs = None
        ndev = 0
    else:
        devs = (ctypes.c_int32 * len(devices))(*devices)
        ndev = len(devices)
    with plan_ref(low) as plan:
        C.check(C.lib().rtpb_trace_host(plan, rays2d.ctypes.data, in_code, n, out.ctypes.data, lo, hi, devs, ndev))
    return out


_DLTENSOR = b"dltensor"
_buffer_seed = itertools.count(1)


def _capsule_api():
    api = ctypes.pythonapi
    api.PyCapsule_New.restype = ctypes.py_object
    api.PyCapsule_New.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p]
    api.PyCapsule_IsValid.restype = ctypes.c_int
    api.PyCapsule_IsValid.argtypes = [ctypes.py_object, ctypes.c_char_p]
    return api


def history_buffer(shape, dtype, device, chunk_bytes=0, stream=None):
    """A C-contiguous torch CUDA tensor of ``shape`` and ``dtype`` (float32 / float64) on ``device`` whose device
    memory is mapped in shuffled 64 MiB chunks, so a history traced into it writes at the fast rate whatever the
    physical state of the card (a history's many-plane write pattern runs 15-45 % slower into physically
    contiguous placements).

    Default (``chunk_bytes`` = 0): allocated by torch's caching allocator in the device's history pool
    (:func:`history_pool`, ABI 7) for ``stream`` (default: the current stream) -- an ordinary torch tensor to
    torch: ``Tensor.record_stream``, ``torch.cuda.memory_allocated`` and out-of-memory handling work as for any
    other tensor.  ``chunk_bytes`` > 0 (placement studies): a library buffer of that chunk size
    (rtpb_buffer_alloc, its own stream-ordered pool; a use on another stream is recorded with
    :func:`record_stream`), exported through DLPack."""
    import torch
    if dtype not in (torch.float32, torch.float64):
        raise ValueError("history_buffer: dtype must be torch.float32 or torch.float64")
    dev = torch.device(device)
    if dev.type != "cuda":
        raise ValueError("history_buffer: a CUDA (HIP) device is required")
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    shape = tuple(int(v) for v in shape)
    if not chunk_bytes:
        if stream is not None and not isinstance(stream, torch.cuda.Stream):
            stream = torch.cuda.ExternalStream(stream, device=torch.device("cuda", idx))
        return pool_empty(shape, dtype, torch.device("cuda", idx), stream)
    elem = 8 if dtype == torch.float64 else 4
    nbytes = elem
    for v in shape:
        nbytes *= v
    if nbytes == 0:
        return torch.empty(shape, dtype=dtype, device=dev)
    if stream is None:
        stream = torch.cuda.current_stream(torch.device("cuda", idx))
    raw_stream = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
    lib = C.lib()
    ptr, handle = ctypes.c_void_p(), ctypes.c_void_p()
    seed = next(_buffer_seed)
    global _LIB_BUFFERS_USED
    _LIB_BUFFERS_USED = True
    if lib.rtpb_buffer_alloc(idx, nbytes, chunk_bytes, seed, raw_stream, ctypes.byref(ptr), ctypes.byref(handle)):
        # the device may be full of blocks torch's caching allocator holds: release them and retry once
        torch.cuda.synchronize(idx)
        trim_history_buffers()
        torch.cuda.empty_cache()
        C.check(lib.rtpb_buffer_alloc(idx, nbytes, chunk_bytes, seed, raw_stream, ctypes.byref(ptr),
                                      ctypes.byref(handle)))
    managed = ctypes.c_void_p()
    ext = (ctypes.c_int64 * len(shape))(*shape)
    rc = lib.rtpb_buffer_dlpack(handle, len(shape), ext, C.RTPB_F64 if elem == 8 else C.RTPB_F32,
                                ctypes.byref(managed))
    if rc != 0:
        lib.rtpb_buffer_free(handle)
        C.check(rc)
    api = _capsule_api()
    capsule = api.PyCapsule_New(managed, _DLTENSOR, None)
    try:
        return torch.utils.dlpack.from_dlpack(capsule)
    except Exception:
        # DLPack protocol: an importer that consumed the capsule renamed it and owns the deleter; only an
        # unconsumed capsule is discarded here (its deleter frees the buffer and the managed tensor)
        if api.PyCapsule_IsValid(capsule, _DLTENSOR):
            lib.rtpb_buffer_dlpack_discard(managed)
        raise


# set once this process has made a buffer of the library's own pool (history_buffer(..., chunk_bytes=N)): only then
# can a traced tensor lie in one, and trace_device records its launches with the library too
_LIB_BUFFERS_USED = False
_POOLS = {}
_ALLOCATORS = {}            # a MemPool holds a raw pointer to its allocator: allocators live as long as the process
_POOL_IDS = {}              # MemPool.id of each live pool (a property call per use otherwise)
_pools_lock = threading.Lock()


def hip_runtimes():
    """The distinct files mapped into this process as a HIP runtime (libamdhip64*), from /proc/self/maps."""
    paths = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                if "libamdhip64" in line:
                    paths.add(os.path.realpath(line.split(None, 5)[-1].strip()))
    except OSError:
        pass
    return sorted(paths)


def torch_hip_runtime():
    """Directory of the HIP runtime torch ships (torch/lib): the one runtime librtpb must bind to."""
    import torch
    return os.path.realpath(os.path.join(os.path.dirname(torch.__file__), "lib"))


def check_one_hip_runtime():
    """Raise unless exactly one HIP runtime is mapped and it is torch's: a second libamdhip64 (e.g. librtpb.so
    loaded before torch, binding /opt/rocm's) would give librtpb its own device context, and pointers it maps for
    torch's caching allocator would be foreign to torch's runtime."""
    paths = hip_runtimes()
    lib_dir = torch_hip_runtime()
    if len(paths) != 1 or os.path.dirname(paths[0]) != lib_dir:
        raise RuntimeError(f"history pool: expected one HIP runtime, torch's ({lib_dir}), mapped in this process; "
                           f"found {paths}")


def pool_allocator(device_index):
    """The CUDAPluggableAllocator of device ``device_index``'s history pool (rtpb_torch_alloc / rtpb_torch_free),
    created once and held for the life of the process.  Holding it is what keeps the pool valid: a MemPool keeps
    only a raw pointer to its allocator's C++ object (torch._C._MemPool takes the allocator by pointer and does not
    keep the Python object alive), so a pool whose allocator had been collected would call through freed memory at
    its first allocation -- the segfault of round 5's first probe."""
    import torch
    idx = int(device_index)
    alloc = _ALLOCATORS.get(idx)
    if alloc is None:
        C.lib()                 # loaded after torch: librtpb binds to torch's HIP runtime
        check_one_hip_runtime()
        alloc = _ALLOCATORS[idx] = torch.cuda.memory.CUDAPluggableAllocator(C.LIB_PATH, "rtpb_torch_alloc",
                                                                            "rtpb_torch_free")
        check_one_hip_runtime()
    return alloc


def history_pool(device_index):
    """The torch.cuda.MemPool of device ``device_index``'s history buffers: torch's caching allocator with
    librtpb's shuffled-chunk mappings as its segment allocator (rtpb_torch_alloc / rtpb_torch_free, ABI 7).
    torch owns everything else -- caching, stream-ordered reuse (Tensor.record_stream), memory statistics and
    out-of-memory handling; ``use_on_oom``: an allocation outside the pool that runs out of memory may take
    the pool's cached blocks.  The pool's unused segments are released by :func:`trim_history_buffers` (a live
    MemPool keeps them through torch.cuda.empty_cache())."""
    import torch
    idx = int(device_index)
    with _pools_lock:
        pool = _POOLS.get(idx)
        if pool is None:
            alloc = pool_allocator(idx)
            with torch.cuda.device(idx):
                pool = torch.cuda.MemPool(alloc.allocator(), use_on_oom=True)
            _POOLS[idx] = pool
            _POOL_IDS[idx] = pool.id
    return pool


def pool_empty(shape, dtype, device, stream=None):
    """torch.empty(shape, dtype, device) allocated in the device's history pool (:func:`history_pool`) for
    ``stream`` (default: the current stream).  torch.cuda.use_mem_pool's calls, made directly (the context
    manager costs a few microseconds of the drop-in call)."""
    import torch
    dev = device if type(device) is torch.device else torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    pool = _POOLS.get(idx)
    if pool is None:
        pool = history_pool(idx)
    pid = _POOL_IDS[idx]
    on_current = idx == torch.cuda.current_device()
    if stream is None and on_current:
        # the drop-in call's case (current device and stream): no context managers
        _begin_pool(idx, pid)
        try:
            return torch.empty(shape, dtype=dtype, device=dev if dev.index is not None else torch.device("cuda", idx))
        finally:
            _end_pool(idx, pid)
            _release_pool(idx, pid)
    dev_ctx = torch.cuda.device(idx) if not on_current else contextlib.nullcontext()
    with dev_ctx:
        ctx = torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()
        with ctx:
            _begin_pool(idx, pid)
            try:
                return torch.empty(shape, dtype=dtype, device=dev if dev.index is not None else torch.device("cuda", idx))
            finally:
                _end_pool(idx, pid)
                _release_pool(idx, pid)


def _pool_calls():
    """torch.cuda.use_mem_pool's three calls (torch 2.10: torch._C._cuda_beginAllocateCurrentThreadToPool,
    _cuda_endAllocateToPool, _cuda_releasePool)."""
    import torch
    return (torch._C._cuda_beginAllocateCurrentThreadToPool, torch._C._cuda_endAllocateToPool,
            torch._C._cuda_releasePool)


def _begin_pool(idx, pid):
    global _begin_pool, _end_pool, _release_pool
    _begin_pool, _end_pool, _release_pool = _pool_calls()
    _begin_pool(idx, pid)


def _end_pool(idx, pid):            # replaced by _begin_pool's first call
    _pool_calls()[1](idx, pid)


def _release_pool(idx, pid):        # replaced by _begin_pool's first call
    _pool_calls()[2](idx, pid)


def buffer_stats(device=-1):
    """librtpb's buffer statistics (rtpb_buffer_stats): live torch-pool segment bytes and count, dead virtual
    bytes and ranges, plain-allocation fallbacks, torch segments allocated / freed, the dead-VA limit."""
    out = (ctypes.c_uint64 * 8)()
    C.check(C.lib().rtpb_buffer_stats(int(device), out, 8))
    keys = ("pool_bytes", "pool_segments", "dead_va_bytes", "dead_va_ranges", "plain_allocs", "segments_allocated",
            "segments_freed", "dead_va_limit")
    return dict(zip(keys, (int(v) for v in out)))


def record_stream(tensor, stream):
    """``tensor.record_stream(stream)`` for every kind of device memory: torch's caching-allocator record
    (history-pool tensors are torch allocations), plus the library's record when the tensor lies in a buffer of
    the library's own pool (``history_buffer(..., chunk_bytes=...)``, rtpb_buffer_record_stream)."""
    tensor.record_stream(stream)
    if tensor.numel() == 0:
        return
    raw = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
    rc = C.lib().rtpb_buffer_record_stream(tensor.data_ptr(), raw)
    if rc < 0:
        C.check(rc)


def history_buffers_held(device=-1):
    """(bytes, segments) of history memory cached but not in use on ``device`` (-1: every device): free bytes of
    the history pools' segments, plus freed buffers of the library's own pool (and retired ones whose last uses
    have not completed yet)."""
    nb, cnt = ctypes.c_uint64(), ctypes.c_int32()
    C.check(C.lib().rtpb_buffer_held(int(device), ctypes.byref(nb), ctypes.byref(cnt)))
    held, n = int(nb.value), int(cnt.value)
    with _pools_lock:
        pools = list(_POOLS.items())
    for idx, pool in pools:
        if device >= 0 and idx != device:
            continue
        for seg in pool.snapshot():
            free = int(seg["total_size"]) - int(seg["allocated_size"])
            if free > 0:
                held += free
                n += 1
    return held, n


def trim_history_buffers():
    """Release the device memory history buffers hold while unused.  A history pool none of whose blocks is in
    use is dropped -- torch returns its segments at once (librtpb unmaps them) and the next history gets a new
    pool.  A pool with live tensors is kept: dropping it would leave their blocks in an orphaned pool whose
    memory nothing here counts or releases when they die; its cached blocks stay available to any
    torch allocation that runs out of memory (use_on_oom), and a later trim releases the pool once its tensors are
    gone.  The library's own pool is emptied too (rtpb_buffer_trim waits for the last recorded uses)."""
    with _pools_lock:
        drop = []
        for idx, pool in list(_POOLS.items()):
            if all(int(seg["allocated_size"]) == 0 for seg in pool.snapshot()):
                drop.append(_POOLS.pop(idx))
                _POOL_IDS.pop(idx, None)
    del drop
    C.check(C.lib().rtpb_buffer_trim())


def device_empty(shape, dtype, device):
    """torch.empty on a CUDA device; on an out-of-memory error the cached history memory (the history pools'
    unused segments, the library's own pool) is released and the allocation retried once."""
    import torch
    try:
        return torch.empty(shape, dtype=dtype, device=device)
    except torch.OutOfMemoryError:
        if history_buffers_held()[1] == 0:
            raise
        trim_history_buffers()
        return torch.empty(shape, dtype=dtype, device=device)


def check_out(out, shape, dtype, device):
    """The caller's ``out=`` history: a C-contiguous CUDA tensor of exactly the history's shape and type."""
    import torch
    if not isinstance(out, torch.Tensor) or not out.is_cuda:
        raise ValueError("out must be a torch CUDA tensor (e.g. ray_trace_pb_amd.raytrace.history_buffer)")
    if tuple(out.shape) != tuple(shape) or out.dtype != dtype or out.device != device or not out.is_contiguous():
        raise ValueError(f"out must be a contiguous {dtype} tensor of shape {tuple(shape)} on {device}; got "
                         f"{out.dtype} {tuple(out.shape)} on {out.device}")
    return out


_STREAMS = {}               # (device, raw hipStream_t) -> torch.cuda.Stream of torch's current stream


def _raw_stream(dev):
    """torch's current raw hipStream_t on device `dev` (torch._C._cuda_getCurrentRawStream: no Stream wrapper)."""
    global _raw_stream
    import torch
    get = getattr(torch._C, "_cuda_getCurrentRawStream", None)
    if get is None:
        def get(d):
            return torch.cuda.current_stream(d).cuda_stream
    _raw_stream = get
    return get(dev)


def trace_device(low, rays, planes, layout_out=C.RTPB_AOS, out=None, stream=None, miss=None, own_out=False):
    """torch CUDA (N, 8) -> torch CUDA (len(planes), N, 8) [AOS] or (len(planes), 8, N) [SOA] of the
    plan's storage type.  ``miss``: a zeroed int32 CUDA tensor the launch sets to 1 when a ray's
    wavelength is not a key of the plan's TABLE materials (rtpb_trace_checked).  ``stream``: None (torch's
    current stream), a torch.cuda.Stream or a raw hipStream_t.  ``own_out``: ``out`` was just allocated by the
    caller on the current stream (its use there needs no record)."""
    import torch
    tdt = torch.float64 if low.dtype == C.RTPB_F64 else torch.float32
    in_code = input_code(rays.dtype)
    want = torch.float32 if in_code == C.RTPB_F32 else torch.float64
    if rays.dtype != want or not rays.is_contiguous():
        rays = rays.to(dtype=want).contiguous()
    n = rays.shape[0]
    dev = rays.get_device()
    fresh_out = (out is None or own_out) and stream is None
    if out is None:
        shape = (len(planes), n, 8) if layout_out == C.RTPB_AOS else (len(planes), 8, n)
        out = device_empty(shape, tdt, rays.device)
    lo, hi = plane_mask(planes)
    if stream is None:
        # torch's current stream: its raw handle, and one torch.cuda.Stream per handle (the wrapper record_stream
        # takes) instead of a new wrapper per call
        stream = _raw_stream(dev)
        cur = _STREAMS.get((dev, stream))
        if cur is None:
            cur = torch.cuda.current_stream(dev)
            if len(_STREAMS) > 64:
                _STREAMS.clear()
            _STREAMS[(dev, stream)] = cur
    elif isinstance(stream, torch.cuda.Stream):
        cur, stream = stream, stream.cuda_stream
    else:
        # a raw hipStream_t: torch's view of it, so the launch's use can be recorded
        cur = _STREAMS.get((dev, stream))
        if cur is None:
            cur = torch.cuda.ExternalStream(stream, device=rays.device)
            if len(_STREAMS) > 64:
                _STREAMS.clear()
            _STREAMS[(dev, stream)] = cur
    lib = C.lib()
    p = _acquire(low)
    try:
        # rtpb_trace_packed with a per-thread argument block per (plan, device, shape, planes, stream): ctypes
        # marshals one pointer instead of 15 arguments (~1 us of the call at C2 size); only the buffers change
        calls = getattr(_TLS, "calls", None)
        if calls is None:
            calls = _TLS.calls = {}
        key = (p.ptr.value, dev, in_code, n, layout_out, lo, hi, stream)
        blk = calls.get(key)
        if blk is None:
            if len(calls) > 64:
                calls.clear()
            c = C.TraceCall(plan=p.ptr.value, device=dev, in_dtype=in_code, n_rays=n, in_layout=C.RTPB_AOS,
                            in_field_stride=0, out_layout=layout_out, out_plane_stride=8 * n, out_field_stride=n,
                            plane_mask_lo=lo, plane_mask_hi=hi, stream=stream)
            blk = calls[key] = (c, ctypes.byref(c))
        c = blk[0]
        c.rays_in = rays.data_ptr()
        c.out = out.data_ptr()
        c.table_miss = None if miss is None else miss.data_ptr()
        rc = lib.rtpb_trace_packed(blk[1])
    finally:
        _release(p)
    if rc:
        C.check(rc)
    if n:
        # the launch's use of `out` and of the rays on this stream, recorded: torch's allocator (a no-op on the
        # tensor's own stream) and the library's own buffer pool then hand the memory to a later owner only after
        # this launch.  (A history this call allocated itself lies on the launch stream already: no record.)
        if not fresh_out:
            out.record_stream(cur)
        rays.record_stream(cur)
        if _LIB_BUFFERS_USED:
            lib.rtpb_buffer_record_stream(out.data_ptr(), stream)
            lib.rtpb_buffer_record_stream(rays.data_ptr(), stream)
    return out
