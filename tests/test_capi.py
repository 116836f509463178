"""librtpb.so loads, exports every symbol include/rtpb.h declares, and validates its arguments
(no compute calls: these run without a GPU)."""
import ctypes
import os
import re

import numpy as np
import pytest

import ray_trace_pb_amd.materials as mat
import ray_trace_pb_amd.raytrace as rt
from ray_trace_pb_amd import _capi as C
import systems

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rtpb.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|double|const char\s*\*|void\s*\*?)\s*(rtpb_\w+)\s*\(", text, flags=re.M)))


def test_library_exports_every_declared_symbol():
    lib = C.lib()
    names = declared_functions()
    assert len(names) >= 10
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(C.SIGNATURES), set(names) ^ set(C.SIGNATURES)


def test_struct_layouts_match_header():
    # rtpb_surface: 2 x int32 + 9 doubles (3 vectors) + 6 doubles; rtpb_material: 2 x int32 + 6 doubles + ptr
    assert ctypes.sizeof(C.Surface) == 8 + 8 * 15
    assert ctypes.sizeof(C.Material) == 8 + 8 * 6 + 8
    # rtpb_trace_call: 5 pointers, 4 int64 + 2 uint64, 4 int32 -- field order as in include/rtpb.h
    assert ctypes.sizeof(C.TraceCall) == 5 * 8 + 6 * 8 + 4 * 4
    assert [f for f, _ in C.TraceCall._fields_] == [
        "plan", "rays_in", "out", "stream", "table_miss", "n_rays", "in_field_stride", "out_plane_stride",
        "out_field_stride", "plane_mask_lo", "plane_mask_hi", "device", "in_dtype", "in_layout", "out_layout"]


def test_packed_trace_validates_without_a_gpu():
    """rtpb_trace_packed: a NULL block and a NULL plan are rejected before any device work."""
    lib = C.lib()
    assert lib.rtpb_trace_packed(None) == C.RTPB_E_INVALID
    assert b"NULL" in lib.rtpb_last_error()
    c = C.TraceCall(n_rays=4, out_plane_stride=32, out_field_stride=4, plane_mask_lo=1)
    assert lib.rtpb_trace_packed(ctypes.byref(c)) == C.RTPB_E_INVALID
    assert b"plan is NULL" in lib.rtpb_last_error()


def test_abi_version_and_device_count():
    lib = C.lib()
    assert lib.rtpb_abi_version() == C.RTPB_ABI_VERSION
    assert lib.rtpb_device_count() >= 0


def _flat_plan_args(nsurf=1):
    surf = (C.Surface * nsurf)()
    for s in surf:
        s.kind = C.RTPB_FLAT
        s.normal[:] = [0, 0, 1]
        s.input_axis[:] = [0, 0, 1]
        s.aperture = 1.0
        s.on_tol = 1e-12
    mats = (C.Material * (nsurf + 1))()
    for m in mats:
        m.kind = C.RTPB_CONSTANT
        m.c[0] = 1.0
    return surf, mats


def test_plan_create_validates():
    lib = C.lib()
    surf, mats = _flat_plan_args(2)
    plan = ctypes.c_void_p()
    assert lib.rtpb_plan_create(surf, 2, mats, 2, C.RTPB_F64, ctypes.byref(plan)) == -1       # nmat != S+1
    assert b"len(surfaces) + 1" in lib.rtpb_last_error()
    assert lib.rtpb_plan_create(surf, 2, mats, 3, 7, ctypes.byref(plan)) == -1                 # bad dtype
    surf[1].kind = 42
    assert lib.rtpb_plan_create(surf, 2, mats, 3, C.RTPB_F64, ctypes.byref(plan)) == -1       # bad kind
    surf[1].kind = C.RTPB_SPHERE
    mats[1].kind = C.RTPB_TABLE                                                               # empty table
    assert lib.rtpb_plan_create(surf, 2, mats, 3, C.RTPB_F64, ctypes.byref(plan)) == -1
    mats[1].kind = C.RTPB_CONSTANT
    assert lib.rtpb_plan_create(surf, 64, mats, 65, C.RTPB_F64, ctypes.byref(plan)) == -4     # > 63 surfaces
    assert lib.rtpb_plan_create(surf, 2, mats, 3, C.RTPB_F64, ctypes.byref(plan)) == 0
    assert plan.value
    assert lib.rtpb_plan_destroy(plan) == 0


@pytest.mark.skipif(C.device_count() > 0, reason="checks the no-GPU error path")
def test_trace_without_gpu_fails_loudly():
    lib = C.lib()
    surf, mats = _flat_plan_args(1)
    plan = ctypes.c_void_p()
    assert lib.rtpb_plan_create(surf, 1, mats, 2, C.RTPB_F64, ctypes.byref(plan)) == 0
    rays = np.zeros((4, 8))
    out = np.zeros((3, 4, 8))
    rc = lib.rtpb_trace_host(plan, rays.ctypes.data, 0, 4, out.ctypes.data, 7, 0, None, 0)
    assert rc == -3 and b"no GPU" in lib.rtpb_last_error()
    rc = lib.rtpb_trace(plan, 0, rays.ctypes.data, 0, 4, 0, 0, out.ctypes.data, 0, 32, 0, 7, 0, None)
    assert rc == -3
    lib.rtpb_plan_destroy(plan)


def test_oneshot_validates_arguments():
    """rtpb_trace_f64 / _f32: bad flags, a material count other than S + 1 and a negative ray
    count fail with RTPB_E_INVALID before any device work."""
    lib = C.lib()
    surf, mats = _flat_plan_args(2)
    assert lib.rtpb_trace_f64(surf, 2, mats, 3, None, 0, None, 0x10, 0, None) == -1
    assert b"plane_mask_flags" in lib.rtpb_last_error()
    assert lib.rtpb_trace_f32(surf, 2, mats, 2, None, 0, None, 0, 0, None) == -1
    assert b"len(surfaces) + 1" in lib.rtpb_last_error()
    assert lib.rtpb_trace_f64(surf, 2, mats, 3, None, -1, None, 0, 0, None) == -1
    assert lib.rtpb_trace_f64(surf, 64, mats, 65, None, 0, None, 0, 0, None) == -4


@pytest.mark.skipif(C.device_count() > 0, reason="checks the no-GPU error path")
def test_oneshot_without_gpu_fails_loudly():
    lib = C.lib()
    surf, mats = _flat_plan_args(1)
    lib.rtpb_oneshot_clear()
    rays = np.zeros((4, 8))
    assert lib.rtpb_trace_f64(surf, 1, mats, 2, rays.ctypes.data, 4, rays.ctypes.data, 0, 0, None) == -3
    assert b"no GPU" in lib.rtpb_last_error()
    assert lib.rtpb_oneshot_plans() == 1            # the system was lowered and cached before the device check
    lib.rtpb_oneshot_clear()
    assert lib.rtpb_oneshot_plans() == 0


@pytest.mark.skipif(C.device_count() > 0, reason="checks the no-GPU error path")
def test_system_ray_trace_raises_without_gpu():
    import ray_trace_pb_amd.materials as mat
    import ray_trace_pb_amd.raytrace as rt
    s = rt.System([rt.FlatSurface([0, 0, 0], [0, 0, 1], 1)], [])
    with pytest.raises(C.RtpbError):
        s.ray_trace(rt.get_collimated_rays([0, 0, -1], 0.5, 3, 0.5), mat.Vacuum(), mat.Vacuum())


def test_missing_extension_fails_loudly(monkeypatch, tmp_path):
    """No silent fallback: without librtpb.so every product call raises (here: a fresh loader pointed
    at a path with no library)."""
    monkeypatch.setattr(C, "_lib", None)
    monkeypatch.setattr(C, "LIB_PATH", str(tmp_path / "librtpb.so"))
    with pytest.raises(RuntimeError, match="not built"):
        C.lib()
    system, rays, m0, m1 = systems.c1_plano_convex(rt, mat)
    with pytest.raises(RuntimeError, match="not built"):
        system.ray_trace(rays, m0, m1)
