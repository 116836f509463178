"""Placement-robust history buffers (rtpb_buffer_alloc / _free / _dlpack, ABI 5) and ``ray_trace(..., out=)``:
the buffer is ordinary device memory to the kernels (bit-identical histories), a torch tensor to the caller,
and released when the tensor dies."""
import ctypes
import gc
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import ray_trace_pb_amd.materials as mat  # noqa: E402
import ray_trace_pb_amd.raytrace as rt  # noqa: E402
from ray_trace_pb_amd import _capi as C  # noqa: E402
from parity import GOLDEN, same_bits  # noqa: E402
from serialize import system_from_json  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def golden(name):
    d = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    system, m0, m1 = system_from_json(rt, mat, str(d["system_json"]))
    return system, m0, m1, d["rays_in"], d["history"]


def test_history_buffer_is_a_plain_cuda_tensor():
    t = rt.history_buffer((3, 1000, 8), torch.float32, DEV)
    assert t.is_cuda and t.dtype == torch.float32 and tuple(t.shape) == (3, 1000, 8) and t.is_contiguous()
    t.copy_(torch.arange(t.numel(), dtype=torch.float32, device=DEV).view_as(t))
    assert float(t.sum()) == float(torch.arange(t.numel(), dtype=torch.float64).sum())
    u = rt.history_buffer((2, 5, 8), torch.float64, torch.device(DEV))
    assert u.dtype == torch.float64 and u.data_ptr() % 256 == 0
    assert rt.history_buffer((0, 5, 8), torch.float32, DEV).numel() == 0


@pytest.mark.parametrize("name", ["c1_plano_convex", "c3_relay", "c4_opm", "stress"])
@pytest.mark.parametrize("dtype", [None, "float32"])
def test_trace_into_history_buffer_bitwise(name, dtype):
    system, m0, m1, rays, ref = golden(name)
    x = torch.from_numpy(rays).to(DEV)
    tdt = torch.float32 if dtype else torch.float64
    out = rt.history_buffer(ref.shape, tdt, DEV)
    got = system.ray_trace(x, m0, m1, dtype=dtype, out=out)
    assert got.data_ptr() == out.data_ptr()
    want = system.ray_trace(x, m0, m1, dtype=dtype)
    assert same_bits(got.cpu().numpy(), want.cpu().numpy())
    if dtype is None:
        assert same_bits(got.cpu().numpy(), ref)
    fin = rt.history_buffer((1,) + ref.shape[1:], tdt, DEV)
    system.ray_trace(x, m0, m1, dtype=dtype, planes="final", out=fin)
    assert same_bits(fin.cpu().numpy()[0], want.cpu().numpy()[-1])


def test_out_validation():
    system, m0, m1, rays, ref = golden("c1_plano_convex")
    x = torch.from_numpy(rays).to(DEV)
    with pytest.raises(ValueError):
        system.ray_trace(x, m0, m1, out=torch.empty((1,) + ref.shape[1:], dtype=torch.float64, device=DEV))
    with pytest.raises(ValueError):
        system.ray_trace(x, m0, m1, out=torch.empty(ref.shape, dtype=torch.float32, device=DEV))
    with pytest.raises(ValueError):
        system.ray_trace(rays, m0, m1, out=torch.empty(ref.shape, dtype=torch.float64, device=DEV))
    with pytest.raises(ValueError):
        system.ray_trace(x[None], m0, m1, out=torch.empty(ref.shape, dtype=torch.float64, device=DEV))


def test_buffers_are_pooled_and_trimmed():
    C.check(C.lib().rtpb_buffer_trim())
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    ptrs = set()
    for _ in range(4):
        t = rt.history_buffer((19, 50_000_000, 8), torch.float32, DEV)      # 30.4 GB: one C3 history
        t[-1, -1].fill_(1.0)
        ptrs.add(t.data_ptr())
        del t
        gc.collect()
    assert len(ptrs) == 1                                                   # the pooled buffer came back
    torch.cuda.synchronize()
    assert torch.cuda.mem_get_info()[0] < free0 - (28 << 30)                # ... and is still held (28.3 GiB)
    C.check(C.lib().rtpb_buffer_trim())
    assert torch.cuda.mem_get_info()[0] >= free0 - (256 << 20)


def test_buffer_abi_errors():
    lib = C.lib()
    p, h = ctypes.c_void_p(), ctypes.c_void_p()
    assert lib.rtpb_buffer_alloc(0, 0, 0, 1, ctypes.byref(p), ctypes.byref(h)) == C.RTPB_E_INVALID
    assert lib.rtpb_buffer_alloc(10_000, 1 << 20, 0, 1, ctypes.byref(p), ctypes.byref(h)) == C.RTPB_E_NODEV
    assert lib.rtpb_buffer_free(None) == C.RTPB_E_INVALID
    assert lib.rtpb_buffer_alloc(0, 5 << 20, 2 << 20, 7, ctypes.byref(p), ctypes.byref(h)) == 0
    shape = (ctypes.c_int64 * 2)(1 << 30, 8)
    m = ctypes.c_void_p()
    assert lib.rtpb_buffer_dlpack(h, 2, shape, C.RTPB_F64, ctypes.byref(m)) == C.RTPB_E_INVALID   # too large
    assert lib.rtpb_buffer_free(h) == 0


def test_large_default_histories_are_pooled_buffers():
    """System.ray_trace without out= allocates histories >= POOLED_HISTORY_BYTES as pooled history buffers:
    the same buffer comes back once the previous result is dropped, and the history is bit-identical to a
    trace into a torch.empty history."""
    system, m0, m1, rays, ref = golden("c3_relay")
    fan = torch.empty((4 * 1000 * 1000, 8), dtype=torch.float64, device=DEV)
    rt.fan_into(fan, np.array([8.0, 0, 0]), np.pi / 180, 2000, 0.635, 2000)
    planes = 2 * len(system.surfaces) + 1
    assert planes * fan.shape[0] * 8 * 4 >= rt.POOLED_HISTORY_BYTES
    h1 = system.ray_trace(fan, m0, m1, dtype="float32")
    p1 = h1.data_ptr()
    ref_t = torch.empty_like(h1)
    system.ray_trace(fan, m0, m1, dtype="float32", out=ref_t)
    assert torch.equal(torch.isnan(h1), torch.isnan(ref_t))
    assert bool(((h1 == ref_t) | torch.isnan(ref_t)).all())
    assert torch.equal(h1.view(torch.int32), ref_t.view(torch.int32))
    del h1
    gc.collect()
    h2 = system.ray_trace(fan, m0, m1, dtype="float32")
    assert h2.data_ptr() == p1
    assert torch.equal(h2.view(torch.int32), ref_t.view(torch.int32))
    small = system.ray_trace(torch.from_numpy(rays).to(DEV), m0, m1)        # small: torch's allocator
    assert same_bits(small.cpu().numpy(), ref)
    del h2
    gc.collect()
    C.check(C.lib().rtpb_buffer_trim())
