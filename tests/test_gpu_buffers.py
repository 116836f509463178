"""Placement-robust history buffers and ``ray_trace(..., out=)``.  Default: torch tensors of the device's history
pool (a torch.cuda.MemPool whose segments librtpb maps in shuffled chunks, rtpb_torch_alloc / _free, ABI 7) --
bit-identical histories, torch's own stream rules (Tensor.record_stream), statistics and out-of-memory handling.
The C ABI's own buffers (rtpb_buffer_alloc / _free / _dlpack, ABI 5-6; ``history_buffer(..., chunk_bytes=)``)
keep their stream-ordered pool: never handed to a new owner while work of the previous owner -- on its
allocation stream or on a recorded stream -- can still touch them."""
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
    """History-pool segments are cached by torch once their tensors die (the same block comes back) and
    released by trim_history_buffers."""
    rt.trim_history_buffers()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    free0 = torch.cuda.mem_get_info()[0]
    ptrs = set()
    for _ in range(4):
        t = rt.history_buffer((19, 50_000_000, 8), torch.float32, DEV)      # 30.4 GB: one C3 history
        t[-1, -1].fill_(1.0)
        ptrs.add(t.data_ptr())
        del t
        gc.collect()
    assert len(ptrs) == 1                                                   # the cached block came back
    torch.cuda.synchronize()
    assert torch.cuda.mem_get_info()[0] < free0 - (28 << 30)                # ... and is still held (28.3 GiB)
    assert rt.history_buffers_held(0)[0] >= 19 * 50_000_000 * 8 * 4
    rt.trim_history_buffers()
    assert torch.cuda.mem_get_info()[0] >= free0 - (256 << 20)
    assert rt.history_buffers_held(0) == (0, 0)


def test_history_buffers_are_torch_allocations():
    """memory_allocated counts a history-pool tensor; librtpb maps (and on release unmaps) its segment."""
    from ray_trace_pb_amd import _engine as E
    rt.trim_history_buffers()
    torch.cuda.synchronize()
    a0, s0 = torch.cuda.memory_allocated(0), E.buffer_stats(0)
    t = rt.history_buffer((11, 1 << 24, 8), torch.float64, DEV)             # 11.8 GB
    assert torch.cuda.memory_allocated(0) - a0 == t.numel() * 8
    s1 = E.buffer_stats(0)
    assert s1["segments_allocated"] == s0["segments_allocated"] + 1 and s1["pool_bytes"] >= t.numel() * 8
    del t
    gc.collect()
    assert torch.cuda.memory_allocated(0) == a0
    rt.trim_history_buffers()
    s2 = E.buffer_stats(0)
    assert s2["segments_freed"] == s1["segments_freed"] + 1 and s2["pool_segments"] == s0["pool_segments"]
    # a released mapping's virtual range is never reserved again: counted as dead address space
    assert s2["dead_va_bytes"] >= s1["dead_va_bytes"] + 11 * (1 << 24) * 8 * 8


def test_buffer_abi_errors():
    lib = C.lib()
    p, h = ctypes.c_void_p(), ctypes.c_void_p()
    assert lib.rtpb_buffer_alloc(0, 0, 0, 1, None, ctypes.byref(p), ctypes.byref(h)) == C.RTPB_E_INVALID
    assert lib.rtpb_buffer_alloc(10_000, 1 << 20, 0, 1, None, ctypes.byref(p), ctypes.byref(h)) == C.RTPB_E_NODEV
    assert lib.rtpb_buffer_free(None) == C.RTPB_E_INVALID
    assert lib.rtpb_buffer_alloc(0, 5 << 20, 2 << 20, 7, None, ctypes.byref(p), ctypes.byref(h)) == 0
    shape = (ctypes.c_int64 * 2)(1 << 30, 8)
    m = ctypes.c_void_p()
    assert lib.rtpb_buffer_dlpack(h, 2, shape, C.RTPB_F64, ctypes.byref(m)) == C.RTPB_E_INVALID   # too large
    # record_stream: inside the live buffer -> recorded (0); outside any live buffer -> 1 (not an error)
    s = torch.cuda.Stream(DEV)
    assert lib.rtpb_buffer_record_stream(ctypes.c_void_p(p.value + 4096), s.cuda_stream) == 0
    assert lib.rtpb_buffer_record_stream(ctypes.c_void_p(p.value + (6 << 20) + 64), s.cuda_stream) == 1
    assert lib.rtpb_buffer_free(h) == 0
    assert lib.rtpb_buffer_record_stream(p, s.cuda_stream) == 1           # freed: no longer live
    # a managed tensor no importer consumed is discarded through its own deleter (the buffer is pooled)
    C.check(lib.rtpb_buffer_trim())
    assert lib.rtpb_buffer_alloc(0, 5 << 20, 2 << 20, 7, None, ctypes.byref(p), ctypes.byref(h)) == 0
    shape = (ctypes.c_int64 * 2)(1024, 8)
    assert lib.rtpb_buffer_dlpack(h, 2, shape, C.RTPB_F64, ctypes.byref(m)) == 0
    assert rt.history_buffers_held(0) == (0, 0)
    assert lib.rtpb_buffer_dlpack_discard(m) == 0
    assert rt.history_buffers_held(0)[1] == 1
    C.check(lib.rtpb_buffer_trim())
    assert rt.history_buffers_held() == (0, 0)


def test_large_default_histories_are_pooled_buffers():
    """System.ray_trace without out= allocates histories >= POOLED_HISTORY_BYTES in the history pool: the same
    block comes back once the previous result is dropped, and the history is bit-identical to a trace into a
    torch.empty history."""
    system, m0, m1, rays, ref = golden("c3_relay")
    fan = torch.empty((4 * 1000 * 1000, 8), dtype=torch.float64, device=DEV)
    rt.fan_into(fan, np.array([8.0, 0, 0]), np.pi / 180, 2000, 0.635, 2000)
    planes = 2 * len(system.surfaces) + 1
    assert planes * fan.shape[0] * 8 * 4 >= rt.POOLED_HISTORY_BYTES
    from ray_trace_pb_amd import _engine as E
    made = E.buffer_stats(0)["segments_allocated"]
    h1 = system.ray_trace(fan, m0, m1, dtype="float32")
    p1 = h1.data_ptr()
    assert any(seg["address"] <= p1 < seg["address"] + seg["total_size"] for seg in E.history_pool(0).snapshot())
    ref_t = torch.empty_like(h1)
    system.ray_trace(fan, m0, m1, dtype="float32", out=ref_t)
    assert torch.equal(h1.view(torch.int32), ref_t.view(torch.int32))
    del h1
    gc.collect()
    h2 = system.ray_trace(fan, m0, m1, dtype="float32")
    assert h2.data_ptr() == p1
    assert E.buffer_stats(0)["segments_allocated"] <= made + 1
    assert torch.equal(h2.view(torch.int32), ref_t.view(torch.int32))
    small = system.ray_trace(torch.from_numpy(rays).to(DEV), m0, m1)        # small: torch's default pool
    assert same_bits(small.cpu().numpy(), ref)
    del h2
    gc.collect()
    rt.trim_history_buffers()


@pytest.mark.skipif(not hasattr(torch.cuda, "_sleep"), reason="torch.cuda._sleep is not available")
def test_default_history_obeys_torch_record_stream():
    """The lightsheet pattern with torch's own idiom (scripts/2024_04_01_lightsheet.py:51-60,134-135): a >= 1 GiB
    default history is copied to the host on a side stream (delayed), recorded with torch's Tensor.record_stream
    and freed while the copy is pending; the next configuration traces into a default history at once.  Both
    read back bitwise: torch never handed the first history's memory to the second trace early."""
    import systems
    rt.trim_history_buffers()
    system = systems.c3_system(rt, mat)
    m0 = m1 = mat.Vacuum()
    nt = nph = 1342                                          # 1,800,964 rays: 19 float32 planes = 1.02 GiB
    P = 2 * len(system.surfaces) + 1
    fans, refs = [], []
    for h in (0.0, 12.0):
        f = torch.empty((nt * nph, 8), dtype=torch.float64, device=DEV)
        rt.fan_into(f, np.array([h, 0, 0]), np.pi / 180, nt, 0.635, nph)
        fans.append(f)
        r = torch.empty((P, nt * nph, 8), dtype=torch.float32, device=DEV)
        system.ray_trace(f, m0, m1, dtype="float32", out=r)
        refs.append(r.cpu())
    a0 = torch.cuda.memory_allocated(0)
    h1 = system.ray_trace(fans[0], m0, m1, dtype="float32")
    assert h1.nbytes >= 1 << 30 and torch.cuda.memory_allocated(0) - a0 >= h1.nbytes     # torch sees it
    host = torch.empty(h1.shape, dtype=h1.dtype, pin_memory=True)
    side = torch.cuda.Stream(DEV)
    side.wait_stream(torch.cuda.current_stream(DEV))
    gc.collect()
    with torch.cuda.stream(side):
        torch.cuda._sleep(1_000_000_000)
        host.copy_(h1, non_blocking=True)
    h1.record_stream(side)                                   # torch's method, nothing of this package
    p1 = h1.data_ptr()
    del h1
    h2 = system.ray_trace(fans[1], m0, m1, dtype="float32")
    # the first history's block stays withheld while the copy is pending (checked only when the side stream is
    # still busy after the allocation: a host slower than the delay frees the block rightly)
    if not side.query():
        assert h2.data_ptr() != p1
    torch.cuda.synchronize()
    assert torch.equal(host.view(torch.int32), refs[0].view(torch.int32))
    assert torch.equal(h2.cpu().view(torch.int32), refs[1].view(torch.int32))
    del h2
    gc.collect()
    rt.trim_history_buffers()


def _sleep_available():
    return hasattr(torch.cuda, "_sleep")


def _delay(stream, cycles=200_000_000):
    """A kernel that spins on `stream` (torch.cuda._sleep) so that work queued after it on that stream runs
    well after the host has moved on."""
    with torch.cuda.stream(stream):
        torch.cuda._sleep(cycles)


@pytest.mark.skipif(not _sleep_available(), reason="torch.cuda._sleep is not available")
def test_reuse_waits_for_the_previous_owners_allocation_stream():
    """Freed on stream A while a (delayed) kernel on A still writes it; the next buffer of that size, taken
    for stream B, is the same memory, and B's work runs only after A's: B's values survive."""
    C.check(C.lib().rtpb_buffer_trim())
    a, b = torch.cuda.Stream(DEV), torch.cuda.Stream(DEV)
    shape = (3, 1 << 20, 8)
    from ray_trace_pb_amd import _engine as E
    t = E.history_buffer(shape, torch.float32, DEV, chunk_bytes=64 << 20, stream=a)
    p = t.data_ptr()
    _delay(a)
    with torch.cuda.stream(a):
        t.fill_(1.0)                       # queued behind the spin: still pending when t is freed
    del t
    gc.collect()
    u = E.history_buffer(shape, torch.float32, DEV, chunk_bytes=64 << 20, stream=b)
    assert u.data_ptr() == p               # the pooled buffer
    with torch.cuda.stream(b):
        u.fill_(2.0)                       # must run after A's fill
    torch.cuda.synchronize()
    assert bool((u == 2.0).all())
    del u
    gc.collect()
    C.check(C.lib().rtpb_buffer_trim())


@pytest.mark.skipif(not _sleep_available(), reason="torch.cuda._sleep is not available")
def test_reuse_waits_for_recorded_streams():
    """Allocated for stream A, used on a side stream S (recorded with record_stream -- torch's own
    Tensor.record_stream ignores this memory) and freed while S's work is pending; the next owner on A
    waits for S."""
    C.check(C.lib().rtpb_buffer_trim())
    a, side = torch.cuda.Stream(DEV), torch.cuda.Stream(DEV)
    from ray_trace_pb_amd import _engine as E
    shape = (5, 1 << 20, 8)
    t = E.history_buffer(shape, torch.float64, DEV, chunk_bytes=64 << 20, stream=a)
    p = t.data_ptr()
    _delay(side)
    with torch.cuda.stream(side):
        t.fill_(3.0)
    rt.record_stream(t, side)
    del t
    gc.collect()
    u = E.history_buffer(shape, torch.float64, DEV, chunk_bytes=64 << 20, stream=a)
    assert u.data_ptr() == p
    with torch.cuda.stream(a):
        u.fill_(4.0)
    torch.cuda.synchronize()
    assert bool((u == 4.0).all())
    del u
    gc.collect()
    C.check(C.lib().rtpb_buffer_trim())


def test_trace_on_a_side_stream_is_recorded():
    """trace_device records its launch stream on an out= history buffer allocated for another stream: the
    next owner of that memory waits for the trace."""
    system, m0, m1, rays, ref = golden("c1_plano_convex")
    from ray_trace_pb_amd import _engine as E
    C.check(C.lib().rtpb_buffer_trim())
    x = torch.from_numpy(np.tile(rays, (2000, 1))).to(DEV)
    a, side = torch.cuda.Stream(DEV), torch.cuda.Stream(DEV)
    shape = (2 * len(system.surfaces) + 1, x.shape[0], 8)
    out = E.history_buffer(shape, torch.float64, DEV, chunk_bytes=64 << 20, stream=a)
    p = out.data_ptr()
    side.wait_stream(torch.cuda.current_stream(DEV))
    with torch.cuda.stream(side):
        if _sleep_available():
            torch.cuda._sleep(100_000_000)
        system.ray_trace(x, m0, m1, out=out)
    del out
    gc.collect()
    u = E.history_buffer(shape, torch.float64, DEV, chunk_bytes=64 << 20, stream=a)
    assert u.data_ptr() == p
    with torch.cuda.stream(a):
        u.fill_(-1.0)
    torch.cuda.synchronize()
    assert bool((u == -1.0).all())
    del u
    gc.collect()
    C.check(C.lib().rtpb_buffer_trim())


def test_pool_keeps_only_the_newest_buffer():
    """The C ABI's own pool (history_buffer(..., chunk_bytes=)) holds one freed buffer per device (the newest),
    not every size seen."""
    from ray_trace_pb_amd import _engine as E
    rt.trim_history_buffers()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    free0 = torch.cuda.mem_get_info()[0]
    bufs = [E.history_buffer((k, 1 << 27, 8), torch.float32, DEV, chunk_bytes=64 << 20) for k in (2, 3, 4)]
    for t in bufs:
        t[-1, -1].fill_(0.0)
    del bufs, t
    gc.collect()
    torch.cuda.synchronize()
    # freeing never blocks (ABI 8): the two older buffers have retired but stay mapped until a call that may
    # synchronise -- here the next allocation that maps new memory
    assert rt.history_buffers_held(0)[1] == 3
    w = E.history_buffer((1, 1 << 20, 8), torch.float32, DEV, chunk_bytes=64 << 20)
    nbytes, nbuf = rt.history_buffers_held(0)
    assert nbuf == 1 and nbytes == 4 << 32                       # the last one freed: 16 GiB
    assert torch.cuda.mem_get_info()[0] >= free0 - (16 << 30) - (512 << 20)
    del w
    gc.collect()
    rt.trim_history_buffers()
    assert torch.cuda.mem_get_info()[0] >= free0 - (512 << 20)


def test_torch_allocation_takes_the_pooled_memory():
    """A torch allocation outside the history pool that only fits in memory the pool caches succeeds: torch
    takes the pool's cached block (MemPool use_on_oom) -- here the drop-in call itself, with a history below
    POOLED_HISTORY_BYTES (a default-pool allocation)."""
    system, m0, m1, rays, ref = golden("c3_relay")
    from ray_trace_pb_amd import _engine as E
    rt.trim_history_buffers()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    big = rt.history_buffer((1, 5 << 30), torch.float64, DEV)         # 40 GiB, then cached by the pool
    big[0, -1].fill_(0.0)
    del big
    gc.collect()
    torch.cuda.synchronize()
    assert rt.history_buffers_held(0)[0] >= 40 << 30
    fan = torch.empty((1000 * 1000, 8), dtype=torch.float64, device=DEV)
    rt.fan_into(fan, np.array([8.0, 0, 0]), np.pi / 180, 1000, 0.635, 1000)
    want = system.ray_trace(fan, m0, m1, dtype="float32").cpu()        # 0.15 GB history
    torch.cuda.synchronize()
    torch.cuda.empty_cache()                                           # its block must not be cached
    free = torch.cuda.mem_get_info()[0]
    filler = torch.empty(free - (256 << 20), dtype=torch.uint8, device=DEV)   # leave 256 MiB free
    try:
        got = system.ray_trace(fan, m0, m1, dtype="float32")               # needs the pool's memory
        assert torch.equal(got.cpu().view(torch.int32), want.view(torch.int32))
        del got
    finally:
        del filler
        torch.cuda.empty_cache()
    assert E.device_empty((4,), torch.float32, DEV).numel() == 4
    rt.trim_history_buffers()


def test_dead_va_limit_falls_back_to_plain_allocations():
    """Past rtpb_set_tuning("buffer_dead_va_limit") of never-reused virtual ranges, new history buffers are plain
    hipMalloc allocations (the bound on reserved address space): traced into, they read back bitwise."""
    from ray_trace_pb_amd import _engine as E
    system, m0, m1, rays, ref = golden("c4_opm")
    x = torch.from_numpy(rays).to(DEV)
    lib = C.lib()
    rt.trim_history_buffers()
    limit0 = E.buffer_stats()["dead_va_limit"]
    try:
        C.check(lib.rtpb_set_tuning(b"buffer_dead_va_limit", 0))
        plain0 = E.buffer_stats()["plain_allocs"]
        for chunk in (0, 64 << 20):                                    # the history pool and the C ABI's pool
            out = E.history_buffer(ref.shape, torch.float64, DEV, chunk_bytes=chunk)
            got = system.ray_trace(x, m0, m1, out=out)
            assert same_bits(got.cpu().numpy(), ref)
            del out, got
            gc.collect()
            rt.trim_history_buffers()
        assert E.buffer_stats()["plain_allocs"] == plain0 + 2
    finally:
        C.check(lib.rtpb_set_tuning(b"buffer_dead_va_limit", limit0))
    assert E.buffer_stats()["dead_va_limit"] == limit0


def test_release_after_unrecorded_side_stream_use_is_safe():
    """a history released while a kernel on a stream nobody recorded still writes it must not be
    unmapped under that kernel (releasing a mapping synchronises the device first) -- no fault, and the next
    allocation reads back its own values."""
    from ray_trace_pb_amd import _engine as E
    rt.trim_history_buffers()
    side = torch.cuda.Stream(DEV)
    t = E.history_buffer((4, 1 << 22, 8), torch.float64, DEV, chunk_bytes=64 << 20)
    side.wait_stream(torch.cuda.current_stream(DEV))
    with torch.cuda.stream(side):
        if _sleep_available():
            torch.cuda._sleep(200_000_000)
        t.fill_(7.0)                                          # not recorded: the library does not know
    del t
    gc.collect()                                              # pooled (the newest freed buffer)
    u = E.history_buffer((5, 1 << 22, 8), torch.float64, DEV, chunk_bytes=64 << 20)
    u.fill_(1.0)
    del u
    gc.collect()                                              # u pooled: t retires and is unmapped -- after a sync
    v = E.history_buffer((6, 1 << 22, 8), torch.float64, DEV, chunk_bytes=64 << 20)
    v.fill_(2.0)
    torch.cuda.synchronize()
    assert bool((v == 2.0).all())
    del v
    gc.collect()
    rt.trim_history_buffers()


def test_writer_streams_large_histories_back_to_back(tmp_path):
    """The lightsheet pattern at scale (scripts/2024_04_01_lightsheet.py:51-60,134-135): >= 1 GiB default
    histories (history buffers) written back to back through io.HistoryWriter, whose device-to-host copies
    run on a side stream while the next configuration traces: every configuration reads back bitwise."""
    from ray_trace_pb_amd import io as rio
    import systems
    rt.trim_history_buffers()
    system = systems.c3_system(rt, mat)
    m0 = m1 = mat.Vacuum()
    nt = nph = 1342                                         # 1,800,964 rays: 19 float32 planes = 1.02 GiB
    fan = torch.empty((nt * nph, 8), dtype=torch.float64, device=DEV)
    heights = [0.0, 5.0, 10.0, 15.0, 2.5]
    P = 2 * len(system.surfaces) + 1
    assert P * nt * nph * 8 * 4 >= rt.POOLED_HISTORY_BYTES
    path = str(tmp_path / "sweep.zarr")
    with rio.HistoryWriter(path, len(heights), P, nt * nph, dtype="float32") as w:
        for k, h in enumerate(heights):
            rt.fan_into(fan, np.array([h, 0, 0]), np.pi / 180, nt, 0.635, nph)
            w.write(k, system.ray_trace(fan, m0, m1, dtype="float32"))
    got = rio.read_array(path)
    for k, h in enumerate(heights):
        rt.fan_into(fan, np.array([h, 0, 0]), np.pi / 180, nt, 0.635, nph)
        ref = torch.empty((P, nt * nph, 8), dtype=torch.float32, device=DEV)
        system.ray_trace(fan, m0, m1, dtype="float32", out=ref)
        assert np.array_equal(got[k].view(np.int32), ref.cpu().numpy().view(np.int32)), k
    C.check(C.lib().rtpb_buffer_trim())


def test_trim_keeps_a_pool_whose_tensors_live():
    """trim_history_buffers drops only history pools none of whose blocks is in use.  A live history
    survives a trim with its pool (still counted by history_buffers_held once freed); freed, the next trim returns
    its memory to the device."""
    from ray_trace_pb_amd import _engine as E
    rt.trim_history_buffers()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    free0 = torch.cuda.mem_get_info()[0]
    t = rt.history_buffer((4, 1 << 28, 8), torch.float32, DEV)            # 32 GiB in the history pool
    t[-1, -1].fill_(3.0)
    pid = E.history_pool(0).id
    rt.trim_history_buffers()
    assert E._POOL_IDS.get(0) == pid                                     # kept: a tensor lives in it
    torch.cuda.synchronize()
    assert float(t[-1, -1, -1]) == 3.0
    del t
    gc.collect()
    assert rt.history_buffers_held(0)[0] >= 32 << 30                     # cached, and counted
    rt.trim_history_buffers()
    assert 0 not in E._POOL_IDS                                          # dropped now
    assert rt.history_buffers_held(0) == (0, 0)
    assert torch.cuda.mem_get_info()[0] >= free0 - (512 << 20)


def test_trim_allocate_cycles_grow_dead_va_by_one_segment_each():
    """every released history-pool segment keeps its virtual range reserved, so a
    trim -> allocate cycle adds exactly that segment's size to the dead address space -- a bounded, linear cost:
    at a C3-size history (30.4 GB) the default 32 TiB limit allows ~1,150 such cycles before new histories fall
    back to plain hipMalloc (still correct, test_dead_va_limit_falls_back_to_plain_allocations)."""
    from ray_trace_pb_amd import _engine as E
    rt.trim_history_buffers()
    seg = None
    dead = [E.buffer_stats()["dead_va_bytes"]]
    for k in range(4):
        t = rt.history_buffer((1, 1 << 27, 8), torch.float32, DEV)        # 4 GiB
        t[0, -1].fill_(float(k))
        seg = E.buffer_stats()["pool_bytes"]
        del t
        gc.collect()
        rt.trim_history_buffers()
        dead.append(E.buffer_stats()["dead_va_bytes"])
    steps = [b - a for a, b in zip(dead, dead[1:])]
    assert all(d == steps[0] for d in steps) and steps[0] >= 4 << 30 and steps[0] <= seg
    limit = E.buffer_stats()["dead_va_limit"]
    assert limit // (19 * 50_007_030 * 8 * 4) >= 1000


@pytest.mark.skipif(not _sleep_available(), reason="torch.cuda._sleep is not available")
def test_trace_on_a_raw_stream_is_recorded_with_torch():
    """trace_device with an explicit raw hipStream_t records its use of `out` and of the rays with torch
    (through torch.cuda.ExternalStream): a torch history traced on a delayed side stream and freed at once is not
    handed to the next allocation of its size before that trace has run -- which then reads back bitwise."""
    from ray_trace_pb_amd import _engine as E
    system, m0, m1, rays, ref = golden("c3_relay")
    mats = [m0] + list(system.materials) + [m1]
    low = E.lower(system.surfaces, mats, lambda: np.unique(rays[:, 7]), C.RTPB_F64)
    x = torch.from_numpy(rays).to(DEV)
    planes = E.resolve_planes("all", len(system.surfaces))
    side = torch.cuda.Stream(DEV)
    side.wait_stream(torch.cuda.current_stream(DEV))
    out = torch.empty(ref.shape, dtype=torch.float64, device=DEV)       # torch's default pool, current stream
    p = out.data_ptr()
    host = torch.empty(ref.shape, dtype=torch.float64, pin_memory=True)
    gc.collect()
    _delay(side, 1_000_000_000)
    E.trace_device(low, x, planes, out=out, stream=side.cuda_stream)     # raw handle
    with torch.cuda.stream(side):
        host.copy_(out, non_blocking=True)
    del out
    nxt = torch.empty(ref.shape, dtype=torch.float64, device=DEV)
    # the block stays withheld while the trace is pending; the check holds when the side stream is still busy
    # AFTER the allocation (so it was at the allocation: a host slower than the delay frees the block rightly)
    if not side.query():
        assert nxt.data_ptr() != p
    nxt.fill_(-1.0)
    torch.cuda.synchronize()
    assert same_bits(host.numpy(), ref)
