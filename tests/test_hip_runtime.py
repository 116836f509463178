"""CPU: the history pool's allocator binds to torch's HIP runtime and stays alive.

Round 5's first MemPool probe (gpurun_out/r05_a) died with SIGSEGV at the pool's first allocation.  Cause
(DESIGN.md §2): torch._C._MemPool takes its allocator by raw pointer and keeps no reference to the Python
CUDAPluggableAllocator, whose C++ object dies with it; the probe's tree dropped that object after building the pool.
_engine.pool_allocator now holds every allocator for the life of the process and refuses to build one unless
exactly one HIP runtime -- torch's -- is mapped (librtpb loaded after torch binds to it by SONAME)."""
import os

import pytest

torch = pytest.importorskip("torch")

from ray_trace_pb_amd import _capi as C  # noqa: E402
from ray_trace_pb_amd import _engine as E  # noqa: E402


def test_one_hip_runtime_and_it_is_torchs():
    C.lib()
    alloc = torch.cuda.memory.CUDAPluggableAllocator(C.LIB_PATH, "rtpb_torch_alloc", "rtpb_torch_free")
    assert alloc.allocator() is not None
    paths = E.hip_runtimes()
    assert len(paths) == 1, paths
    assert os.path.dirname(paths[0]) == E.torch_hip_runtime()
    E.check_one_hip_runtime()


def test_pool_allocator_is_held_for_the_process():
    a = E.pool_allocator(0)
    assert E._ALLOCATORS[0] is a
    assert E.pool_allocator(0) is a                    # created once: a pool's raw pointer stays valid
    assert E.hip_runtimes() == [os.path.join(E.torch_hip_runtime(), "libamdhip64.so")]


def test_guard_refuses_a_second_runtime(monkeypatch):
    monkeypatch.setattr(E, "hip_runtimes", lambda: [os.path.join(E.torch_hip_runtime(), "libamdhip64.so"),
                                                     "/opt/rocm-7.2.0/lib/libamdhip64.so.7.2"])
    with pytest.raises(RuntimeError, match="one HIP runtime"):
        E.check_one_hip_runtime()
    monkeypatch.setattr(E, "hip_runtimes", lambda: ["/opt/rocm-7.2.0/lib/libamdhip64.so.7.2"])
    with pytest.raises(RuntimeError, match="torch's"):
        E.check_one_hip_runtime()
