"""Where does the NumPy end-to-end time go? (diagnostic)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ray_trace_pb_amd.materials as mat  # noqa: E402
import ray_trace_pb_amd.raytrace as rt  # noqa: E402
from ray_trace_pb_amd import _capi as C, _engine as E  # noqa: E402
import systems  # noqa: E402


def tm(fn, reps=5):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e3


n = 1_000_000
system, rays = systems.c2_system(rt, mat), systems.c2_rays(n)
V = mat.Vacuum()
low = E.lower(system.surfaces, [V] + list(system.materials) + [V], lambda: np.unique(rays[:, 7]), C.RTPB_F64)
sel = E.resolve_planes("all", 5)
print("cpus", os.cpu_count(), "sched", len(os.sched_getaffinity(0)))
print("np.empty 704MB             %.1f ms" % tm(lambda: np.empty((11, n, 8))))
print("np.empty + touch (fill)    %.1f ms" % tm(lambda: np.empty((11, n, 8)).fill(0)))
pre = np.empty((11, n, 8)); pre.fill(0)
print("trace_host (pinned pool)   %.1f ms" % tm(lambda: E.trace_host(low, rays, sel)))
print("trace_host into fresh np   %.1f ms" % tm(lambda: E.trace_host(low, rays, sel, out=np.empty((11, n, 8)))))
t0 = time.perf_counter(); h = system.ray_trace(rays, V, V); t1 = time.perf_counter()
print("System.ray_trace           %.1f ms (first pinned alloc of this size in this process? %s)" % ((t1 - t0) * 1e3, "no"))
del h
print("System.ray_trace repeated  %.1f ms" % tm(lambda: system.ray_trace(rays, V, V)))
print("trace_host into touched    %.1f ms" % tm(lambda: E.trace_host(low, rays, sel, out=pre)))
a = np.ones((11, n, 8)); b = np.empty_like(a); b.fill(0)
print("np.copyto 704MB (1 thread) %.1f ms" % tm(lambda: np.copyto(b, a)))
pin = torch.empty((11, n, 8), dtype=torch.float64, pin_memory=True)
d = torch.empty((11, n, 8), dtype=torch.float64, device="cuda:0")
print("D2H pinned 704MB (torch)   %.1f ms" % tm(lambda: (pin.copy_(d), torch.cuda.synchronize())))
pg = torch.empty((11, n, 8), dtype=torch.float64)
print("D2H pageable 704MB (torch) %.1f ms" % tm(lambda: (pg.copy_(d), torch.cuda.synchronize())))
