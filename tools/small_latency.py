"""Per-call latency of small traces (the reference's typical script usage: ~1k rays per call)."""
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


def tm(fn, reps=50):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e6


system, rays, m0, m1 = systems.c1_plano_convex(rt, mat)
mats = [m0] + list(system.materials) + [m1]
print("C1 ray_trace numpy (1001 rays)      %8.1f us" % tm(lambda: system.ray_trace(rays, m0, m1)))
print("  lower()                           %8.1f us" % tm(lambda: E.lower(system.surfaces, mats, lambda: None, 0)))
low = E.lower(system.surfaces, mats, lambda: None, 0)
sel = E.resolve_planes("all", 3)
print("  plan_for() (cache hit)            %8.1f us" % tm(lambda: E.plan_for(low)))
print("  trace_host()                      %8.1f us" % tm(lambda: E.trace_host(low, rays, sel)))
x = torch.from_numpy(rays).cuda()
print("C1 ray_trace torch (1001 rays)      %8.1f us" % tm(lambda: (system.ray_trace(x, m0, m1), torch.cuda.synchronize())))
print("auto_focus ray-fan (3 rays)         %8.1f us" % tm(lambda: system.auto_focus(0.5, m0, m1, mode="collimated")))
s2 = systems.c2_system(rt, mat)
r2 = systems.c2_rays(1000)
print("C2 ray_trace numpy (1000 rays)      %8.1f us" % tm(lambda: s2.ray_trace(r2, mat.Vacuum(), mat.Vacuum())))
