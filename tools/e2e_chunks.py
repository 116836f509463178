import os, sys, time
sys.path[:0] = ['/root/repo', '/root/repo/tests/golden']
import numpy as np, torch
import ray_trace_pb_amd.materials as mat, ray_trace_pb_amd.raytrace as rt
from ray_trace_pb_amd import _capi as C
import systems
system, rays = systems.c2_system(rt, mat), systems.c2_rays(1_000_000)
V = mat.Vacuum()
system.ray_trace(rays, V, V)
for mib in (8, 16, 32, 64, 128, 256):
    C.check(C.lib().rtpb_set_tuning(b"host_chunk_mib", mib))
    for planes in ("all", "final"):
        ts = []
        for _ in range(7):
            t0 = time.perf_counter(); out = system.ray_trace(rays, V, V, planes=planes); ts.append(time.perf_counter() - t0)
        print(f"chunk {mib:4d} MiB planes={planes}: {np.median(ts)*1e3:.2f} ms")
