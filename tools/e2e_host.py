"""End-to-end NumPy path (what a drop-in user calls): host rays in, host history out, PCIe included.
Also write-only / copy bandwidth references on the device."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ray_trace_pb_amd.materials as mat  # noqa: E402
import ray_trace_pb_amd.raytrace as rt  # noqa: E402
import systems  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
system, rays = systems.c2_system(rt, mat), systems.c2_rays(n)
V = mat.Vacuum()
out = system.ray_trace(rays, V, V)            # warm (plan, allocations)
for planes in ("all", "final"):
    ts = []
    for _ in range(15):
        t0 = time.perf_counter()
        out = system.ray_trace(rays, V, V, planes=planes)
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    print(f"numpy e2e planes={planes}: median {t * 1e3:.1f} ms (min {min(ts) * 1e3:.1f}) -> {n * 5 / t:.3g} "
          f"ray-surf/s, host bytes {(rays.nbytes + out.nbytes) / t / 1e9:.1f} GB/s")
dev = torch.device("cuda:0")
buf = torch.empty(88_000_000, dtype=torch.float64, device=dev)
src = torch.empty(96_000_000, dtype=torch.float64, device=dev)
dst = torch.empty_like(src)
for name, fn, nbytes in (("fill 704MB (write only)", lambda: buf.fill_(1.0), buf.numel() * 8),
                         ("copy 768MB (r+w)", lambda: dst.copy_(src), 2 * src.numel() * 8)):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(f"{name}: {ms:.4f} ms -> {nbytes / ms / 1e6:.0f} GB/s")
