"""Wall time per back-to-back trace launch (C2, 1M rays, f64 full history) with and without the
per-launch timing events, and replayed from a captured HIP graph -- how much of bench.py's
ms_per_step is launch/dispatch overhead rather than kernel time."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ray_trace_pb_amd.materials as mat  # noqa: E402
import ray_trace_pb_amd.raytrace as rt  # noqa: E402
from ray_trace_pb_amd import _capi as C  # noqa: E402
from ray_trace_pb_amd import _engine as E  # noqa: E402
import systems  # noqa: E402


def main(steps=400):
    dev = torch.device("cuda:0")
    system = systems.c2_system(rt, mat)
    rays_np = systems.c2_rays(1_000_000)
    S = len(system.surfaces)
    low = E.lower(system.surfaces, [mat.Vacuum()] + list(system.materials) + [mat.Vacuum()],
                  lambda: np.unique(rays_np[:, 7]), C.RTPB_F64)
    x = torch.from_numpy(rays_np).to(dev)
    sel = E.resolve_planes("all", S)
    out = torch.empty((len(sel), x.shape[0], 8), dtype=torch.float64, device=dev)
    lib = C.lib()
    plan = E.plan_for(low)
    lo, hi = E.plane_mask(sel)
    n = x.shape[0]

    def raw(stream):
        C.check(lib.rtpb_trace(plan, 0, x.data_ptr(), E.input_code(x.dtype), n, C.RTPB_AOS, 0, out.data_ptr(), C.RTPB_AOS, 8 * n, n,
                               lo, hi, stream))

    def wall(fn, k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k * 1e3

    s = torch.cuda.current_stream().cuda_stream
    res = {}
    for _ in range(20):
        raw(s)
    res["engine.trace_device, no events"] = wall(lambda: E.trace_device(low, x, sel, out=out), steps)
    res["raw rtpb_trace, no events"] = wall(lambda: raw(s), steps)
    lib.rtpb_timing_enable(1)
    res["raw rtpb_trace, timing events"] = wall(lambda: raw(s), steps)
    tot, cnt = ctypes.c_double(), ctypes.c_int64()
    C.check(lib.rtpb_timing_collect(ctypes.byref(tot), ctypes.byref(cnt)))
    lib.rtpb_timing_enable(0)
    res["  (event kernel avg)"] = tot.value / cnt.value
    # graph of 10 launches
    g = torch.cuda.CUDAGraph()
    cs = torch.cuda.Stream()
    cs.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(cs):
        raw(cs.cuda_stream)
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=cs):
        for _ in range(10):
            raw(cs.cuda_stream)
    torch.cuda.synchronize()
    res["graph replay (per launch)"] = wall(g.replay, steps // 10) / 10
    for k, v in res.items():
        print(f"{k:36s} {v:.4f} ms")


if __name__ == "__main__":
    main()
