"""Streaming history writer throughput: K device-traced C2 histories written to a
zarr-v2 store by io.HistoryWriter (pinned async D2H + writer thread), vs tracing alone.

    python tools/bench_writer.py [--configs K] [--rays N] [--dir /tmp/rtpb_writer]
    python tools/bench_writer.py --compressor zlib --chunk-rays 65536 --workers 16     # zlib chunks, 16 threads
"""
import argparse
import json
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ray_trace_pb_amd.materials as mat  # noqa: E402
import ray_trace_pb_amd.raytrace as rt  # noqa: E402
from ray_trace_pb_amd import io as rio  # noqa: E402
import systems  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", type=int, default=8)
    ap.add_argument("--rays", type=int, default=250_000)
    ap.add_argument("--dir", default="/tmp/rtpb_writer")
    ap.add_argument("--compressor", default=None, help="none (default) or zlib[:level]")
    ap.add_argument("--chunk-rays", type=int, default=None)
    ap.add_argument("--workers", type=int, default=None)
    args = ap.parse_args()
    comp = None
    if args.compressor and args.compressor != "none":
        name, _, level = args.compressor.partition(":")
        comp = (name, int(level or 1))
    dev = torch.device("cuda:0")
    system = systems.c2_system(rt, mat)
    x = torch.from_numpy(systems.c2_rays(args.rays)).to(dev)
    P = 2 * len(system.surfaces) + 1
    system.ray_trace(x, mat.Vacuum(), mat.Vacuum())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.configs):
        system.ray_trace(x, mat.Vacuum(), mat.Vacuum())
    torch.cuda.synchronize()
    t_trace = time.perf_counter() - t0
    shutil.rmtree(args.dir, ignore_errors=True)
    t0 = time.perf_counter()
    with rio.HistoryWriter(args.dir, args.configs, P, args.rays, attrs={"workload": "C2"}, compressor=comp,
                           chunk_rays=args.chunk_rays, workers=args.workers) as w:
        for k in range(args.configs):
            w.write(k, system.ray_trace(x, mat.Vacuum(), mat.Vacuum()))
    t_total = time.perf_counter() - t0
    nbytes = args.configs * P * args.rays * 64
    stored = sum(os.path.getsize(os.path.join(args.dir, "rays", f)) for f in os.listdir(os.path.join(args.dir, "rays"))
                 if not f.startswith("."))
    back = rio.read_array(args.dir)
    ok = np.array_equal(back[-1], system.ray_trace(x, mat.Vacuum(), mat.Vacuum()).cpu().numpy(), equal_nan=True)
    shutil.rmtree(args.dir, ignore_errors=True)
    print(json.dumps({"configs": args.configs, "rays": args.rays, "planes": P, "bytes": nbytes,
                      "trace_only_s": t_trace, "trace_and_write_s": t_total,
                      "write_GBps": nbytes / t_total / 1e9, "readback_exact": bool(ok),
                      "compressor": comp, "chunk_rays": args.chunk_rays, "stored_bytes": stored,
                      "ratio": nbytes / max(stored, 1)}))


if __name__ == "__main__":
    main()
