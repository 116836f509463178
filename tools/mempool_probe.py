"""How torch's caching allocator treats a MemPool whose segments come from librtpb (rtpb_torch_alloc /
rtpb_torch_free): reuse, Tensor.record_stream, memory statistics, empty_cache, out-of-memory, pool release,
and the C3 trace's rate into such memory vs torch.empty.  One process, prints one line per finding.

    python tools/mempool_probe.py [--timing]
"""
import argparse
import gc
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ray_trace_pb_amd import _engine as E  # noqa: E402

DEV = torch.device("cuda", 0)
GiB = 1 << 30


def say(*a):
    print(*a, flush=True)


def stats(tag):
    s = E.buffer_stats(0)
    say(f"  [{tag}] alloc={torch.cuda.memory_allocated(0) / GiB:.3f} GiB reserved="
        f"{torch.cuda.memory_reserved(0) / GiB:.3f} GiB free={torch.cuda.mem_get_info(0)[0] / GiB:.1f} GiB "
        f"segs={s['pool_segments']} seg_bytes={s['pool_bytes'] / GiB:.3f} made={s['segments_allocated']} "
        f"freed={s['segments_freed']} dead_va={s['dead_va_bytes'] / GiB:.2f} GiB")


def section(name, fn):
    say(f"== {name}")
    try:
        fn()
    except Exception as e:  # noqa: BLE001
        say(f"  EXCEPTION {type(e).__name__}: {e}")
    gc.collect()
    torch.cuda.synchronize()


def basic():
    stats("start")
    t = E.pool_empty((GiB // 4,), torch.float32, DEV)
    p = t.data_ptr()
    stats("1 GiB live")
    t.fill_(1.0)
    del t
    gc.collect()
    stats("freed")
    u = E.pool_empty((GiB // 4,), torch.float32, DEV)
    say(f"  same block again: {u.data_ptr() == p}")
    v = E.pool_empty((GiB // 8,), torch.float32, DEV)
    say(f"  a second, smaller tensor: new segment? ptr inside first={p <= v.data_ptr() < p + GiB}")
    stats("two live")
    del u, v


def record_stream():
    side = torch.cuda.Stream(DEV)
    t = E.pool_empty((GiB // 4,), torch.float32, DEV)
    p = t.data_ptr()
    side.wait_stream(torch.cuda.current_stream(DEV))
    with torch.cuda.stream(side):
        torch.cuda._sleep(300_000_000)
        t.fill_(3.0)
    t.record_stream(side)
    del t
    gc.collect()
    u = E.pool_empty((GiB // 4,), torch.float32, DEV)
    say(f"  next allocation while the side stream is pending: same block={u.data_ptr() == p}")
    u.fill_(4.0)
    torch.cuda.synchronize()
    say(f"  values survive: {bool((u == 4.0).all())}")
    stats("after record_stream")
    del u


def empty_cache():
    stats("before empty_cache")
    torch.cuda.empty_cache()
    stats("after torch.cuda.empty_cache")


def other_stream():
    a = torch.cuda.Stream(DEV)
    t = E.pool_empty((GiB // 4,), torch.float32, DEV, stream=a)
    p = t.data_ptr()
    del t
    gc.collect()
    u = E.pool_empty((GiB // 4,), torch.float32, DEV)
    say(f"  freed on stream A, allocated on the current stream: same block={u.data_ptr() == p}")
    stats("other stream")
    del u


def oom():
    torch.cuda.empty_cache()
    free = torch.cuda.mem_get_info(0)[0]
    n = int(free * 0.7)
    t = E.pool_empty((n,), torch.uint8, DEV)
    t[-1] = 1
    del t
    gc.collect()
    stats("70 % cached in the pool")
    try:
        r = torch.empty((n,), dtype=torch.uint8, device=DEV)
        r[-1] = 2
        say(f"  a regular allocation of the same size: OK (inside a pool segment: "
            f"{any(s['address'] <= r.data_ptr() < s['address'] + s['total_size'] for s in E.history_pool(0).snapshot())})")
        del r
    except torch.OutOfMemoryError as e:
        say(f"  a regular allocation of the same size: OOM ({str(e)[:120]})")
    stats("after regular allocation")


def release_pool():
    t = E.pool_empty((GiB // 4,), torch.float32, DEV)
    stats("live, before dropping the MemPool")
    pool = E._POOLS.pop(0)
    del pool
    gc.collect()
    stats("MemPool object dropped, tensor alive")
    t.fill_(5.0)
    torch.cuda.synchronize()
    say(f"  tensor still valid: {bool((t == 5.0).all())}")
    del t
    gc.collect()
    stats("tensor freed")
    torch.cuda.empty_cache()
    stats("empty_cache")
    u = E.pool_empty((GiB // 4,), torch.float32, DEV)
    stats("new pool, one tensor")
    del u


def timing():
    import ray_trace_pb_amd.materials as mat
    import ray_trace_pb_amd.raytrace as rt
    from ray_trace_pb_amd import _capi as C
    import systems
    system = systems.c3_system(rt, mat)
    nt, nph = 3163, 3162
    per = nt * nph
    rays = torch.empty((per * 5, 8), dtype=torch.float64, device=DEV)
    for k, h in enumerate(systems.C3_FIELDS):
        rt.fan_into(rays[k * per:(k + 1) * per], np.array([h, 0, 0]), np.pi / 180, nt, 0.635, nph)
    mats = [mat.Vacuum()] + list(system.materials) + [mat.Vacuum()]
    low = E.lower(system.surfaces, mats, lambda: np.array([0.635]), C.RTPB_F32)
    planes = E.resolve_planes("all", len(system.surfaces))
    shape = (len(planes), rays.shape[0], 8)
    bufs = {}
    for k in range(2):
        bufs[f"pool{k}"] = E.pool_empty(shape, torch.float32, DEV)
        bufs[f"shuffled{k}"] = E.history_buffer(shape, torch.float32, DEV)
    stats("timing buffers")
    st = torch.cuda.current_stream(DEV).cuda_stream
    res = {k: [] for k in bufs}
    for rnd in range(3):
        for k, b in bufs.items():
            E.trace_device(low, rays, planes, out=b, stream=st)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                E.trace_device(low, rays, planes, out=b, stream=st)
            e1.record()
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) / 5)
    for k, v in res.items():
        say(f"  {k}: {' '.join(f'{x:.3f}' for x in v)} ms")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--timing", action="store_true")
    args = ap.parse_args()
    torch.cuda.init()
    say(f"torch {torch.__version__} hip {torch.version.hip}")
    for name, fn in [("basic", basic), ("record_stream", record_stream), ("empty_cache", empty_cache),
                     ("other_stream", other_stream), ("oom", oom), ("release_pool", release_pool)]:
        t0 = time.perf_counter()
        section(name, fn)
        say(f"  ({time.perf_counter() - t0:.2f} s)")
    if args.timing:
        section("timing", timing)
    say("done")


if __name__ == "__main__":
    main()
