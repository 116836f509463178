"""Placement study, counter level: which memory channels does a slow C3 history buffer load?

One process allocates several C3-size histories (30.4 GB each; the history pool's shuffled 64 MiB chunks,
_engine.pool_empty), times the same trace into each (interleaved rounds, HIP events), then traces twice more into
the slowest and twice into the fastest.  Run under `rocprofv3 --pmc` with per-instance TCC counters
(TCC_EA0_WRREQ etc.: 16 channels x 8 XCDs) to compare the per-channel write traffic and stalls of the two
buffers; `--analyze DIR` reads the counter_collection CSV(s) and this script's own log (its ORDER line names
every trace dispatch in launch order).

    rocprofv3 --pmc TCC_EA0_WRREQ TCC_EA0_WRREQ_DRAM_CREDIT_STALL ... -d OUT -o pmc -- \\
        python3 tools/placement_channels.py --buffers 6 > OUT/run.log
    python3 tools/placement_channels.py --analyze OUT --log OUT/run.log
"""
import argparse
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]

import numpy as np  # noqa: E402


def run(args):
    import torch
    import ray_trace_pb_amd.materials as mat
    import ray_trace_pb_amd.raytrace as rt
    from ray_trace_pb_amd import _capi as C
    from ray_trace_pb_amd import _engine as E
    import systems
    dev = torch.device("cuda", 0)
    system = systems.c3_system(rt, mat)
    nt, nph = 3163, 3162
    per = nt * nph
    rays = torch.empty((per * 5, 8), dtype=torch.float64, device=dev)
    for k, h in enumerate(systems.C3_FIELDS):
        rt.fan_into(rays[k * per:(k + 1) * per], np.array([h, 0, 0]), np.pi / 180, nt, 0.635, nph)
    mats = [mat.Vacuum()] + list(system.materials) + [mat.Vacuum()]
    low = E.lower(system.surfaces, mats, lambda: np.array([0.635]), C.RTPB_F32)
    planes = E.resolve_planes("all", len(system.surfaces))
    shape = (len(planes), rays.shape[0], 8)
    bufs = [E.pool_empty(shape, torch.float32, dev) if args.kind == "pool" else
            E.history_buffer(shape, torch.float32, dev, chunk_bytes=64 << 20) for _ in range(args.buffers)]
    st = torch.cuda.current_stream(dev).cuda_stream
    order = []

    def launch(k):
        E.trace_device(low, rays, planes, out=bufs[k], stream=st)
        order.append(k)

    times = [[] for _ in bufs]
    for k in range(len(bufs)):
        launch(k)
    torch.cuda.synchronize()
    for _ in range(args.rounds):
        for k in range(len(bufs)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                launch(k)
            e1.record()
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / args.reps)
    med = [float(np.median(t)) for t in times]
    slow, fast = int(np.argmax(med)), int(np.argmin(med))
    for k in (slow, slow, fast, fast):
        launch(k)
    torch.cuda.synchronize()
    print("BUFFERS " + json.dumps({"ms": med, "slow": slow, "fast": fast,
                                   "ptr": [b.data_ptr() for b in bufs]}), flush=True)
    print("ORDER " + json.dumps(order), flush=True)


def analyze(args):
    meta = order = None
    for line in open(args.log):
        if line.startswith("BUFFERS "):
            meta = json.loads(line[8:])
        elif line.startswith("ORDER "):
            order = json.loads(line[6:])
    rows = collections.defaultdict(lambda: collections.defaultdict(dict))   # dispatch -> counter -> key -> value
    for f in glob.glob(os.path.join(args.analyze, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "trace_kernel" not in r.get("Kernel_Name", ""):
                continue
            key = tuple((k, r[k]) for k in sorted(r) if k.lower().startswith(("dimension", "instance", "xcc")))
            rows[int(r["Dispatch_Id"])][r["Counter_Name"]][key] = float(r["Counter_Value"])
    ids = sorted(rows)
    print(f"{len(ids)} trace dispatches with counters, {len(order or [])} launches in ORDER; buffers {meta}")
    if not ids or order is None or len(ids) != len(order):
        print("cannot align dispatches with launches")
        return
    for label, k in (("slow", meta["slow"]), ("fast", meta["fast"])):
        sel = [d for d, b in zip(ids, order) if b == k][-2:]
        # derived per-slice counters (tools/placement_counters.py): one vector per family, e.g. RTPB_WR_CH00..15
        fams = collections.defaultdict(list)
        for c in sorted(rows[sel[0]]):
            if c.startswith("RTPB_"):
                fams[c.rsplit("_", 1)[0] + "_" + "".join(ch for ch in c.rsplit("_", 1)[1] if not ch.isdigit())].append(c)
        for fam, names in sorted(fams.items()):
            v = np.array([np.mean([sum(rows[d][c].values()) for d in sel]) for c in names])
            m = max(v.mean(), 1e-30)
            print(f"{label} buffer {k} ({meta['ms'][k]:.3f} ms) {fam}: sum={v.sum():.4g} cv={v.std() / m:.3f} "
                  f"max/mean={v.max() / m:.3f} min/mean={v.min() / m:.3f} per-slice/mean={np.round(v / m, 3).tolist()}")
        for c in sorted(rows[sel[0]]):
            v = np.array([[rows[d][c][key] for key in sorted(rows[d][c])] for d in sel]).mean(axis=0)
            desc = f"n={v.size} sum={v.sum():.4g}"
            if v.size > 1:
                desc += (f" mean={v.mean():.4g} cv={v.std() / max(v.mean(), 1e-30):.3f} max/mean="
                         f"{v.max() / max(v.mean(), 1e-30):.3f} min/mean={v.min() / max(v.mean(), 1e-30):.3f}")
                if v.size == 128:
                    # 8 XCDs x 16 channels in the CSV's key order: per-channel totals over the XCDs and per-XCD totals
                    desc += f" top5={np.round(np.sort(v)[-5:] / v.mean(), 3).tolist()}"
            print(f"{label} buffer {k} ({meta['ms'][k]:.3f} ms) {c}: {desc}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--buffers", type=int, default=6)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--kind", default="pool", choices=["pool", "legacy"])
    ap.add_argument("--analyze", default="")
    ap.add_argument("--log", default="")
    args = ap.parse_args()
    if args.analyze:
        analyze(args)
    else:
        run(args)


if __name__ == "__main__":
    main()
