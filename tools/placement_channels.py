"""Placement study, counter level: which memory channels does a slow C3 history buffer load?

One process allocates several C3-size histories (30.4 GB each; the history pool's shuffled 64 MiB chunks,
_engine.pool_empty), times the same trace into each (interleaved rounds, HIP events), then traces twice more into
the slowest and twice into the fastest.  Run under `rocprofv3 --pmc` with per-instance TCC counters
(TCC_EA0_WRREQ etc.: 16 channels x 8 XCDs) to compare the per-channel write traffic and stalls of the two
buffers; `--analyze DIR` reads rocprofv3's JSON output and this script's own log (its ORDER line names every trace
dispatch in launch order).

    rocprofv3 --pmc TCC_EA0_WRREQ TCC_EA0_WRREQ_DRAM_CREDIT_STALL ... --output-format json -d OUT -o pmc -- \\
        python3 tools/placement_channels.py --buffers 6 > OUT/run.log
    python3 tools/placement_channels.py --analyze OUT --log OUT/run.log
"""
import argparse
import collections
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
    """Per-instance counters from rocprofv3's JSON output (`--output-format json`): each dispatch's records hold one
    value per counter instance, in the order of the counter's `instances` list -- for the TCC_EA0_* counters 16
    channels (DIMENSION_INSTANCE) x 8 XCDs (DIMENSION_XCC), the channel varying fastest.  (The CSV output sums the
    instances; rocprofv3 -L did not accept derived per-slice counters through ROCPROFILER_METRICS_PATH, r05_j/k/l.)"""
    meta = order = None
    for line in open(args.log):
        if line.startswith("BUFFERS "):
            meta = json.loads(line[8:])
        elif line.startswith("ORDER "):
            order = json.loads(line[6:])
    paths = glob.glob(os.path.join(args.analyze, "**", "*results.json"), recursive=True)
    if not paths or meta is None or order is None:
        print("no JSON counter output or no BUFFERS / ORDER lines")
        return
    d = json.load(open(paths[0]))["rocprofiler-sdk-tool"][0]
    names = {k["kernel_id"]: k["truncated_kernel_name"] or k["kernel_name"] for k in d["kernel_symbols"]}
    counters = {c["id"]["handle"]: c for c in d["counters"]}
    rows = []
    for r in d["callback_records"]["counter_collection"]:
        info = r["dispatch_data"]["dispatch_info"]
        if "trace_kernel" not in names.get(info["kernel_id"], ""):
            continue
        per = collections.defaultdict(list)
        for rec in r["records"]:
            per[counters[rec["counter_id"]["handle"]]["name"]].append(rec["value"])
        rows.append((info["dispatch_id"], {k: np.array(v) for k, v in per.items()}))
    rows.sort(key=lambda x: x[0])
    print(f"{len(rows)} trace dispatches with counters, {len(order)} launches in ORDER; buffers {meta}")
    if len(rows) != len(order):
        print("cannot align dispatches with launches")
        return
    shape = {}
    for c in counters.values():
        dims = {dd["name"]: dd["instance_size"] for dd in c["dimensions"]}
        if set(dims) == {"DIMENSION_INSTANCE", "DIMENSION_XCC"}:
            shape[c["name"]] = (dims["DIMENSION_XCC"], dims["DIMENSION_INSTANCE"])
    for label, k in (("slow", meta["slow"]), ("fast", meta["fast"])):
        sel = [v for (_, v), b in zip(rows, order) if b == k][-2:]
        for c in sorted(sel[0]):
            a = np.mean([s[c] for s in sel], axis=0)
            m = max(a.mean(), 1e-30)
            print(f"{label} buffer {k} ({meta['ms'][k]:.3f} ms) {c}: per launch {a.sum():.4g}, over {a.size} instances "
                  f"cv {a.std() / m:.3f} min/mean {a.min() / m:.3f} max/mean {a.max() / m:.3f}")
            if c in shape and a.size == shape[c][0] * shape[c][1]:
                g = a.reshape(shape[c])                     # [xcc][channel]
                ch, xc = g.sum(0), g.sum(1)
                print(f"    per channel / mean (16, summed over XCDs): {np.round(ch / ch.mean(), 3).tolist()}")
                print(f"    per XCD / mean (8, summed over channels):  {np.round(xc / xc.mean(), 3).tolist()}")


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
