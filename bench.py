"""Benchmark: ray-surface intersections/s of System.ray_trace on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): Thorlabs AC508-100-B achromat system -- flat,
3-surface doublet (N-LAK22 / N-SF6HT Sellmeier glasses), flat at the paraxial focus: S = 5 surfaces --
1,000,000 rays per GPU at 3 wavelengths {0.7065, 0.855, 1.015} um, float64, full drop-in history
(2S+1 = 11 planes of (N, 8) float64).  A step = one trace of the GPU's bundle, inputs and outputs
resident in HBM.  Multi-GPU: one process per GPU (torchrun), each traces its own 1M-ray bundle (rays are
independent: no data-path collective) -> weak scaling; the step time is the max over ranks.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

Rank 0 prints ONE JSON line with the metric, a `roofline` object for the trace kernel (algorithmic
bytes / average launch duration from HIP events on the launch stream around the timed launches; optionally the
PMC-measured HBM traffic) and a `cpu_baseline` object (the NumPy port of the reference, timed on this
host on a bounded sample, N=1 only).
"""
import argparse
import json
import os
import shutil
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]

import numpy as np  # noqa: E402

METRIC = "ray-surface intersections/sec at 1/2/4/8 MI355X; achieved HBM GB/s vs peak"
UNIT = "ray-surface intersections/s"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
SEED = 20241008


def shard_seed(rank):
    return SEED + 7919 * rank


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--rays", type=int, default=1_000_000, help="rays per GPU")
    ap.add_argument("--dtype", default="float64", choices=["float64", "float32"])
    ap.add_argument("--planes", default="all", choices=["all", "final"])
    ap.add_argument("--layout", default="aos", choices=["aos", "soa"])
    ap.add_argument("--cpu-baseline", default="auto", choices=["auto", "off"])
    ap.add_argument("--cpu-rays", type=int, default=1_000_000)
    ap.add_argument("--traffic", default="auto", choices=["auto", "off"],
                    help="measure HBM bytes with a separate rocprofv3 --pmc child run (rank 0, N=1)")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args()


def dist_env():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), int(os.environ.get("LOCAL_RANK", 0))


def build_workload(rt, mat, n_rays, rank):
    import systems
    system = systems.c2_system(rt, mat)
    rays = systems.c2_rays(n_rays, seed=shard_seed(rank))
    return system, rays, mat.Vacuum(), mat.Vacuum()


def cpu_baseline(n_rays):
    """The reference's algorithm as NumPy (oracle/rt_numpy.py with the reference's history
    re-concatenation), 1 process, on the same C2 system and bundle shape."""
    import ray_trace_pb_amd.materials as mat
    import ray_trace_pb_amd.raytrace as rt
    from oracle import rt_numpy as O
    from serialize import material_to_dict, surface_to_dict
    system, rays, m0, m1 = build_workload(rt, mat, n_rays, 0)
    S = [surface_to_dict(s) for s in system.surfaces]
    M = [material_to_dict(m) for m in [m0] + list(system.materials) + [m1]]
    reps, t_total = 0, 0.0
    while reps < 2 or t_total < 8.0:
        t0 = time.perf_counter()
        O.ray_trace(S, M, rays, reference_costs=True)
        t_total += time.perf_counter() - t0
        reps += 1
        if reps >= 6:
            break
    rate = reps * n_rays * len(S) / t_total
    return {"value": rate, "unit": UNIT, "cores": 1, "kind": "port",
            "sample": f"C2 system, {n_rays} rays x {reps} passes, float64 full history, 1 process "
                      f"(oracle/rt_numpy.py, reference_costs=True), {t_total:.1f} s",
            "cpu_model": cpu_model()}


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_worker(args):
    """One process of the parallel CPU baseline: trace ray shard [lo, hi) repeatedly for ~`secs`."""
    lo, hi, n_rays, secs = args
    import ray_trace_pb_amd.materials as mat
    import ray_trace_pb_amd.raytrace as rt
    from oracle import rt_numpy as O
    from serialize import material_to_dict, surface_to_dict
    system, rays, m0, m1 = build_workload(rt, mat, n_rays, 0)
    S = [surface_to_dict(s) for s in system.surfaces]
    M = [material_to_dict(m) for m in [m0] + list(system.materials) + [m1]]
    shard = np.ascontiguousarray(rays[lo:hi])
    O.ray_trace(S, M, shard[:64], reference_costs=True)
    passes, t0 = 0, time.perf_counter()
    while passes < 1 or time.perf_counter() - t0 < secs:
        O.ray_trace(S, M, shard, reference_costs=True)
        passes += 1
    return passes * (hi - lo) * len(S), time.perf_counter() - t0


def cpu_baseline_parallel(n_rays, procs, secs=4.0):
    """SURVEY §8d mode (ii): `procs` single-threaded processes on contiguous shards of the bundle."""
    import multiprocessing as mp
    bounds = [(n_rays * k // procs, n_rays * (k + 1) // procs, n_rays, secs) for k in range(procs)]
    env_old = os.environ.get("OMP_NUM_THREADS")
    os.environ["OMP_NUM_THREADS"] = "1"
    try:
        # spawn (fork + exec in the child): never fork a process that has initialised the GPU
        with mp.get_context("spawn").Pool(procs) as pool:
            res = pool.map(_cpu_worker, bounds)
    finally:
        if env_old is None:
            os.environ.pop("OMP_NUM_THREADS", None)
        else:
            os.environ["OMP_NUM_THREADS"] = env_old
    units = sum(u for u, _ in res)
    return {"value": units / max(t for _, t in res), "unit": UNIT, "cores": procs, "kind": "port",
            "sample": f"C2 system, {n_rays} rays split over {procs} processes, ~{secs:.0f} s each"}


def measure_traffic(args):
    """HBM bytes per trace launch from rocprofv3 PMC counters (separate child run, FETCH_SIZE and
    WRITE_SIZE in separate passes; gfx950: FETCH_SIZE counts half the bytes of wide streaming reads,
    so it is doubled -- MI355X_MICROARCH.md §HBM)."""
    prof = shutil.which("rocprofv3")
    if not prof:
        return None, "rocprofv3 not found"
    out = {}
    outdir = os.path.join(ROOT, "gpurun_out", "bench_pmc")
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = os.path.join(outdir, ctr)
        shutil.rmtree(d, ignore_errors=True)
        cmd = [prof, "--pmc", ctr, "--output-format", "csv", "-d", d, "-o", "pmc", "--",
               sys.executable, os.path.abspath(__file__), "--pmc-child", "--rays", str(args.rays),
               "--dtype", args.dtype, "--planes", args.planes, "--layout", args.layout]
        try:
            subprocess.run(cmd, check=True, timeout=300, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                           env=dict(os.environ, TMPDIR="/tmp"))
        except Exception as e:  # noqa: BLE001
            return None, f"rocprofv3 {ctr} failed: {e}"
        vals = []
        for dp, _, files in os.walk(d):
            for f in files:
                if f.endswith("counter_collection.csv"):
                    import csv
                    with open(os.path.join(dp, f)) as fh:
                        for row in csv.DictReader(fh):
                            if "trace_kernel" in row.get("Kernel_Name", "") and row.get("Counter_Name") == ctr:
                                vals.append(float(row["Counter_Value"]))
        if not vals:
            return None, f"no {ctr} rows"
        out[ctr] = float(np.median(vals))
    # counters are in KiB units
    return (2.0 * out["FETCH_SIZE"] + out["WRITE_SIZE"]) * 1024.0, None


def main():
    args = parse()
    rank, world, local = dist_env()
    import torch
    import ray_trace_pb_amd.materials as mat
    import ray_trace_pb_amd.raytrace as rt
    from ray_trace_pb_amd import _capi as C
    from ray_trace_pb_amd import _engine as E

    # one GPU per rank; the modulo only matters when rehearsing several ranks on one GPU
    dev = torch.device("cuda", local % max(torch.cuda.device_count(), 1))
    torch.cuda.set_device(dev)
    if world > 1:
        # Control plane only (barriers + one max-reduction of the step time): rays are independent, so
        # the trace has no data-path exchange and needs no RCCL communicator.
        import torch.distributed as dist
        dist.init_process_group("gloo")

    system, rays_np, m0, m1 = build_workload(rt, mat, args.rays, rank)
    S = len(system.surfaces)
    code = C.RTPB_F64 if args.dtype == "float64" else C.RTPB_F32
    tdt = torch.float64 if code == C.RTPB_F64 else torch.float32
    w = 8 if code == C.RTPB_F64 else 4
    rays = torch.from_numpy(rays_np).to(dev, dtype=tdt)
    mats = [m0] + list(system.materials) + [m1]
    low = E.lower(system.surfaces, mats, lambda: np.unique(rays_np[:, 7]), code)
    planes = E.resolve_planes(args.planes, S)
    layout = C.RTPB_AOS if args.layout == "aos" else C.RTPB_SOA
    out_shape = (len(planes), args.rays, 8) if layout == C.RTPB_AOS else (len(planes), 8, args.rays)
    out = torch.empty(out_shape, dtype=tdt, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def step():
        E.trace_device(low, rays, planes, layout_out=layout, out=out, stream=stream)

    if args.pmc_child:
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        return

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # HIP events on the launch stream (torch's current stream, which step() launches on) bracket the K
    # back-to-back launches: their elapsed time / K is the average launch duration.  (Per-launch event
    # pairs would insert ~6 us of marker work between kernels -- measured by tools/launch_overhead.py.)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        step()
    ev1.record()
    torch.cuda.synchronize()
    # each rank's own clock stops at its device sync; the job time is the max over ranks (all_reduce
    # below), so the closing barrier's own latency (gloo over loopback, ~0.1-0.5 ms) is not charged
    # to the K steps -- it would dominate at the driver's small K
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    kernel_ms = ev0.elapsed_time(ev1) / args.steps

    # the same output buffer written by a plain fill (one contiguous stream): the delivered write rate of
    # this placement, for context (the multi-plane history is placement-sensitive, fill is not)
    if rank == 0:
        out.fill_(0.0)
        f0, f1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        f0.record()
        for _ in range(10):
            out.fill_(0.0)
        f1.record()
        torch.cuda.synchronize()
        fill_ms = f0.elapsed_time(f1) / 10
        fill_gbs = out.numel() * out.element_size() / (fill_ms * 1e-3) / 1e9

    if world > 1:
        t = torch.tensor([elapsed, kernel_ms], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kernel_ms_max = t.tolist()
    else:
        kernel_ms_max = kernel_ms

    total_units = world * args.rays * S * args.steps
    value = total_units / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    # algorithmic bytes per launch: read the input record once, write every stored plane once
    bytes_per_ray = 8 * w * (1 + len(planes))
    alg_bytes = args.rays * bytes_per_ray
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9

    if rank == 0:
        traffic = None
        traffic_note = None
        if world == 1 and args.traffic == "auto":
            tb, err = measure_traffic(args)
            traffic = tb
            traffic_note = err
        cpu = None
        if world == 1 and args.cpu_baseline == "auto":
            cpu = cpu_baseline(args.cpu_rays)
            try:
                procs = max(1, min(16, len(os.sched_getaffinity(0))))
                cpu["parallel"] = cpu_baseline_parallel(args.cpu_rays, procs)
            except Exception as e:  # noqa: BLE001 -- the single-process baseline stands on its own
                cpu["parallel"] = {"error": repr(e)}
        line = {
            "metric": METRIC, "value": value, "unit": UNIT, "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64" if code == C.RTPB_F64 else "f32", "data": "synthetic",
            "config": {"workload": "C2: AC508-100-B achromat system (flat + N-LAK22/N-SF6HT doublet + focal flat, "
                                   "S=5), collimated rays in a 10 mm disk at 3 wavelengths",
                       "rays_per_gpu": args.rays, "surfaces": S, "planes_stored": len(planes),
                       "layout": args.layout, "parallelism": f"ray shards x{world} (no collective)"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": (traffic / 1.0) if traffic is not None else None,
                         "kernel": "trace_kernel", "kernel_ms_avg": kernel_ms, "kernel_ms_max_rank": kernel_ms_max,
                         "kernel_ms_method": "HIP events on the launch stream around the K launches / K",
                         "alg_bytes_per_launch": alg_bytes, "alg_bytes_per_ray_surface": bytes_per_ray / S,
                         "output_fill_GBps": fill_gbs, "frac_of_output_fill": achieved / fill_gbs},
            "cpu_baseline": cpu,
        }
        if traffic_note:
            line["roofline"]["traffic_note"] = traffic_note
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
