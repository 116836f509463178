"""Benchmark: ray-surface intersections/s of System.ray_trace on MI355X (BASELINE.json metric).

Headline workload (BASELINE.json configs[2], the largest single-GPU config): the 4f
relay of scripts/2024_08_08_achromat_imaging.py:13-70 -- object flat, two Thorlabs AC508-075-A-ML
doublets (Ebaf11 / N-SF11), pupil flat, image flat: S = 9 surfaces -- traced with 5 field points
h in {0, 4, 8, 12, 16} mm x get_ray_fan(h, 1 deg, 3163, 0.635 um, nphis=3162) = 50,007,030 rays per GPU,
the full drop-in history (2S+1 = 19 planes) stored as float32 (BASELINE precision; arithmetic float64,
input rays float64 as the generator makes them, so the history is the reference's rounded once).  A step
= one System.ray_trace of the GPU's bundle, inputs and outputs resident in HBM.  Multi-GPU: one process
per GPU (torchrun), each traces its own bundle (rays are independent: no data-path collective) -> weak
scaling; the job time is the max over ranks.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2]
    torchrun --nproc-per-node N bench.py --gpus N ...

Rank 0 prints ONE JSON line with the metric, a `roofline` object for the trace kernel (algorithmic bytes /
average launch duration from HIP events on the launch stream around the timed launches; the PMC-measured
HBM bytes per launch from a separate rocprofv3 child), per-rank kernel times (N>1), a secondary object
for BASELINE configs[1] (C2: AC508-100-B achromat, 1M rays, float64), and a `cpu_baseline` object:
oracle/rt_refcost.py (the reference's algorithm and data flow, calibrated against the reference in
tests/golden/cpu_calibration.json) timed on this host on a bounded sample of the same workload, plus
C1 (BASELINE configs[0], the plano-convex CPU case) -- N=1 only.
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
C3_FAN = (3163, 3162)          # scripts/2024_08_08_achromat_imaging.py fan at 10M rays per field
C3_CPU_FAN = (448, 447)        # CPU-baseline sample of C3: 5 fields x 200,256 rays


def shard_seed(rank):
    return SEED + 7919 * rank


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c3", choices=["c3", "c2"])
    ap.add_argument("--scale", type=float, default=1.0, help="c3: fraction of the per-axis fan sizes")
    ap.add_argument("--rays", type=int, default=1_000_000, help="c2: rays per GPU")
    ap.add_argument("--secondary", default="auto", choices=["auto", "off"], help="C2 float64 object (N=1)")
    ap.add_argument("--cpu-baseline", default="auto", choices=["auto", "off"])
    ap.add_argument("--traffic", default="auto", choices=["auto", "off"],
                    help="measure HBM bytes with separate rocprofv3 --pmc child runs (rank 0, N=1)")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args()


def dist_env():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), int(os.environ.get("LOCAL_RANK", 0))


class Workload:
    """One BASELINE config on one GPU: system, device-resident input rays, output history buffer."""

    def __init__(self, config, dev, rank, scale=1.0, c2_rays=1_000_000):
        import torch
        import ray_trace_pb_amd.materials as mat
        import ray_trace_pb_amd.raytrace as rt
        from ray_trace_pb_amd import _capi as C
        from ray_trace_pb_amd import _engine as E
        import systems
        self.config = config
        if config == "c3":
            self.system, self.m0, self.m1 = systems.c3_system(rt, mat), mat.Vacuum(), mat.Vacuum()
            nt, nph = int(C3_FAN[0] * scale), int(C3_FAN[1] * scale)
            per = nt * nph
            self.rays = torch.empty((per * len(systems.C3_FIELDS), 8), dtype=torch.float64, device=dev)
            for k, h in enumerate(systems.C3_FIELDS):       # generated in HBM, bit-identical to get_ray_fan
                rt.fan_into(self.rays[k * per:(k + 1) * per], np.array([h, 0, 0]), np.pi / 180, nt, 0.635, nph)
            self.code = C.RTPB_F32
            self.workload = (f"C3: 4f relay of scripts/2024_08_08_achromat_imaging.py:13-70 (flat + 2x AC508-075-A-ML "
                             f"Ebaf11/N-SF11 doublet + pupil flat + image flat, S=9), 5 fields h=0..16 mm x "
                             f"get_ray_fan(h, 1 deg, {nt}, 0.635 um, nphis={nph}), full 19-plane history")
            self.storage = "f32 history (float64 input rays, float64 arithmetic)"
            wl_keys = np.array([0.635])
        else:
            self.system, self.m0, self.m1 = systems.c2_system(rt, mat), mat.Vacuum(), mat.Vacuum()
            rays_np = systems.c2_rays(c2_rays, seed=shard_seed(rank))
            self.rays = torch.from_numpy(rays_np).to(dev)
            self.code = C.RTPB_F64
            self.workload = ("C2: AC508-100-B achromat system of scripts/2022_08_04_ACT508-100-B.py (flat + "
                             "N-LAK22/N-SF6HT doublet + focal flat, S=5), collimated rays in a 10 mm disk at 3 "
                             "wavelengths, full 11-plane history")
            self.storage = "f64"
            wl_keys = np.unique(rays_np[:, 7])
        self.S = len(self.system.surfaces)
        self.n = self.rays.shape[0]
        mats = [self.m0] + list(self.system.materials) + [self.m1]
        self.low = E.lower(self.system.surfaces, mats, lambda: wl_keys, self.code)
        self.planes = E.resolve_planes("all", self.S)
        w = 8 if self.code == C.RTPB_F64 else 4
        self.out = torch.empty((len(self.planes), self.n, 8), dtype=torch.float64 if w == 8 else torch.float32,
                               device=dev)
        self.stream = torch.cuda.current_stream(dev).cuda_stream
        # algorithmic bytes per launch: read each input record once (float64), write every stored plane once
        self.bytes_per_ray = 8 * self.rays.element_size() + 8 * w * len(self.planes)
        self.alg_bytes = self.n * self.bytes_per_ray
        self._E = E

    def step(self):
        self._E.trace_device(self.low, self.rays, self.planes, out=self.out, stream=self.stream)

    def timed(self, steps):
        """Average launch duration (ms) from HIP events on the launch stream around `steps` launches, and
        the host wall time of the whole run (s)."""
        import torch
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record()
        for _ in range(steps):
            self.step()
        ev1.record()
        torch.cuda.synchronize()
        return ev0.elapsed_time(ev1) / steps, time.perf_counter() - t0

    def fill_rate(self):
        """The output buffer's delivered plain-write rate (GB/s, torch fill_): context for the history's
        multi-plane write pattern, which is placement-sensitive."""
        import torch
        flat = self.out.view(-1)
        # chunks below 2^31 elements keep torch on its vectorised fill kernel
        chunks = [flat[k:k + (1 << 30)] for k in range(0, flat.numel(), 1 << 30)]
        for c in chunks:
            c.fill_(0.0)
        f0, f1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        f0.record()
        for _ in range(5):
            for c in chunks:
                c.fill_(0.0)
        f1.record()
        torch.cuda.synchronize()
        return self.out.numel() * self.out.element_size() / (f0.elapsed_time(f1) / 5 * 1e-3) / 1e9


def stream_copy_rate(device, nbytes=4 << 30, reps=10):
    """Measured copy rate of the device (GB/s, read + write bytes of a torch copy_ between two fresh
    `nbytes` buffers): the measured stream-copy figure SURVEY §8(d) asks for beside the 8 TB/s spec.  It is
    torch's elementwise copy kernel, not a tuned one (4.7 TB/s on MI355X, below the trace kernel's own
    rate), so `frac` stays priced against the spec peak."""
    import torch
    src = torch.ones(nbytes // 8, dtype=torch.float64, device=device)
    dst = torch.empty_like(src)
    dst.copy_(src)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        dst.copy_(src)
    e1.record()
    torch.cuda.synchronize()
    rate = 2 * nbytes / (e0.elapsed_time(e1) / reps * 1e-3) / 1e9
    del src, dst
    torch.cuda.empty_cache()
    return rate


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_bundle(config):
    import ray_trace_pb_amd.materials as mat
    import ray_trace_pb_amd.raytrace as rt
    from serialize import material_to_dict, surface_to_dict
    import systems
    if config == "c3":
        system, rays, m0, m1 = systems.c3_system(rt, mat), systems.c3_rays(rt, *C3_CPU_FAN), mat.Vacuum(), mat.Vacuum()
        label = f"C3 system, 5 fields x fan {C3_CPU_FAN[0]}x{C3_CPU_FAN[1]} ({rays.shape[0]} rays)"
    elif config == "c2":
        system, rays, m0, m1 = systems.c2_system(rt, mat), systems.c2_rays(1_000_000), mat.Vacuum(), mat.Vacuum()
        label = "C2 system, 1,000,000 rays"
    else:
        system, rays, m0, m1 = systems.c1_plano_convex(rt, mat)
        label = "C1 plano-convex (BASELINE configs[0]), 1,001 rays, the whole config"
    S = [surface_to_dict(s) for s in system.surfaces]
    M = [material_to_dict(m) for m in [m0] + list(system.materials) + [m1]]
    return S, M, rays, label


def cpu_time(config, min_s):
    """The reference-cost port (oracle/rt_refcost.py), 1 process: rate over >= min_s seconds."""
    from oracle import rt_refcost as RC
    S, M, rays, label = _cpu_bundle(config)
    RC.ray_trace(S, M, rays[:64])
    reps, t = 0, 0.0
    while reps < 1 or t < min_s:
        t0 = time.perf_counter()
        RC.ray_trace(S, M, rays)
        t += time.perf_counter() - t0
        reps += 1
    return {"value": reps * rays.shape[0] * len(S) / t, "unit": UNIT, "cores": 1, "kind": "port",
            "sample": f"{label} x {reps} passes, float64 full history, 1 process, {t:.1f} s "
                      f"(oracle/rt_refcost.py: the reference's algorithm and data flow)"}


def _cpu_worker(args):
    """One process of the parallel CPU baseline: trace ray shard [lo, hi) of the sample for ~`secs`."""
    config, lo, hi, secs = args
    from oracle import rt_refcost as RC
    S, M, rays, _ = _cpu_bundle(config)
    shard = np.ascontiguousarray(rays[lo:hi])
    RC.ray_trace(S, M, shard[:64])
    passes, t0 = 0, time.perf_counter()
    while passes < 1 or time.perf_counter() - t0 < secs:
        RC.ray_trace(S, M, shard)
        passes += 1
    return passes * (hi - lo) * len(S), time.perf_counter() - t0


def cpu_parallel(config, procs, secs=4.0):
    """SURVEY §8d mode (ii): `procs` single-threaded processes on contiguous shards of the sample."""
    import multiprocessing as mp
    _, _, rays, label = _cpu_bundle(config)
    n = rays.shape[0]
    bounds = [(config, n * k // procs, n * (k + 1) // procs, secs) for k in range(procs)]
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
            "sample": f"{label} split over {procs} processes, ~{secs:.0f} s each"}


def measure_traffic(args, config):
    """HBM bytes per trace launch from rocprofv3 PMC counters (separate child runs, FETCH_SIZE and
    WRITE_SIZE in separate passes; gfx950: FETCH_SIZE counts half the bytes of wide streaming reads, so
    it is doubled -- MI355X_MICROARCH.md §HBM)."""
    prof = shutil.which("rocprofv3")
    if not prof:
        return None, "rocprofv3 not found"
    out = {}
    outdir = os.path.join(ROOT, "gpurun_out", "bench_pmc", config)
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = os.path.join(outdir, ctr)
        shutil.rmtree(d, ignore_errors=True)
        cmd = [prof, "--pmc", ctr, "--output-format", "csv", "-d", d, "-o", "pmc", "--",
               sys.executable, os.path.abspath(__file__), "--pmc-child", "--config", config,
               "--scale", str(args.scale), "--rays", str(args.rays)]
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


def roofline(wl, kernel_ms, traffic=None, traffic_note=None, fill=None, copy=None):
    achieved = wl.alg_bytes / (kernel_ms * 1e-3) / 1e9
    r = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
         "traffic": traffic, "kernel": "trace_kernel", "kernel_ms_avg": kernel_ms,
         "kernel_ms_method": "HIP events on the launch stream around the K launches / K",
         "alg_bytes_per_launch": wl.alg_bytes, "alg_bytes_per_ray": wl.bytes_per_ray,
         "alg_bytes_per_ray_surface": wl.bytes_per_ray / wl.S}
    if fill:
        r.update(output_fill_GBps=fill, frac_of_output_fill=achieved / fill)
    if copy:
        r.update(torch_copy_GBps=copy, frac_of_torch_copy=achieved / copy)
    if traffic_note:
        r["traffic_note"] = traffic_note
    return r


def main():
    args = parse()
    rank, world, local = dist_env()
    import torch

    # one GPU per rank; the modulo only matters when rehearsing several ranks on one GPU
    dev = torch.device("cuda", local % max(torch.cuda.device_count(), 1))
    torch.cuda.set_device(dev)
    if world > 1:
        # Control plane only (barriers, max-reduction of the step time, per-rank kernel times): rays are
        # independent, so the trace has no data-path exchange and needs no RCCL communicator.
        import torch.distributed as dist
        dist.init_process_group("gloo")

    wl = Workload(args.config, dev, rank, scale=args.scale, c2_rays=args.rays)
    if args.pmc_child:
        for _ in range(3):
            wl.step()
        torch.cuda.synchronize()
        return

    for _ in range(args.warmup):
        wl.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # each rank's own clock stops at its device sync; the job time is the max over ranks (all_reduce
    # below), so the closing barrier's own latency is not charged to the K steps
    kernel_ms, elapsed = wl.timed(args.steps)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    fill = wl.fill_rate() if rank == 0 else None
    copy = stream_copy_rate(dev) if rank == 0 else None

    per_rank = None
    if world > 1:
        t = torch.tensor([elapsed, kernel_ms], dtype=torch.float64)
        gathered = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(gathered, t)
        per_rank = [{"rank": r, "kernel_ms": float(g[1]), "GBps": wl.alg_bytes / (float(g[1]) * 1e-3) / 1e9,
                     "wall_s": float(g[0])} for r, g in enumerate(gathered)]
        elapsed = max(p["wall_s"] for p in per_rank)
        kernel_ms_max = max(p["kernel_ms"] for p in per_rank)
    else:
        kernel_ms_max = kernel_ms

    total_units = world * wl.n * wl.S * args.steps
    value = total_units / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    if rank == 0:
        traffic, note = (None, None)
        if world == 1 and args.traffic == "auto":
            traffic, note = measure_traffic(args, args.config)
        rl = roofline(wl, kernel_ms_max, traffic, note, fill, copy)
        rl["kernel_ms_max_rank"] = kernel_ms_max
        line = {
            "metric": METRIC, "value": value, "unit": UNIT, "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": wl.workload, "storage": wl.storage, "rays_per_gpu": wl.n, "surfaces": wl.S,
                       "planes_stored": len(wl.planes), "layout": "aos",
                       "parallelism": f"ray shards x{world} (no collective)"},
            "roofline": rl,
        }
        if per_rank:
            line["per_rank"] = per_rank
        if world == 1 and args.secondary == "auto" and args.config != "c2":
            del wl
            torch.cuda.empty_cache()
            w2 = Workload("c2", dev, 0, c2_rays=args.rays)
            for _ in range(max(args.warmup, 5)):
                w2.step()
            torch.cuda.synchronize()
            k2, e2 = w2.timed(max(args.steps, 50))
            tr2, note2 = (None, None)
            if args.traffic == "auto":
                tr2, note2 = measure_traffic(args, "c2")
            line["secondary"] = {"config": "BASELINE configs[1]: " + w2.workload, "dtype": "f64",
                                 "value": w2.n * w2.S * max(args.steps, 50) / e2, "unit": UNIT,
                                 "rays": w2.n, "surfaces": w2.S,
                                 "roofline": roofline(w2, k2, tr2, note2, w2.fill_rate(), copy)}
        if world == 1 and args.cpu_baseline == "auto":
            cpu = cpu_time(args.config, 8.0)
            cpu["cpu_model"] = cpu_model()
            try:
                # the GPU box allots 16 host CPUs per GPU; os.cpu_count() there reports the whole machine
                procs = max(1, min(16, len(os.sched_getaffinity(0))))
                cpu["parallel"] = cpu_parallel(args.config, procs)
            except Exception as e:  # noqa: BLE001 -- the single-process baseline stands on its own
                cpu["parallel"] = {"error": repr(e)}
            cpu["c1"] = cpu_time("c1", 2.0)
            cpu["calibration"] = ("tests/golden/cpu_calibration.json: rt_refcost runs at 0.92-1.15x the reference's "
                                  "own speed on C1-C5 samples (same host, interleaved)")
            line["cpu_baseline"] = cpu
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
