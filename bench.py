"""Benchmark: ray-surface intersections/s of the sequential ray trace on MI355X (BASELINE.json metric).

Headline workload (BASELINE.json configs[2], the largest single-GPU config): the 4f
relay of scripts/2024_08_08_achromat_imaging.py:13-70 -- object flat, two Thorlabs AC508-075-A-ML
doublets (Ebaf11 / N-SF11), pupil flat, image flat: S = 9 surfaces -- traced with 5 field points
h in {0, 4, 8, 12, 16} mm x get_ray_fan(h, 1 deg, 3163, 0.635 um, nphis=3162) = 50,007,030 rays per GPU,
the full drop-in history (2S+1 = 19 planes) stored as float32 (BASELINE precision; arithmetic float64,
input rays float64 as the generator makes them, so the history is the reference's rounded once).  A timed
step = one launch of the fused trace kernel (rtpb_trace through the C ABI: the body of System.ray_trace,
RT:641-661) on the GPU's bundle, the plan lowered once before the timed region, inputs and outputs
resident in HBM.  The whole drop-in call System.ray_trace(torch rays, ...) -- lowering, table keys of the
Ebaf11 crown (MAT:128-144), output allocation, launch -- is timed separately as `e2e_ms`.
Multi-GPU: one process per GPU (torchrun), each traces its own C3 bundle (rays are independent: no
data-path collective) -> weak scaling; the job time is the max over ranks.

The same JSON line carries the other BASELINE configs under "configs":
  configs[1] C2  AC508-100-B achromat, 1M rays, float64 history (rank 0, N=1 only)
  configs[3] C4  ideal OPM (scripts/2022_01_25_ray_trace_ideal_opm.py:59-92): the 10001 x 10000 fan
                 (100,010,000 rays, 11 surfaces, 23-plane float32 history) STRONG-scaled over the ranks:
                 rank r generates and traces phi rows shard_bounds(10000, N)[r] on its own GPU
  configs[4] C5  spot-diagram sweep (scripts/2021_10_06_ray_trace_system.py:120-145,186): 64 field points
                 x 7 wavelengths x 10,001,406-ray fans (4.48e9 rays, 14 surfaces, float64, statistics
                 only) -- the fused sweep kernel; field points split over the ranks (strong scaling)
and `cpu_baseline` (N=1, rank 0): oracle/rt_refcost.py -- the reference's algorithm and data flow,
calibrated against the reference in tests/golden/cpu_calibration.json -- timed on this host on a bounded
sample of C3, plus C1 (BASELINE configs[0], the plano-convex CPU case).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2] [--configs c2,c4,c5 | none]
    torchrun --nproc-per-node N bench.py --gpus N ...

`python bench.py --gpus N` (N > 1) outside torchrun starts `torch.distributed.run --nproc-per-node N` on
itself as a child process and exits with its code; the ranks' JSON line (rank 0) is forwarded as is.
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
F64_VALU_PEAK_TFLOPS = 78.6    # MI355X FP64 vector: 1/2 of the 157.3 TFLOP/s FP32 vector peak (MI355X_MICROARCH.md:41)
SEED = 20241008
C3_FAN = (3163, 3162)          # scripts/2024_08_08_achromat_imaging.py fan at 10M rays per field
C3_CPU_FAN = (448, 447)        # CPU-baseline sample of C3: 5 fields x 200,256 rays
C4_FAN = (10001, 10000)        # scripts/2022_01_25_ray_trace_ideal_opm.py:59-92
C5_FAN = (3163, 3162)          # scripts/2021_10_06_ray_trace_system.py:186 (10M rays per group)


def _trim_buffers():
    """Release the memory of freed history buffers (ray_trace_pb_amd's buffer pool) with torch's cache."""
    from ray_trace_pb_amd import _engine as E
    E.trim_history_buffers()


def _log(msg):
    """Progress on stderr (the JSON line alone goes to stdout)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def shard_seed(rank):
    return SEED + 7919 * rank


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c3", choices=["c3", "c2", "c4", "c5", "c5_1wl"],
                    help="headline workload (c5, c5_1wl: --pmc-child only)")
    ap.add_argument("--configs", default="c2,c4,c5", help="other BASELINE configs in the same line ('none')")
    ap.add_argument("--scale", type=float, default=1.0, help="c3 / c4: fraction of the per-axis fan sizes")
    ap.add_argument("--rays", type=int, default=1_000_000, help="c2: rays per GPU")
    ap.add_argument("--c5-fields", type=int, default=64, help="c5: field points (square grid)")
    ap.add_argument("--c5-steps", type=int, default=2, help="c5: timed sweeps")
    ap.add_argument("--cpu-baseline", default="auto", choices=["auto", "off"])
    ap.add_argument("--traffic", default="auto", choices=["auto", "off"],
                    help="measure HBM bytes / FLOPs with separate rocprofv3 --pmc child runs (rank 0, N=1)")
    ap.add_argument("--extras", default="on", choices=["on", "off"],
                    help="off: only the headline loop's launches (no placement check / drop-in calls), e.g. "
                         "under rocprofv3 so the kernel's csv average is the timed launches'")
    ap.add_argument("--oversubscribe", action="store_true",
                    help="allow --gpus N above the visible GPU count (ranks share GPUs: a rehearsal, not a measurement)")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--pmc-shard", default="0,1", help=argparse.SUPPRESS)       # rank,world of a c4 PMC child
    return ap.parse_args()


def dist_env():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), int(os.environ.get("LOCAL_RANK", 0))


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_argv(gpus, argv, port):
    """The torchrun command that runs this script as `gpus` ranks (one process per GPU) with the same
    arguments: `python bench.py --gpus N` launched without torchrun starts it as a child process."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def check_world(args, world, visible):
    """--gpus N must name the job's world size; N GPUs must be visible unless --oversubscribe (rehearsal)."""
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU with "
                         f"--gpus equal to the number of ranks")
    if args.gpus > visible and not args.oversubscribe:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but only {visible} GPU(s) visible (use --oversubscribe "
                         f"to rehearse several ranks on shared GPUs)")


def launch_ranks(args):
    """No torchrun environment and N > 1: run `torchrun --nproc-per-node N bench.py <same args>` as a child
    process (never exec: the parent has not touched the GPU, but nothing is replaced either), forward its
    output and return its exit code."""
    import torch
    visible = torch.cuda.device_count()          # counts devices without initialising the GPU on this image
    check_world(args, args.gpus, visible)
    cmd = launcher_argv(args.gpus, sys.argv[1:], _free_port())
    _log(f"launching {args.gpus} ranks: {' '.join(cmd)}")
    return subprocess.run(cmd, stdin=subprocess.DEVNULL).returncode


def device_identity(dev):
    """The rank's GPU: index, PCI domain:bus:device and UUID (distinct physical GPUs are checkable)."""
    import torch
    p = torch.cuda.get_device_properties(dev)
    return {"device": dev.index, "pci": f"{getattr(p, 'pci_domain_id', 0):04x}:{getattr(p, 'pci_bus_id', 0):02x}:"
                                       f"{getattr(p, 'pci_device_id', 0):02x}",
            "uuid": str(getattr(p, "uuid", "")), "name": p.name}


def _gather_objects(world, obj):
    if world == 1:
        return [obj]
    import torch.distributed as dist
    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


class Workload:
    """One history config on one GPU: system, device-resident input rays, output history buffer.
    C4 takes the rank's shard (phi rows) of the 100M-ray fan; C3 and C2 a whole bundle per GPU."""

    def __init__(self, config, dev, rank, world=1, scale=1.0, c2_rays=1_000_000):
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
        elif config == "c4":
            import ray_trace_pb_amd.raytrace as rtm
            self.system, self.m0, self.m1 = systems.c4_system(rt, mat), mat.Constant(systems.OPM_N1), mat.Vacuum()
            nt, nph = int(C4_FAN[0] * scale), int(C4_FAN[1] * scale)
            p0, p1 = rtm.shard_bounds(nph, world)[rank]
            self.total_rays = nt * nph
            self.rays = torch.empty(((p1 - p0) * nt, 8), dtype=torch.float64, device=dev)
            theta = 30 * np.pi / 180
            rt.fan_into(self.rays, np.array([1e-3, 1e-3, 1e-3 * np.tan(theta)]), np.arcsin(1.35 / systems.OPM_N1),
                        nt, systems.OPM_WAVELENGTH, nph, phi_rows=(p0, p1))
            self.code = C.RTPB_F32
            self.workload = (f"C4: ideal OPM of scripts/2022_01_25_ray_trace_ideal_opm.py:59-92 (6 PerfectLens + 5 "
                             f"flats, one tilted 30 deg, S=11), get_ray_fan(asin(1.35/1.4), {nt}, 532e-6, "
                             f"nphis={nph}) = {nt * nph} rays sharded by phi rows over the ranks, full 23-plane "
                             f"history")
            self.storage = "f32 history (float64 input rays, float64 arithmetic)"
            wl_keys = np.array([systems.OPM_WAVELENGTH])
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
        # the history: the product's placement-robust buffer (raytrace.history_buffer / rtpb_buffer_alloc,
        # the out= of repeated traces), so the rate does not depend on where this process's first large
        # allocation lands; second_buffer() times a default torch allocation beside it
        self.out = E.history_buffer((len(self.planes), self.n, 8), torch.float64 if w == 8 else torch.float32, dev)
        self.stream = torch.cuda.current_stream(dev).cuda_stream
        # algorithmic bytes per launch, SURVEY.md §8(d) / BASELINE.md: 16 w (S+1) per ray for the full history
        # (one read of an input record and one write of each of the 2S+1 planes at the storage width w)
        self.bytes_per_ray = 16 * w * (self.S + 1)
        self.alg_bytes = self.n * self.bytes_per_ray
        # bytes the launch physically moves: the input is read at ITS width (float64 rays: 64 B)
        self.phys_bytes_per_ray = 8 * self.rays.element_size() + 8 * w * len(self.planes)
        self.phys_bytes = self.n * self.phys_bytes_per_ray
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

    def second_buffer(self, steps):
        """Average launch duration (ms) of the same trace into a history allocated by torch's default
        allocator (what System.ray_trace allocates without out=): the many-plane write pattern runs at a
        rate that depends on where that memory lies (placement), so the line shows it beside
        the timed history buffer."""
        import torch
        main_out = self.out
        self.out = torch.empty(main_out.shape, dtype=main_out.dtype, device=main_out.device)
        try:
            self.step()
            kernel_ms, _ = self.timed(steps)
        finally:
            self.out = main_out
        return kernel_ms

    def e2e(self, reps=15):
        """The drop-in call on device-resident rays: System.ray_trace(torch rays, m0, m1, dtype) -- lowering,
        table keys, output allocation and the launch (ms per call, synchronised)."""
        import torch
        dt = "float32" if self.code != self._E.C.RTPB_F64 else None
        # System.ray_trace allocates its own history: a history of >= 512 MiB comes from the history pool, whose
        # caching allocator hands a repeated call the block the previous history freed -- first the timed loop's
        # own buffer, then the same one call after call (torch's stream-ordered reuse on the launch stream)
        del self.out
        h = self.system.ray_trace(self.rays, self.m0, self.m1, dtype=dt)
        del h
        torch.cuda.synchronize()
        import ctypes
        C = self._E.C
        lib = C.lib()
        # the call's wall time (synchronised), with the library's launch timing OFF: its two events per launch are a
        # measurement aid, not part of the drop-in call
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            h = self.system.ray_trace(self.rays, self.m0, self.m1, dtype=dt)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
            del h
        # the same calls' kernel (HIP events around the library's own launch), in a second pass
        ks = []
        for _ in range(reps):
            lib.rtpb_timing_enable(1)
            h = self.system.ray_trace(self.rays, self.m0, self.m1, dtype=dt)
            torch.cuda.synchronize()
            tot, cnt = ctypes.c_double(), ctypes.c_int64()
            C.check(lib.rtpb_timing_collect(ctypes.byref(tot), ctypes.byref(cnt)))
            lib.rtpb_timing_enable(0)
            ks.append(tot.value)
            del h
        return float(np.median(ts)) * 1e3, float(np.median(ks))

    def fill_rate(self):
        """The output buffer's delivered plain-write rate (GB/s, torch fill_): context for the history's
        multi-plane write pattern."""
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
    `nbytes` buffers): the measured stream-copy figure SURVEY §8(d) asks for beside the 8 TB/s spec."""
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
    _trim_buffers()
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


# ---------------------------------------------------------------------------------------------- PMC
def _pmc_run(args, config, counters, kernel, shard=(0, 1)):
    """One rocprofv3 --pmc child run of this script (--pmc-child --config CONFIG): per-dispatch counter
    values of the kernels whose name contains `kernel` -> {counter: [values]} or an error string.  `shard`: the
    (rank, world) whose C4 shard the child traces (the child runs on the calling rank's GPU)."""
    import csv
    prof = shutil.which("rocprofv3")
    if not prof:
        return None, "rocprofv3 not found"
    d = os.path.join(ROOT, "gpurun_out", "bench_pmc", config, "_".join(counters))
    shutil.rmtree(d, ignore_errors=True)
    cmd = [prof, "--pmc"] + list(counters) + ["--output-format", "csv", "-d", d, "-o", "pmc", "--",
                                              sys.executable, os.path.abspath(__file__), "--pmc-child",
                                              "--config", config, "--scale", str(args.scale), "--rays",
                                              str(args.rays), "--pmc-shard", f"{shard[0]},{shard[1]}"]
    try:
        subprocess.run(cmd, check=True, timeout=300, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                       stdin=subprocess.DEVNULL, env=dict(os.environ, TMPDIR="/tmp"))
    except Exception as e:  # noqa: BLE001
        return None, f"rocprofv3 {counters} failed: {e}"
    vals = {c: [] for c in counters}
    for dp, _, files in os.walk(d):
        for f in files:
            if f.endswith("counter_collection.csv"):
                with open(os.path.join(dp, f)) as fh:
                    for row in csv.DictReader(fh):
                        if kernel in row.get("Kernel_Name", "") and row.get("Counter_Name") in vals:
                            vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    if not all(vals.values()):
        return None, f"no {counters} rows for {kernel}"
    return vals, None


def measure_traffic(args, config, shard=(0, 1)):
    """HBM bytes per trace launch from rocprofv3 PMC counters (FETCH_SIZE and WRITE_SIZE in separate
    passes; gfx950: FETCH_SIZE counts half the bytes of wide streaming reads, so it is doubled --
    MI355X_MICROARCH.md §HBM).  Counters are in KiB.  `shard`: C4's (rank, world) shard."""
    out = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        vals, err = _pmc_run(args, config, [ctr], "trace_kernel", shard)
        if err:
            return None, err
        out[ctr] = float(np.median(vals[ctr]))
    return (2.0 * out["FETCH_SIZE"] + out["WRITE_SIZE"]) * 1024.0, None


F64_COUNTERS = ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F64")
MIX_COUNTERS = ("SQ_INSTS_VALU", "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_CVT")
# VALU issue cost per wave64 instruction (SIMD cycles): every VALU instruction issues in 4 cycles at the full rate
# (the float64 vector peak 78.6 TFLOP/s = 1024 SIMDs x 2.4 GHz x 64 lanes x 2 FLOP / 4 cycles); a float64
# transcendental (v_rcp_f64 / v_rsq_f64) costs 17.83 / 6.0 = 2.97 times an FMA (tools/valu/valu_rates.hip,
# profiles/r04/g/valu_rates.log, two waves per SIMD) and does not overlap with FMAs
ISSUE_CYCLES = {"valu": 4.0, "trans_f64": 4.0 * 17.83 / 6.0}
SIMDS, PEAK_CLOCK_HZ = 1024, 2.4e9


def measure_c5_flops(args):
    """float64 FLOPs and the VALU instruction mix per ray of the fused sweep kernel from one PMC pass over a
    reduced C5 sweep (one field point x 7 wavelengths x the full 10M-ray fan: the same per-ray work as the full
    sweep).  FLOPs = 64 lanes x (2 FMA + MUL + ADD + TRANS) per wave-instruction.  The mix gives the sweep's
    issue-time ceiling: every VALU instruction at ISSUE_CYCLES on 1024 SIMDs at 2.4 GHz."""
    vals, err = _pmc_run(args, "c5", list(F64_COUNTERS) + list(MIX_COUNTERS), "sweep_kernel")
    if err:
        return None, err
    tot = {k: sum(v) for k, v in vals.items()}

    def f64_flops(t):
        return 64.0 * (2 * t["SQ_INSTS_VALU_FMA_F64"] + t["SQ_INSTS_VALU_MUL_F64"] + t["SQ_INSTS_VALU_ADD_F64"] +
                       t["SQ_INSTS_VALU_TRANS_F64"])
    rays = 7 * C5_FAN[0] * C5_FAN[1]
    trans = tot["SQ_INSTS_VALU_TRANS_F64"]
    cycles = (tot["SQ_INSTS_VALU"] - trans) * ISSUE_CYCLES["valu"] + trans * ISSUE_CYCLES["trans_f64"]
    res = {"executed_flops_per_ray": f64_flops(tot) / rays, "f64_wave_instructions": {k: tot[k] for k in F64_COUNTERS},
           "valu_mix_wave_instructions": {k: tot[k] for k in MIX_COUNTERS}, "pmc_sample_rays": rays,
           "issue_simd_cycles_per_ray": cycles / rays}
    # the algorithmic FLOPs of a ray: the same sweep at one wavelength, where every ray is traced alone (the bundle
    # rows share generation and the first surface between a field point's wavelengths, which removes executed work)
    one, err1 = _pmc_run(args, "c5_1wl", list(F64_COUNTERS), "sweep_kernel")
    if err1:
        res["flops_per_ray"], res["flops_kind"] = res["executed_flops_per_ray"], f"executed ({err1})"
    else:
        res["flops_per_ray"] = f64_flops({k: sum(v) for k, v in one.items()}) / (C5_FAN[0] * C5_FAN[1])
        res["flops_kind"] = "algorithmic"
    return res, None


def roofline(wl, kernel_ms, traffic=None, traffic_note=None, fill=None, copy=None):
    achieved = wl.alg_bytes / (kernel_ms * 1e-3) / 1e9
    phys = wl.phys_bytes / (kernel_ms * 1e-3) / 1e9
    r = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
         "traffic": traffic, "kernel": "trace_kernel", "kernel_ms_avg": kernel_ms,
         "kernel_ms_method": "HIP events on the launch stream around the K launches / K",
         "alg_bytes_per_launch": wl.alg_bytes, "alg_bytes_per_ray": wl.bytes_per_ray,
         "alg_bytes_formula": "SURVEY.md 8(d) / BASELINE.md: 16 w (S+1) per ray, w = storage width",
         "alg_bytes_per_ray_surface": wl.bytes_per_ray / wl.S,
         "physical_bytes_per_launch": wl.phys_bytes, "physical_bytes_per_ray": wl.phys_bytes_per_ray,
         "achieved_physical": phys, "frac_physical": phys / HBM_PEAK_GBS,
         "physical_note": "the input rays are float64 (64 B read per ray); traffic (PMC) counts these bytes"}
    if fill:
        r.update(output_fill_GBps=fill, frac_of_output_fill=phys / fill)
    if copy:
        r.update(torch_copy_GBps=copy)
    if traffic_note:
        r["traffic_note"] = traffic_note
    return r


# ---------------------------------------------------------------------------------------------- configs
def _barrier(world):
    import torch
    torch.cuda.synchronize()
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def _gather(world, vals):
    """[per-rank list of floats] (gloo all_gather; the control plane only)."""
    import torch
    t = torch.tensor(vals, dtype=torch.float64)
    if world == 1:
        return [t.tolist()]
    import torch.distributed as dist
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [o.tolist() for o in out]


def strong_scaling(t1_ms, tn_ms, world):
    """Strong-scaling fields of a config traced whole on one GPU (t1_ms per step, rank 0 alone, before the sharded
    run in the same job) and sharded over `world` ranks (tn_ms per step, max over ranks):
    efficiency = t1 / (N tN) -- 1.0 is linear scaling."""
    return {"t1_ms": t1_ms, "tN_ms": tn_ms, "speedup": t1_ms / tn_ms, "scaling_efficiency": t1_ms / (world * tn_ms),
            "scaling_method": "t1: the whole config on rank 0's GPU alone, timed in this job before the sharded run "
                              "(same box); tN: the sharded run's max-over-ranks step time; efficiency = t1 / (N tN)"}


def host_e2e(w, reps=3):
    """the end-to-end rate with the PCIe transfers -- System.ray_trace on a NumPy bundle in host
    memory returning the NumPy history (rtpb_trace_host: pinned staging, chunked H2D / trace / D2H)."""
    host = w.rays.cpu().numpy()
    h = w.system.ray_trace(host, w.m0, w.m1)
    ts = []
    for _ in range(reps):
        del h
        t0 = time.perf_counter()
        h = w.system.ray_trace(host, w.m0, w.m1)
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    nbytes = host.nbytes + h.nbytes
    return {"ms": t * 1e3, "ray_surface_per_s": w.n * w.S / t, "host_bytes": nbytes, "host_GBps": nbytes / t / 1e9,
            "note": "NumPy rays in host memory -> NumPy history (H2D + trace + D2H through rtpb_trace_host); "
                    "never the headline value"}


def run_c2(args, dev, copy):
    import torch
    w2 = Workload("c2", dev, 0, c2_rays=args.rays)
    for _ in range(max(args.warmup, 5)):
        w2.step()
    torch.cuda.synchronize()
    steps = max(args.steps, 50)
    k2, e2 = w2.timed(steps)
    tr2, note2 = (None, None)
    if args.traffic == "auto":
        tr2, note2 = measure_traffic(args, "c2")
    res = {"baseline_config": "configs[1]", "workload": w2.workload, "dtype": "f64", "storage": w2.storage,
           "value": w2.n * w2.S * steps / e2, "unit": UNIT, "n_gpus": 1, "steps": steps, "ms_per_step": e2 / steps * 1e3,
           "rays": w2.n, "surfaces": w2.S, "roofline": roofline(w2, k2, tr2, note2, w2.fill_rate(), copy)}
    # the drop-in call with its default history allocation (System.ray_trace on the device bundle, no out=)
    e2e_ms, e2e_kernel_ms = w2.e2e(reps=31)
    res.update(e2e_ms=e2e_ms, e2e_kernel_ms=e2e_kernel_ms, e2e_overhead_ms=e2e_ms - e2e_kernel_ms,
               e2e_over_loop_kernel=e2e_ms / k2,
               e2e_note="System.ray_trace(torch rays, Vacuum(), Vacuum()) on the device-resident C2 bundle, the median "
                        "of 31 calls: lowering (memoised), history allocation (the default: the history pool's "
                        "shuffled-chunk memory, reused through torch's caching allocator), launch, synchronise; "
                        "e2e_kernel_ms: the median kernel of 31 more such calls (HIP events the library records "
                        "around its launch, off while the calls are timed)")
    res["host_e2e"] = host_e2e(w2)
    del w2
    torch.cuda.empty_cache()
    _trim_buffers()
    return res


def run_c4(args, dev, rank, world, copy):
    """BASELINE configs[3]: the 100M-ray OPM fan strong-scaled over the ranks (each rank its phi rows).  With N > 1
    rank 0 first traces the whole fan alone (N = 1 in the same job, so the line carries its own scaling
    efficiency), the other ranks waiting at a barrier."""
    import torch
    steps = max(3, min(args.steps, 20))
    t1_ms = None
    if world > 1:
        if rank == 0:
            _log("c4: the whole fan on rank 0 alone (t1)")
            w1 = Workload("c4", dev, 0, world=1, scale=args.scale)
            for _ in range(max(2, min(args.warmup, 5))):
                w1.step()
            torch.cuda.synchronize()
            _, wall1 = w1.timed(steps)
            t1_ms = wall1 / steps * 1e3
            del w1
            torch.cuda.empty_cache()
            _trim_buffers()
        _barrier(world)
    wl = Workload("c4", dev, rank, world=world, scale=args.scale)
    for _ in range(max(2, min(args.warmup, 5))):
        wl.step()
    _barrier(world)
    kernel_ms, wall = wl.timed(steps)
    _barrier(world)
    g = _gather(world, [wall, kernel_ms, float(wl.n)])
    max_wall = max(x[0] for x in g)
    res = None
    if rank == 0:
        traffic, note = (None, None)
        if args.traffic == "auto":
            # N > 1: rank 0's own shard, in child runs on its GPU (the other ranks wait at the next barrier)
            traffic, note = measure_traffic(args, "c4", (rank, world))
        per_rank = [{"rank": r, "rays": int(x[2]), "kernel_ms": x[1],
                     "alg_GBps": x[2] * wl.bytes_per_ray / (x[1] * 1e-3) / 1e9,
                     "frac_8TBs": x[2] * wl.bytes_per_ray / (x[1] * 1e-3) / 1e9 / HBM_PEAK_GBS, "wall_s": x[0]}
                    for r, x in enumerate(g)]
        res = {"baseline_config": "configs[3]", "workload": wl.workload, "dtype": "f64", "storage": wl.storage,
               "value": wl.total_rays * wl.S * steps / max_wall, "unit": UNIT, "n_gpus": world, "steps": steps,
               "ms_per_step": max_wall / steps * 1e3, "scaling": "strong", "total_rays": wl.total_rays,
               "surfaces": wl.S, "planes_stored": len(wl.planes),
               "parallelism": f"phi-row ray shards x{world} (no collective)",
               "roofline": roofline(wl, max(x[1] for x in g), traffic, note, wl.fill_rate() if world == 1 else None,
                                    copy),
               "roofline_scope": "per GPU: rank 0's shard bytes over the slowest rank's kernel time" if world > 1
                                 else "the whole fan on one GPU",
               "per_rank": per_rank}
        if world == 1:
            res["roofline"]["note"] = "N=1: the whole 100M-ray fan on one GPU (80 GB in HBM)"
        else:
            res.update(strong_scaling(t1_ms, res["ms_per_step"], world))
    del wl
    torch.cuda.empty_cache()
    _trim_buffers()
    return res


def run_c5(args, dev, rank, world):
    """BASELINE configs[4]: the fused spot-diagram sweep, field points split over the ranks."""
    import torch
    import ray_trace_pb_amd.materials as mat
    import ray_trace_pb_amd.raytrace as rt
    from ray_trace_pb_amd import analysis
    import systems
    n_side = int(round(np.sqrt(args.c5_fields)))
    fields = systems.c5_field_points(n_side)
    f0, f1 = rt.shard_bounds(len(fields), world)[rank]
    mine = fields[f0:f1]
    system = systems.c5_system(rt, mat)
    wls = systems.C5_WAVELENGTHS
    theta = 0.5 * np.pi / 180
    analysis.spot_sweep(system, mat.Constant(1), mat.Constant(1), mine[:1], wls, theta, 33, 32, device=dev)
    t1_ms = None
    if world > 1:
        # the whole sweep on rank 0 alone first (N = 1 in the same job: the line's own scaling efficiency)
        if rank == 0:
            _log("c5: every field point on rank 0 alone (t1)")
            w1 = []
            for _ in range(args.c5_steps):
                t0 = time.perf_counter()
                analysis.spot_sweep(system, mat.Constant(1), mat.Constant(1), fields, wls, theta, C5_FAN[0],
                                    C5_FAN[1], device=dev)
                torch.cuda.synchronize()
                w1.append(time.perf_counter() - t0)
            t1_ms = float(np.median(w1)) * 1e3
        _barrier(world)
    kms, walls, hbm = [], [], 0.0
    summ = None
    for _ in range(args.c5_steps):
        _barrier(world)
        t0 = time.perf_counter()
        summ, timing = analysis.spot_sweep(system, mat.Constant(1), mat.Constant(1), mine, wls, theta, C5_FAN[0],
                                           C5_FAN[1], device=dev)
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t0)
        kms.append(sum(p["kernel_ms"] for p in timing["per_device"]))
        hbm = sum(p["hbm_bytes"] for p in timing["per_device"])
    _barrier(world)
    my_rays = float(len(mine) * len(wls) * C5_FAN[0] * C5_FAN[1])
    g = _gather(world, [float(np.median(walls)), float(np.median(kms)), my_rays, hbm])
    if rank != 0:
        return None
    S = len(system.surfaces)
    total = sum(x[2] for x in g)
    max_wall = max(x[0] for x in g)
    kmax = max(x[1] for x in g)
    per_rank = [{"rank": r, "rays": int(x[2]), "kernel_ms": x[1], "hbm_bytes": x[3],
                 "hbm_GBps": x[3] / (x[1] * 1e-3) / 1e9} for r, x in enumerate(g)]
    res = {"baseline_config": "configs[4]", "workload": (
        f"C5: spot-diagram sweep of scripts/2021_10_06_ray_trace_system.py:120-145,186 (ODT excitation path, "
        f"4 doublets + PerfectLens + flat, S=14), {len(fields)} field points x {len(wls)} wavelengths x "
        f"get_ray_fan(0.5 deg, {C5_FAN[0]}, nphis={C5_FAN[1]}), final plane reduced to per-group spot statistics "
        f"in the fused sweep kernel"), "dtype": "f64", "value": total * S / max_wall, "unit": UNIT,
        "n_gpus": world, "steps": args.c5_steps, "ms_per_step": max_wall * 1e3, "scaling": "strong",
        "total_rays": int(total), "surfaces": S, "parallelism": f"field-point shards x{world} (no collective)",
        "per_rank": per_rank,
        "rms_radius_um_field0": (summ["rms_radius"][0] * 1e3).tolist() if rank == 0 else None}
    if world > 1:
        res.update(strong_scaling(t1_ms, res["ms_per_step"], world))
    rl = {"bound": "valu_f64", "peak": F64_VALU_PEAK_TFLOPS, "unit": "TFLOP/s", "kernel": "sweep_kernel",
          "kernel_ms_max_rank": kmax, "hbm_GBps_max_rank": max(p["hbm_GBps"] for p in per_rank),
          "hbm_note": "the rays never leave registers: HBM carries only the per-tile partial sums"}
    if args.traffic == "auto":
        # N > 1: the per-ray counts of a 1-field sample on rank 0's GPU (the sweep's work per ray does not depend on
        # the field split); achieved / frac are then per GPU (rank 0's rays over its kernel time)
        fl, err = measure_c5_flops(args)
        if fl:
            rays0 = g[0][2]
            S14 = len(system.surfaces)
            mix = fl["valu_mix_wave_instructions"]
            per_rs = lambda v: v * 64.0 / (fl["pmc_sample_rays"] * S14)       # wave-instructions -> per ray-surface
            issue_s = fl["issue_simd_cycles_per_ray"] * rays0 / SIMDS / PEAK_CLOCK_HZ
            rl.update(achieved=fl["executed_flops_per_ray"] * rays0 / (g[0][1] * 1e-3) / 1e12,
                      executed_flops_per_ray=fl["executed_flops_per_ray"],
                      achieved_effective=fl["flops_per_ray"] * rays0 / (g[0][1] * 1e-3) / 1e12,
                      effective_flops_per_ray=fl["flops_per_ray"], effective_flops_kind=fl["flops_kind"],
                      f64_wave_instructions_sample=fl["f64_wave_instructions"],
                      pmc_sample_rays=fl["pmc_sample_rays"],
                      flops_method="achieved / frac: the float64 FLOPs the kernel EXECUTES -- PMC "
                                   "SQ_INSTS_VALU_{FMA,MUL,ADD,TRANS}_F64 x 64 lanes (FMA = 2) on a 1-field x "
                                   "7-wavelength sample, scaled per ray (a hardware-utilisation figure); "
                                   "achieved_effective / frac_effective: the algorithmic FLOPs of a ray traced alone "
                                   "(the same counters on a 1-field sweep at ONE wavelength), which the bundle rows "
                                   "do not all execute -- they share each ray's generation and first surface between "
                                   "a field point's wavelengths; frac_issue: how close the kernel runs to its "
                                   "instruction-issue ceiling",
                      valu_per_ray_surface=per_rs(mix["SQ_INSTS_VALU"]),
                      valu_mix_per_ray_surface={
                          "f64_add_mul_fma": per_rs(sum(fl["f64_wave_instructions"][k] for k in F64_COUNTERS[:3])),
                          "f64_trans": per_rs(fl["f64_wave_instructions"]["SQ_INSTS_VALU_TRANS_F64"]),
                          "int32": per_rs(mix["SQ_INSTS_VALU_INT32"]), "int64": per_rs(mix["SQ_INSTS_VALU_INT64"]),
                          "cvt": per_rs(mix["SQ_INSTS_VALU_CVT"])},
                      issue_ceiling_s=issue_s, frac_issue=issue_s / (g[0][1] * 1e-3),
                      issue_method=("PMC VALU wave-instructions of the 1-field sample scaled to the rank's rays, each at "
                                    "4 SIMD cycles (the full wave64 rate: 78.6 TF f64 = 1024 SIMDs x 2.4 GHz x 64 x 2 / "
                                    "4) and a float64 transcendental at 2.97x (tools/valu/valu_rates.hip), over 1024 "
                                    "SIMDs at 2.4 GHz; frac_issue = that ceiling / the measured kernel time"))
            rl["frac"] = rl["achieved"] / F64_VALU_PEAK_TFLOPS
            rl["scope"] = "per GPU: rank 0's rays over its kernel time" if world > 1 else "one GPU"
            rl["frac_effective"] = rl["achieved_effective"] / F64_VALU_PEAK_TFLOPS
        else:
            rl["flops_note"] = err
    res["roofline"] = rl
    return res


def pmc_child(args, dev):
    """Target of the rocprofv3 --pmc child runs: a few launches of one config's kernel."""
    import torch
    if args.config in ("c5", "c5_1wl"):
        import ray_trace_pb_amd.materials as mat
        import ray_trace_pb_amd.raytrace as rt
        from ray_trace_pb_amd import analysis
        import systems
        # c5_1wl: one wavelength, so every ray is traced alone (no bundle sharing) -- the algorithmic FLOPs per ray
        wls = systems.C5_WAVELENGTHS if args.config == "c5" else systems.C5_WAVELENGTHS[3:4]
        analysis.spot_sweep(systems.c5_system(rt, mat), mat.Constant(1), mat.Constant(1),
                            systems.c5_field_points(8)[:1], wls, 0.5 * np.pi / 180, C5_FAN[0], C5_FAN[1], device=dev)
    else:
        r, w = (int(v) for v in args.pmc_shard.split(","))
        wl = Workload(args.config, dev, r, world=w, scale=args.scale, c2_rays=args.rays)
        for _ in range(3):
            wl.step()
    torch.cuda.synchronize()


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1 and not args.pmc_child:
        sys.exit(launch_ranks(args))
    rank, world, local = dist_env()
    import torch

    if not args.pmc_child:
        check_world(args, world, torch.cuda.device_count())
    # one GPU per rank; the modulo only matters when rehearsing several ranks on one GPU (--oversubscribe)
    dev = torch.device("cuda", local % max(torch.cuda.device_count(), 1))
    torch.cuda.set_device(dev)
    if args.pmc_child:
        pmc_child(args, dev)
        return
    if world > 1:
        # Control plane only (barriers, max-reduction of the step time, per-rank kernel times): rays are
        # independent, so the trace has no data-path exchange and needs no RCCL communicator.
        import torch.distributed as dist
        dist.init_process_group("gloo")

    _log(f"rank {rank}/{world}: headline {args.config}")
    wl = Workload(args.config, dev, rank, world=1, scale=args.scale, c2_rays=args.rays)
    for _ in range(args.warmup):
        wl.step()
    _barrier(world)
    # each rank's own clock stops at its device sync; the job time is the max over ranks (gathered below),
    # so the closing barrier's own latency is not charged to the K steps
    kernel_ms, elapsed = wl.timed(args.steps)
    _barrier(world)
    fill = wl.fill_rate() if rank == 0 else None
    extras = args.extras == "on"
    alt_ms = wl.second_buffer(args.steps) if (extras and world == 1 and args.config in ("c3", "c2")) else None
    e2e_ms, e2e_kernel_ms = wl.e2e() if (extras and args.config == "c3") else (None, None)
    g = _gather(world, [elapsed, kernel_ms])
    ids = _gather_objects(world, device_identity(dev))
    per_rank = [{"rank": r, "kernel_ms": x[1], "alg_GBps": wl.alg_bytes / (x[1] * 1e-3) / 1e9, "wall_s": x[0],
                 **ids[r]} for r, x in enumerate(g)]
    elapsed = max(p["wall_s"] for p in per_rank)
    kernel_ms_max = max(p["kernel_ms"] for p in per_rank)
    total_units = world * wl.n * wl.S * args.steps
    value = total_units / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    head = wl
    del wl
    torch.cuda.empty_cache()
    _trim_buffers()
    copy = stream_copy_rate(dev) if rank == 0 else None

    line = None
    if rank == 0:
        traffic, note = (None, None)
        if world == 1 and args.traffic == "auto":
            _log("PMC traffic of the headline kernel")
            traffic, note = measure_traffic(args, args.config)
        rl = roofline(head, kernel_ms_max, traffic, note, fill, copy)
        rl["kernel_ms_max_rank"] = kernel_ms_max
        line = {
            "metric": METRIC, "value": value, "unit": UNIT, "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64", "storage_dtype": "f32" if head.code != 0 else "f64",
            "data": "synthetic",
            "config": {"workload": head.workload, "baseline_config": "configs[2]" if args.config == "c3" else None,
                       "storage": head.storage, "rays_per_gpu": head.n, "surfaces": head.S,
                       "planes_stored": len(head.planes), "layout": "aos",
                       "parallelism": f"ray shards x{world} (no collective)"},
            "roofline": rl,
        }
        if e2e_ms is not None:
            line["e2e_ms"] = e2e_ms
            line["e2e_over_kernel"] = e2e_ms / e2e_kernel_ms        # the call against its own kernel
            line["e2e_over_loop_kernel"] = e2e_ms / kernel_ms       # ... and against the timed loop's
            line["e2e_kernel_ms"] = e2e_kernel_ms
            line["e2e_overhead_ms"] = e2e_ms - e2e_kernel_ms
            line["e2e_note"] = ("System.ray_trace(torch rays, Vacuum(), Vacuum(), dtype='float32') on the device-"
                                "resident C3 bundle, the median of 15 calls: lowering (memoised by content), "
                                "Ebaf11 table keys (the previous bundle's, checked by the kernel's table-miss "
                                "flag), history allocation (the history pool, torch's caching allocator: the timed "
                                "loop's block, reused), launch, miss-flag read, synchronise. e2e_kernel_ms: the median "
                                "kernel of 15 more such calls (HIP events the library records around its launch, off "
                                "while the calls are timed); e2e_overhead_ms: the host-side cost of the drop-in call "
                                "(tools/e2e_phases.py splits it by phase)")
        if alt_ms is not None:
            line["placement_check"] = {
                "kernel_ms_history_buffer": kernel_ms, "kernel_ms_torch_empty": alt_ms,
                "note": "value: the trace into raytrace.history_buffer (a tensor of the history pool: torch's caching "
                        "allocator over librtpb's shuffled 64 MiB chunk mappings, the default allocation of "
                        "System.ray_trace for histories of POOLED_HISTORY_BYTES = 512 MiB or more); "
                        "kernel_ms_torch_empty: the same launches into a torch.empty history (torch's default pool, "
                        "System.ray_trace's allocation below 512 MiB), whose many-plane write rate depends on where "
                        "it lands (DESIGN.md 5)"}
        line["per_rank"] = per_rank
        line["distinct_gpus"] = len({(p["pci"], p["uuid"]) for p in per_rank})
        if line["distinct_gpus"] < world:
            line["config"]["oversubscribed"] = (f"{world} ranks on {line['distinct_gpus']} GPU(s): a rehearsal of "
                                                f"the N>1 path, not a scaling measurement")
    del head

    configs = [c for c in args.configs.split(",") if c and c != "none"]
    others = {}
    if "c2" in configs and world == 1 and rank == 0:
        _log("configs[1] c2")
        others["c2"] = run_c2(args, dev, copy)
    if "c4" in configs and args.config != "c4":
        _log(f"rank {rank}: configs[3] c4")
        r = run_c4(args, dev, rank, world, copy)
        if rank == 0:
            others["c4"] = r
    if "c5" in configs:
        _log(f"rank {rank}: configs[4] c5")
        r = run_c5(args, dev, rank, world)
        if rank == 0:
            others["c5"] = r

    if rank == 0:
        line["configs"] = others
        if world == 1 and args.cpu_baseline == "auto":
            _log("cpu baseline")
            cpu = cpu_time(args.config if args.config != "c4" else "c3", 8.0)
            cpu["cpu_model"] = cpu_model()
            try:
                # the GPU box allots 16 host CPUs per GPU; os.cpu_count() there reports the whole machine
                procs = max(1, min(16, len(os.sched_getaffinity(0))))
                cpu["parallel"] = cpu_parallel("c3", procs)
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
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
