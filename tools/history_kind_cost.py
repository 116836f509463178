"""Where a history trace's VALU instructions go, surface by surface: the bench bundle of a config (C3 / C4, scaled
down) traced through the first K surfaces of its system for K = 1 .. S (final plane only, so the stores stay small;
--planes all: the full history, the bench's own kernel),
each under its own `rocprofv3 --pmc SQ_INSTS_VALU` run; successive differences are the VALU per ray of each surface
step (kind, and whether it sits on the z axis, printed beside it).

    python tools/history_kind_cost.py --run OUT --config c4 --scale 0.1
    python tools/history_kind_cost.py --run OUT --config c4 --scale 0.1 --planes all
    python tools/history_kind_cost.py --config c4 --surfaces 3 --scale 0.1     # one trace (what each PMC run executes)
"""
import argparse
import csv
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]


def workload(config, scale):
    import torch
    import bench
    wl = bench.Workload(config, torch.device("cuda:0"), 0, scale=scale)
    return wl


def trace(config, k, scale, planes):
    import torch
    import ray_trace_pb_amd.raytrace as rt
    wl = workload(config, scale)
    system = rt.System(wl.system.surfaces[:k], wl.system.materials[:k - 1])
    dt = "float32" if config in ("c3", "c4") else None
    for _ in range(2):
        system.ray_trace(wl.rays, wl.m0, wl.m1, planes=planes, dtype=dt)
    torch.cuda.synchronize()
    print(f"surfaces {k}: rays {wl.rays.shape[0]}", flush=True)


def run(out, config, scale, planes):
    import ray_trace_pb_amd.materials as mat
    import ray_trace_pb_amd.raytrace as rt
    import systems
    system = {"c3": systems.c3_system, "c4": systems.c4_system}[config](rt, mat)
    S = len(system.surfaces)
    env = dict(os.environ, TMPDIR="/tmp")
    per_ray, rays = {}, None
    for k in range(1, S + 1):
        d = os.path.join(out, f"k{k}")
        cmd = ["timeout", "-k", "10", "300", "rocprofv3", "--pmc", "SQ_INSTS_VALU", "--output-format", "csv", "-d", d,
               "-o", "pmc", "--", sys.executable, os.path.abspath(__file__), "--config", config, "--surfaces", str(k),
               "--scale", str(scale), "--planes", planes]
        p = subprocess.run(cmd, env=env, capture_output=True, text=True)
        if p.returncode != 0:
            print(p.stdout[-1000:], p.stderr[-2000:])
            sys.exit(p.returncode)
        line = [ln for ln in p.stdout.splitlines() if ln.startswith("surfaces ")][-1]
        rays = int(line.split("rays ")[1])
        vals = []
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                if "trace_kernel" in row["Kernel_Name"] and row["Counter_Name"] == "SQ_INSTS_VALU":
                    vals.append(float(row["Counter_Value"]))
        per_ray[k] = sorted(vals)[len(vals) // 2] * 64 / rays          # median launch, wave-instructions -> per ray
    prev = 0.0
    for k in range(1, S + 1):
        s = system.surfaces[k - 1]
        ax = ("axial" if (tuple(s.input_axis) == (0.0, 0.0, 1.0) and s.center[0] == 0 and s.center[1] == 0) else
              "x-z" if (float(s.center[1]) == 0 and float(getattr(s, "normal", s.input_axis)[1]) == 0
                        and not isinstance(s, rt.SphericalSurface)) else "general")
        print(f"surface {k - 1:2d} {type(s).__name__:17s} {ax:8s} VALU per ray {per_ray[k] - prev:7.1f}  "
              f"(cumulative {per_ray[k]:8.1f})", flush=True)
        prev = per_ray[k]
    print(f"{config}: {per_ray[S]:.1f} VALU per ray = {per_ray[S] / S:.1f} per ray-surface ({'final plane only' if planes == 'final' else 'all planes'})")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--run", default="")
    ap.add_argument("--config", default="c4", choices=["c3", "c4"])
    ap.add_argument("--surfaces", type=int, default=0)
    ap.add_argument("--scale", type=float, default=0.1)
    ap.add_argument("--planes", default="final", choices=["final", "all"])
    a = ap.parse_args()
    if a.run:
        run(a.run, a.config, a.scale, a.planes)
    else:
        trace(a.config, a.surfaces, a.scale, a.planes)


if __name__ == "__main__":
    main()
