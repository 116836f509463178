"""Where the C5 sweep's VALU instructions go, per surface kind: the one-field C5 sweep (7 wavelengths x 10M-ray
fans) through the first K surfaces of the ODT system (K = 12: the axial spheres; 13: + the PerfectLens; 14: the
whole system, + the final flat), each under its own `rocprofv3 --pmc SQ_INSTS_VALU` run.  The differences between
prefixes give the cost of one lens step and one flat step per ray; the 12-sphere run, the spheres' (with the
per-ray generation, first-surface sharing and reduction spread over them).

    python tools/c5_kind_cost.py --run OUT          # the three PMC runs, then the table
    python tools/c5_kind_cost.py --run OUT --ks 1 2 3 12 13 14   # + the fixed per-ray part (K = 1, 2, 3 surfaces)
    python tools/c5_kind_cost.py --surfaces 13      # one sweep (what each PMC run executes)
"""
import argparse
import csv
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]


def sweep(k):
    import numpy as np
    import torch
    import ray_trace_pb_amd.materials as mat
    import ray_trace_pb_amd.raytrace as rt
    from ray_trace_pb_amd import analysis
    import systems
    full = systems.c5_system(rt, mat)
    system = rt.System(full.surfaces[:k], full.materials[:k - 1])
    fields = systems.c5_field_points(1)
    summ, t = analysis.spot_sweep(system, mat.Constant(1), mat.Constant(1), fields, systems.C5_WAVELENGTHS,
                                  0.5 * np.pi / 180, 3163, 3162, device="cuda:0")
    torch.cuda.synchronize()
    print(f"surfaces {k}: rays {t['rays']}, kernel ms {t['per_device'][0]['kernel_ms']:.3f}, "
          f"count {int(summ['count'].sum())}", flush=True)


def run(out, ks=(12, 13, 14)):
    env = dict(os.environ, TMPDIR="/tmp")
    res = {}
    for k in ks:
        d = os.path.join(out, f"k{k}")
        cmd = ["timeout", "-k", "10", "300", "rocprofv3", "--pmc", "SQ_INSTS_VALU", "--output-format", "csv", "-d", d,
               "-o", "pmc", "--", sys.executable, os.path.abspath(__file__), "--surfaces", str(k)]
        p = subprocess.run(cmd, env=env, capture_output=True, text=True)
        print(p.stdout.strip().splitlines()[-1] if p.stdout.strip() else "", flush=True)
        if p.returncode != 0:
            print(p.stderr[-2000:])
            sys.exit(p.returncode)
        tot = 0.0
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                if "sweep_kernel" in row["Kernel_Name"] and row["Counter_Name"] == "SQ_INSTS_VALU":
                    tot += float(row["Counter_Value"])
        res[k] = tot
    rays = 7 * 3163 * 3162
    per_ray = {k: v * 64 / rays for k, v in res.items()}    # wave-instructions -> per ray (64 lanes)
    for k in sorted(per_ray):
        print(f"surfaces {k:2d}: {per_ray[k]:8.1f} VALU per ray", flush=True)
    if all(k in per_ray for k in (1, 2, 3)):
        # K = 1: generation, the shared first sphere and the reduction; K = 2, 3 add one and two sphere steps
        step = (per_ray[3] - per_ray[1]) / 2
        print(f"fixed per-ray part (generation, first surface shared over the bundle, reduction, run switches): "
              f"{per_ray[1]:.1f} = K=1; a sphere step {step:.1f}; fixed part beyond one step {per_ray[1] - step:.1f}")
    if all(k in per_ray for k in (12, 13, 14)):
        print(f"VALU per ray: 12 surfaces {per_ray[12]:.1f} ({per_ray[12] / 12:.1f} per sphere incl. generation, "
              f"sharing and reduction), lens step {per_ray[13] - per_ray[12]:.1f}, flat step "
              f"{per_ray[14] - per_ray[13]:.1f}, whole system {per_ray[14]:.1f} = {per_ray[14] / 14:.1f} per "
              f"ray-surface")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--run", default="")
    ap.add_argument("--surfaces", type=int, default=14)
    ap.add_argument("--ks", type=int, nargs="+", default=[12, 13, 14],
                    help="--run: the prefixes (numbers of surfaces) to count")
    a = ap.parse_args()
    if a.run:
        run(a.run, tuple(a.ks))
    else:
        sweep(a.surfaces)


if __name__ == "__main__":
    main()
