"""Calibrate bench.py's CPU baseline against the REFERENCE itself, in this container.

    python tests/golden/calibrate_cpu.py          # writes tests/golden/cpu_calibration.json

/root/reference does not exist on the GPU box, so bench.py times oracle/rt_refcost.py there (the
reference's algorithm with the reference's data flow, pinned bit for bit to the golden vectors by
tests/test_cpu_baseline.py).  This script shows that the stand-in costs what the reference costs: in a
child interpreter whose path holds /root/reference/src first (as make_golden.py), the reference and both
NumPy restatements trace the same bundles of the BASELINE configs, one process, interleaved passes; the
port's history is asserted identical to the reference's on every bundle.
SURVEY.md §8d asks the timed port to be within +-20 % of the reference.
"""
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF_SRC = "/root/reference/src"
MIN_SECONDS = 3.0


def bundles(rt, mat):
    """(name, system, rays, m0, m1) of the BASELINE configs at CPU-sized samples."""
    import systems
    out = []
    s, r, m0, m1 = systems.c1_plano_convex(rt, mat)
    out.append(("C1 plano-convex, 1,001 rays", s, r, m0, m1))
    out.append(("C2 AC508-100-B system, 1,000,000 rays", systems.c2_system(rt, mat), systems.c2_rays(1_000_000),
                mat.Vacuum(), mat.Vacuum()))
    out.append(("C3 4f relay, 5 fields x fan 448x447", systems.c3_system(rt, mat), systems.c3_rays(rt, 448, 447),
                mat.Vacuum(), mat.Vacuum()))
    out.append(("C4 ideal OPM, fan 317x316", systems.c4_system(rt, mat), systems.c4_rays(rt, 317, 316),
                mat.Constant(systems.OPM_N1), mat.Vacuum()))
    out.append(("C5 ODT, 16 fields x 7 wavelengths x fan 45x44", systems.c5_system(rt, mat),
                systems.c5_rays(rt, 4, 45, 44), mat.Constant(1), mat.Constant(1)))
    return out


def timed_pair(fns, units, rounds=5):
    """Median rate of each callable over `rounds` interleaved passes (each pass >= MIN_SECONDS / rounds),
    so slow drifts of a shared host hit every contender alike."""
    for fn in fns:
        fn()                                        # warm (imports, first-touch pages)
    rates = [[] for _ in fns]
    for _ in range(rounds):
        for k, fn in enumerate(fns):
            reps, t = 0, 0.0
            while reps < 1 or t < MIN_SECONDS / rounds:
                t0 = time.perf_counter()
                fn()
                t += time.perf_counter() - t0
                reps += 1
            rates[k].append(units * reps / t)
    return [sorted(r)[len(r) // 2] for r in rates]


def _child(out_path):
    import numpy as np
    import raytrace.raytrace as rt                   # the REFERENCE (only REF_SRC and HERE on the path)
    import raytrace.materials as mat
    assert os.path.abspath(rt.__file__).startswith(REF_SRC), rt.__file__
    sys.path.append(ROOT)                            # after the reference's `raytrace` is bound: oracle only
    from oracle import rt_numpy as O
    from oracle import rt_refcost as RC
    from serialize import system_to_json
    import warnings
    warnings.simplefilter("ignore")
    rows = []
    for name, s, r, m0, m1 in bundles(rt, mat):
        spec = json.loads(system_to_json(s, m0, m1))
        r = np.asarray(r, dtype=np.float64)
        ref = s.ray_trace(r, m0, m1)
        assert np.array_equal(RC.ray_trace(spec["surfaces"], spec["materials"], r), ref, equal_nan=True), name
        units = r.shape[0] * len(s.surfaces)
        a, b, c = timed_pair([lambda: s.ray_trace(r, m0, m1),
                              lambda: RC.ray_trace(spec["surfaces"], spec["materials"], r),
                              lambda: O.ray_trace(spec["surfaces"], spec["materials"], r)], units)
        row = {"name": name, "rays": int(r.shape[0]), "surfaces": len(s.surfaces), "reference": a,
               "refcost_port": b, "column_oracle": c, "refcost_over_reference": b / a}
        print(json.dumps(row), flush=True)
        rows.append(row)
    import platform
    out = {"unit": "ray-surface intersections/s, 1 process (medians of 5 interleaved passes)",
           "numpy": np.__version__, "python": platform.python_version(), "cpu": _cpu_model(),
           "identical_histories": True, "rows": rows}
    with open(out_path, "w") as f:
        json.dump(out, f, indent=1)


def main():
    env = dict(os.environ, PYTHONPATH=f"{REF_SRC}:{HERE}", RTPB_CALIB_CHILD=os.path.join(HERE, "cpu_calibration.json"),
               MPLBACKEND="Agg", PYTHONDONTWRITEBYTECODE="1", OMP_NUM_THREADS="1")
    sys.exit(subprocess.run([sys.executable, os.path.abspath(__file__)], env=env, cwd="/tmp").returncode)


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


if __name__ == "__main__":
    if os.environ.get("RTPB_CALIB_CHILD"):
        _child(os.environ["RTPB_CALIB_CHILD"])
    else:
        main()
