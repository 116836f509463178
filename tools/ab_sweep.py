"""A/B of the fused spot-sweep kernel between librtpb builds in one process (C5 system, reduced fan count).
    python tools/ab_sweep.py ray_trace_pb_amd/exp_X.so [--fields 16] [--nt 1001] [--nph 1000]"""
import argparse
import collections
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden"), os.path.join(ROOT, "tools")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ray_trace_pb_amd.materials as mat  # noqa: E402
import ray_trace_pb_amd.raytrace as rt  # noqa: E402
from ray_trace_pb_amd import _capi as C, _engine as E, analysis  # noqa: E402
import systems  # noqa: E402
from ab_libs import load  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*")
    ap.add_argument("--fields", type=int, default=16)
    ap.add_argument("--nt", type=int, default=1001)
    ap.add_argument("--nph", type=int, default=1000)
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    libs = {"base": C.lib()}
    for p in args.libs:
        libs[os.path.basename(p)] = load(p)
    caches = {k: collections.OrderedDict() for k in libs}
    system = systems.c5_system(rt, mat)
    fields = systems.c5_field_points(int(round(np.sqrt(args.fields))))
    times = collections.defaultdict(list)
    ref = None
    for _ in range(args.rounds):
        for name in np.random.default_rng(len(times)).permutation(list(libs)):
            C._lib, E._PLANS = libs[name], caches[name]
            summ, t = analysis.spot_sweep(system, mat.Constant(1), mat.Constant(1), fields, systems.C5_WAVELENGTHS,
                                          0.5 * np.pi / 180, args.nt, args.nph, device="cuda:0")
            times[name].append(t["seconds"])
            if ref is None:
                ref = summ
            else:
                assert all(np.array_equal(ref[k], summ[k], equal_nan=True) for k in ref), name
    C._lib, E._PLANS = libs["base"], caches["base"]
    base = np.median(times["base"])
    for k, v in times.items():
        print(f"{k:20s} {np.median(v):.4f} s  x{np.median(v) / base:.3f}")


if __name__ == "__main__":
    main()
