"""Debug helper: per-plane / per-column mismatch counts of one rtpb_trace variant on one golden case.

    python tools/debug_abi_case.py CASE OUT_CODE IN_CODE IN_LAYOUT OUT_LAYOUT [PAD]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
import numpy as np  # noqa: E402
import test_gpu_abi_matrix as M  # noqa: E402
from ray_trace_pb_amd import _capi as C  # noqa: E402
from ray_trace_pb_amd import _engine as E  # noqa: E402


def main():
    name, out_code, in_code, il, ol = sys.argv[1], *map(int, sys.argv[2:6])
    if len(sys.argv) > 6:
        M.PAD = int(sys.argv[6])
    system, materials, rays, ref = M._load(name)
    n, S = rays.shape[0], len(system.surfaces)
    sel = list(range(2 * S + 1))
    low = E.lower(system.surfaces, materials, lambda: E.distinct_wavelengths(rays[:, 7]), out_code)
    with E.plan_ref(low) as plan:
        x, _, st = M._device_input(rays, in_code, il)
        got, pad_ok = M._trace((plan, E.plane_mask(sel)), x, in_code, il, st, n, len(sel), out_code, ol)
    exp = ref.astype(M.NP_DT[out_code])
    bad = ~((got == exp) | (np.isnan(got) & np.isnan(exp)))
    print("pad_ok", pad_ok, "n", n, "bad total", int(bad.sum()))
    for p in range(bad.shape[0]):
        if bad[p].any():
            rows = np.nonzero(bad[p].any(1))[0]
            print("plane", p, "cols", bad[p].sum(0).tolist(), "rows", rows[:10].tolist(), len(rows))
    p = int(np.nonzero(bad.any((1, 2)))[0][0]) if bad.any() else None
    if p is not None:
        r = int(np.nonzero(bad[p].any(1))[0][0])
        print("first bad plane", p, "ray", r)
        print("in  ", rays[r])
        for q in range(max(0, p - 2), min(bad.shape[0], p + 2)):
            print(q, "got", got[q, r])
            print(q, "exp", exp[q, r])


if __name__ == "__main__":
    main()
