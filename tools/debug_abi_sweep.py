"""Debug helper: which (case, storage, input type, input layout, output layout, planes) variants of
rtpb_trace differ from the expected history (tests/test_gpu_abi_matrix.py without stopping)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
import numpy as np  # noqa: E402
import test_gpu_abi_matrix as M  # noqa: E402
from parity import CASES  # noqa: E402
from ray_trace_pb_amd import _capi as C  # noqa: E402
from ray_trace_pb_amd import _engine as E  # noqa: E402


def main():
    cases = sys.argv[1].split(",") if len(sys.argv) > 1 else CASES
    for name in cases:
        system, materials, rays, ref = M._load(name)
        n, S = rays.shape[0], len(system.surfaces)
        if S > C.RTPB_MAX_SURFACES:
            continue
        sel = list(range(2 * S + 1))
        fails = []
        for out_code in (C.RTPB_F64, C.RTPB_F32):
            low = E.lower(system.surfaces, materials, lambda: E.distinct_wavelengths(rays[:, 7]), out_code)
            feat = None
            with E.plan_ref(low) as plan:
                for il in (C.RTPB_AOS, C.RTPB_SOA):
                    for ol in (C.RTPB_AOS, C.RTPB_SOA):
                        if il == C.RTPB_SOA and out_code != C.RTPB_F64 and False:
                            continue
                        in_code = out_code
                        x, _, st = M._device_input(rays, in_code, il)
                        got, pad_ok = M._trace((plan, E.plane_mask(sel)), x, in_code, il, st, n, len(sel), out_code, ol)
                        if in_code == C.RTPB_F64:
                            exp = ref.astype(M.NP_DT[out_code])
                        else:
                            continue
                        bad = ~((got == exp) | (np.isnan(got) & np.isnan(exp)))
                        if bad.any() or not pad_ok:
                            fails.append((out_code, il, ol, int(bad.sum()), bad.sum((0, 1)).tolist()))
        print(name, "OK" if not fails else fails, flush=True)


if __name__ == "__main__":
    main()
