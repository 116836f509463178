"""Debug helper: which rays the deferred guards of the final-plane kernel flag (exp build with
-DRTPB_EXP_MARK_BAD writes x = 12345 for them)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "tests", "golden")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ab_variants  # noqa: E402
from ray_trace_pb_amd import _capi as C  # noqa: E402
from ray_trace_pb_amd import _engine as E  # noqa: E402


def main():
    lib = ab_variants.load(sys.argv[1])
    dev = torch.device("cuda:0")
    for cfg in sys.argv[2].split(","):
        system, m0, m1, x, code = ab_variants.build_case(cfg, dev)
        n, S = x.shape[0], len(system.surfaces)
        low = E.lower(system.surfaces, [m0] + list(system.materials) + [m1],
                      lambda: E.distinct_wavelengths(x[:, 7]), code)
        import ctypes
        plan = ctypes.c_void_p()
        C.check(lib.rtpb_plan_create(low.surfaces, low.nsurf, low.materials, low.nsurf + 1, low.dtype, ctypes.byref(plan)))
        out = torch.empty((1, n, 8), dtype=torch.float64 if code == C.RTPB_F64 else torch.float32, device=dev)
        lo, hi = E.plane_mask([2 * S])
        in_code = C.RTPB_F64 if x.dtype == torch.float64 else C.RTPB_F32
        rc = lib.rtpb_trace(plan, 0, x.data_ptr(), in_code, n, C.RTPB_AOS, 0, out.data_ptr(), C.RTPB_AOS, 8 * n, 0, lo, hi,
                            torch.cuda.current_stream(dev).cuda_stream)
        assert rc == 0
        torch.cuda.synchronize()
        bad = (out[0, :, 0] == 12345.0).nonzero().flatten().cpu().numpy()
        print(cfg, "rays", n, "flagged", bad.size, "waves with a flag", np.unique(bad // 64).size, "of", (n + 63) // 64)
        for k in bad[:5]:
            print("  ray", k, x[k].cpu().numpy())


if __name__ == "__main__":
    main()
