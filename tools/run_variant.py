"""Run ONE trace variant a few times (target of rocprofv3 --pmc passes):

    python tools/run_variant.py --config c3:0.5 --planes all [--lib ray_trace_pb_amd/exp_prev.so]
        [--knob rays_per_lane=2] [--reps 5]

Configs as tools/ab_variants.py (float64 device fans; C3/C4 stored as float32, C2/C5 as float64)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "tests", "golden")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from ray_trace_pb_amd import _capi as C  # noqa: E402
from ray_trace_pb_amd import _engine as E  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3:0.5")
ap.add_argument("--planes", default="all")
ap.add_argument("--lib", default="")
ap.add_argument("--knob", default="")
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
if a.lib:
    C.LIB_PATH = os.path.abspath(a.lib)
import ab_variants  # noqa: E402

dev = torch.device("cuda:0")
lib = C.lib()
if a.knob:
    k, _, v = a.knob.partition("=")
    C.check(lib.rtpb_set_tuning(k.encode(), int(v)))
system, m0, m1, x, code = ab_variants.build_case(a.config, dev)
wl = np.unique(x[:, 7].cpu().numpy())
low = E.lower(system.surfaces, [m0] + list(system.materials) + [m1], lambda: wl, code)
sel = E.resolve_planes(a.planes, len(system.surfaces))
out = torch.empty((len(sel), x.shape[0], 8), dtype=torch.float64 if code == C.RTPB_F64 else torch.float32, device=dev)
for _ in range(a.reps):
    E.trace_device(low, x, sel, out=out)
torch.cuda.synchronize()
print("done", x.shape[0], len(sel))
