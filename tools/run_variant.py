"""Run ONE trace variant a few times (target of rocprofv3 --pmc passes):
python tools/run_variant.py --config c2 --dtype f64 --planes all --layout aos --reps 5"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ray_trace_pb_amd.materials as mat  # noqa: E402
import ray_trace_pb_amd.raytrace as rt  # noqa: E402
from ray_trace_pb_amd import _capi as C  # noqa: E402
from ray_trace_pb_amd import _engine as E  # noqa: E402
import systems  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
ap.add_argument("--rays", type=int, default=1_000_000)
ap.add_argument("--dtype", default="f64")
ap.add_argument("--planes", default="all")
ap.add_argument("--layout", default="aos")
ap.add_argument("--staging", type=int, default=1)
ap.add_argument("--nt", type=int, default=0)
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
if a.config == "c2":
    system, rays, m0, m1 = systems.c2_system(rt, mat), systems.c2_rays(a.rays), mat.Vacuum(), mat.Vacuum()
else:
    system, rays, m0, m1 = systems.c5_system(rt, mat), systems.c5_rays(rt, 1, 101, max(1, a.rays // 707)), \
        mat.Constant(1), mat.Constant(1)
code = C.RTPB_F64 if a.dtype == "f64" else C.RTPB_F32
tdt = torch.float64 if a.dtype == "f64" else torch.float32
dev = torch.device("cuda:0")
x = torch.from_numpy(rays).to(dev, dtype=tdt)
low = E.lower(system.surfaces, [m0] + list(system.materials) + [m1], lambda: np.unique(rays[:, 7]), code)
sel = E.resolve_planes(a.planes, len(system.surfaces))
lc = C.RTPB_AOS if a.layout == "aos" else C.RTPB_SOA
n = x.shape[0]
out = torch.empty((len(sel), n, 8) if lc == C.RTPB_AOS else (len(sel), 8, n), dtype=tdt, device=dev)
C.check(C.lib().rtpb_set_tuning(b"aos_staging", a.staging))
C.check(C.lib().rtpb_set_tuning(b"nt_stores", a.nt))
for _ in range(a.reps):
    E.trace_device(low, x, sel, layout_out=lc, out=out)
torch.cuda.synchronize()
print("done", n, len(sel))
