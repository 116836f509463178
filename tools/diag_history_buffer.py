"""Diagnosis of history_buffer traces in the order tests/test_gpu_buffers.py runs them: each trace into a
fresh history_buffer compared (direct copy and via a device clone) with the default allocation."""
import gc
import os
import sys

sys.path[:0] = ['.', 'tests', 'tests/golden']
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ray_trace_pb_amd.materials as mat  # noqa: E402
import ray_trace_pb_amd.raytrace as rt  # noqa: E402
from parity import GOLDEN, same_bits  # noqa: E402
from serialize import system_from_json  # noqa: E402


def case(name):
    d = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    system, m0, m1 = system_from_json(rt, mat, str(d["system_json"]))
    return system, m0, m1, d["rays_in"], d["history"]


for dtype, tdt in ((None, torch.float64), ("float32", torch.float32)):
    for name in ["c1_plano_convex", "c3_relay", "c4_opm", "stress"]:
        system, m0, m1, rays, ref = case(name)
        x = torch.from_numpy(rays).to("cuda:0")
        out = rt.history_buffer(ref.shape, tdt, "cuda:0")
        got = system.ray_trace(x, m0, m1, dtype=dtype, out=out)
        torch.cuda.synchronize()
        a = got.cpu().numpy()
        b = got.clone().cpu().numpy()
        want = system.ray_trace(x, m0, m1, dtype=dtype).cpu().numpy()
        again = got.cpu().numpy()
        bad = [p for p in range(a.shape[0]) if not same_bits(a[p], want[p])]
        badc = [p for p in range(a.shape[0]) if not same_bits(b[p], want[p])]
        bada = [p for p in range(a.shape[0]) if not same_bits(again[p], want[p])]
        print(dtype, name, "bad planes direct", bad, "clone", badc, "reread", bada, "ptr", hex(out.data_ptr()),
              flush=True)
        if bad:
            p = bad[0]
            print("   plane", p, "got", a[p][:2].tolist(), "want", want[p][:2].tolist(), flush=True)
        fin = rt.history_buffer((1,) + ref.shape[1:], tdt, "cuda:0")
        system.ray_trace(x, m0, m1, dtype=dtype, planes="final", out=fin)
        print("   final ok", same_bits(fin.cpu().numpy()[0], want[-1]), "ptr", hex(fin.data_ptr()), flush=True)
        del got, out, fin
        gc.collect()
