import os, sys
sys.path[:0] = ['.', 'tests', 'tests/golden']
import numpy as np, torch
import ray_trace_pb_amd.materials as mat, ray_trace_pb_amd.raytrace as rt
from parity import GOLDEN, same_bits
from serialize import system_from_json
d = np.load(os.path.join(GOLDEN, "c3_relay.npz"))
system, m0, m1 = system_from_json(rt, mat, str(d["system_json"]))
x = torch.from_numpy(d["rays_in"]).to("cuda:0")
ref = d["history"]
for dtype, tdt in ((None, torch.float64), ("float32", torch.float32)):
    want = system.ray_trace(x, m0, m1, dtype=dtype).cpu().numpy()
    for trial in range(3):
        out = rt.history_buffer(ref.shape, tdt, "cuda:0")
        out.fill_(-7.0)
        got = system.ray_trace(x, m0, m1, dtype=dtype, out=out)
        torch.cuda.synchronize()
        a = got.cpu().numpy()
        b = got.clone().cpu().numpy()
        bad = [p for p in range(a.shape[0]) if not same_bits(a[p], want[p])]
        badc = [p for p in range(a.shape[0]) if not same_bits(b[p], want[p])]
        print(dtype, trial, "direct-bad-planes", bad, "clone-bad-planes", badc, "ptr", hex(out.data_ptr()), flush=True)
        if bad:
            p = bad[0]
            print("  plane", p, "got[:2]", a[p][:2], "want[:2]", want[p][:2], flush=True)
    t2 = torch.empty(ref.shape, dtype=tdt, device="cuda:0")
    g2 = system.ray_trace(x, m0, m1, dtype=dtype, out=t2).cpu().numpy()
    print(dtype, "torch out bad planes", [p for p in range(g2.shape[0]) if not same_bits(g2[p], want[p])], flush=True)
