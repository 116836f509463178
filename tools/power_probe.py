"""Socket power and shader clock while one trace variant runs back to back (read-only rocm-smi samples):
tests whether a history kernel is power-limited (DVFS) rather than bound by HBM or by the VALU alone.

    python tools/power_probe.py --config c4:1.0 --planes all [--lib exp.so] [--seconds 6]
"""
import argparse
import json
import os
import re
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "tests", "golden")]
import numpy as np  # noqa: E402


def sample(stop, out):
    while not stop.is_set():
        try:
            r = subprocess.run(["rocm-smi", "--showpower", "--showgpuclocks", "--json"], capture_output=True,
                               text=True, timeout=10)
            out.append((time.perf_counter(), r.stdout))
        except Exception as e:  # noqa: BLE001
            out.append((time.perf_counter(), repr(e)))
        time.sleep(0.3)


def parse(txt):
    try:
        d = json.loads(txt)
    except ValueError:
        return None, None
    card = next(iter(d.values()))
    power = clock = None
    for k, v in card.items():
        kl = k.lower()
        if "power" in kl and "(w)" in kl:
            try:
                power = float(v)
            except ValueError:
                pass
        if "sclk" in kl:
            m = re.search(r"\((\d+)\s*mhz\)", str(v).lower())
            if m:
                clock = float(m.group(1))
    return power, clock


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4:1.0")
    ap.add_argument("--planes", default="all")
    ap.add_argument("--lib", default="")
    ap.add_argument("--seconds", type=float, default=6.0)
    a = ap.parse_args()
    import torch
    from ray_trace_pb_amd import _capi as C
    if a.lib:
        C.LIB_PATH = os.path.abspath(a.lib)
    from ray_trace_pb_amd import _engine as E
    import ab_variants
    dev = torch.device("cuda:0")
    system, m0, m1, x, code = ab_variants.build_case(a.config, dev)
    wl = np.unique(x[:, 7].cpu().numpy())
    low = E.lower(system.surfaces, [m0] + list(system.materials) + [m1], lambda: wl, code)
    sel = E.resolve_planes(a.planes, len(system.surfaces))
    out = torch.empty((len(sel), x.shape[0], 8), dtype=torch.float64 if code == C.RTPB_F64 else torch.float32,
                      device=dev)
    E.trace_device(low, x, sel, out=out)
    torch.cuda.synchronize()
    idle = []
    stop = threading.Event()
    th = threading.Thread(target=sample, args=(stop, idle))
    th.start()
    time.sleep(1.0)
    stop.set()
    th.join()
    samples = []
    stop = threading.Event()
    th = threading.Thread(target=sample, args=(stop, samples))
    t0 = time.perf_counter()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 0
    th.start()
    ev0.record()
    while time.perf_counter() - t0 < a.seconds:
        for _ in range(10):
            E.trace_device(low, x, sel, out=out)
            n += 1
        torch.cuda.synchronize()
    ev1.record()
    torch.cuda.synchronize()
    stop.set()
    th.join()
    ms = ev0.elapsed_time(ev1) / n
    busy = [parse(s) for t, s in samples if t - t0 > 1.0]
    idle_p = [parse(s) for _, s in idle]
    res = {"config": a.config, "planes": a.planes, "lib": a.lib or "in-tree", "kernel_ms": ms, "launches": n,
           "busy_power_W": [p for p, _ in busy], "busy_sclk_MHz": [c for _, c in busy],
           "idle_power_W": [p for p, _ in idle_p], "idle_sclk_MHz": [c for _, c in idle_p],
           "raw_first": samples[len(samples) // 2][1][:2000] if samples else None}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
