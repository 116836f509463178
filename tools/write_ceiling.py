"""Write-bandwidth ceiling probes on one MI355X: torch fill_ / zero_ / hipMemset-backed zero of a
704 MB buffer vs the device ray-fan kernel (pure staged writes)."""
import torch
import numpy as np


def timed(fn, reps=50):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    dev = torch.device("cuda:0")
    for mb in (704, 2816):
        n = mb * 1000 * 1000 // 8
        buf = torch.empty(n, dtype=torch.float64, device=dev)
        for name, fn in (("fill_(1.5)", lambda: buf.fill_(1.5)), ("zero_()", lambda: buf.zero_())):
            ms = timed(fn)
            print(f"{mb:5d} MB {name:12s} {ms:.4f} ms  {n * 8 / ms / 1e6:.0f} GB/s")
        del buf
    import sys, os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import ray_trace_pb_amd.raytrace as rt
    out = torch.empty((11_000_000, 8), dtype=torch.float64, device=dev)
    ms = timed(lambda: rt.fan_into(out, [0, 0, 0], 0.1, 11000, 0.5, 1000))
    print(f"  704 MB ray fan     {ms:.4f} ms  {out.numel() * 8 / ms / 1e6:.0f} GB/s (API incl. host tables)")


if __name__ == "__main__":
    main()
