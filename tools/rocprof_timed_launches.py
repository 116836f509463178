"""Per-phase durations of one kernel in a rocprofv3 kernel trace of bench.py: the W warmup launches, the K
timed launches (the ones the bench line's kernel_ms_avg covers), and everything after them (the placement
check into a torch.empty history and the drop-in calls), in dispatch order.

    python tools/rocprof_timed_launches.py TRACE_CSV KERNEL_SUBSTRING [--warmup 5] [--steps 20]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("kernel")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if a.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    w, k = a.warmup, a.steps
    timed, rest = d[w:w + k], d[w + k:]
    print(f"kernel: {rows[0]['Kernel_Name'] if rows else a.kernel}")
    print(f"launches: {len(d)}")
    print(f"warmup ({w}): " + ", ".join(f"{x:.3f}" for x in d[:w]))
    print(f"timed ({k}): avg {sum(timed) / len(timed):.4f} ms, min {min(timed):.4f}, max {max(timed):.4f}")
    if rest:
        print(f"after ({len(rest)}): avg {sum(rest) / len(rest):.4f} ms, min {min(rest):.4f}, max {max(rest):.4f}")
    print(f"all: avg {sum(d) / len(d):.4f} ms")


if __name__ == "__main__":
    main()
