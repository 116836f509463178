"""Per-channel TCC counters for rocprofv3: writes a copy of rocprofiler-sdk's counter_defs.yaml with derived
counters that select one TCC channel (DIMENSION_INSTANCE, summed over the 8 XCDs) or one XCD (DIMENSION_XCC,
summed over the channels) of TCC_EA0_WRREQ and TCC_EA0_WRREQ_DRAM_CREDIT_STALL, for ROCPROFILER_METRICS_PATH.
rocprofv3's CSV sums a counter over its dimensions; these name each slice.

    python3 tools/placement_counters.py OUT.yaml        # prints the counter names it added
"""
import sys

SRC = "/opt/rocm/share/rocprofiler-sdk/counter_defs.yaml"
BASE = {"WR": "TCC_EA0_WRREQ", "ST": "TCC_EA0_WRREQ_DRAM_CREDIT_STALL"}


def entries():
    out = []
    for tag, ctr in BASE.items():
        for k in range(16):
            out.append((f"RTPB_{tag}_CH{k:02d}", f"reduce(select({ctr},[DIMENSION_INSTANCE=[{k}]]),sum)"))
        for x in range(8):
            out.append((f"RTPB_{tag}_XCC{x}", f"reduce(select({ctr},[DIMENSION_XCC=[{x}]]),sum)"))
    return out


def main():
    dst = sys.argv[1]
    text = open(SRC).read().rstrip("\n") + "\n"
    for name, expr in entries():
        text += (f"  - name: {name}\n    description: per-slice {name}\n    properties: []\n    definitions:\n"
                 f"    - architectures:\n      - gfx950\n      expression: {expr}\n")
    with open(dst, "w") as f:
        f.write(text)
    print(" ".join(n for n, _ in entries()))


if __name__ == "__main__":
    main()
