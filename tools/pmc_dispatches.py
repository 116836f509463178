"""Per-dispatch PMC values (in dispatch order) of the kernels whose name contains KERNEL, from the
rocprofv3 --pmc CSVs under OUTDIR (one subdirectory per pass, as tools/pmc_groups.sh writes them).

    python tools/pmc_dispatches.py OUTDIR KERNEL
"""
import collections
import csv
import glob
import os
import sys


def main():
    out, kern = sys.argv[1], sys.argv[2]
    for d in sorted(glob.glob(os.path.join(out, "p*")), key=lambda q: (len(q), q)):
        if not os.path.isdir(d):
            continue
        rows = collections.defaultdict(dict)
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                if kern in row["Kernel_Name"]:
                    rows[int(row["Dispatch_Id"])][row["Counter_Name"]] = float(row["Counter_Value"])
        if not rows:
            continue
        names = sorted({k for r in rows.values() for k in r})
        print(f"== {os.path.basename(d)}: dispatch " + " ".join(names))
        for i, (did, r) in enumerate(sorted(rows.items())):
            print(f"{i:3d} {did:6d} " + " ".join(f"{r.get(k, float('nan')):.4g}" for k in names))


if __name__ == "__main__":
    main()
