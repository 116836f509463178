#!/bin/bash
# PMC passes over one command, one rocprofv3 --pmc run per line of GROUPFILE (counters of one pass on one
# line; no tracing domains), summarised for the dispatches whose kernel name contains KERNEL.
# usage: tools/pmc_groups.sh OUTDIR KERNEL GROUPFILE cmd...
OUT=$1; KERNEL=$2; GROUPS_FILE=$3; shift 3
export TMPDIR=/tmp
mkdir -p "$OUT"
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o pmc -- "$@" < /dev/null > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done < "$GROUPS_FILE"
python3 - "$OUT" "$KERNEL" <<'PY'
import csv, glob, os, sys, collections
out, kern = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(list)
for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        if kern in row["Kernel_Name"]:
            agg[row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:44s} median={sorted(v)[len(v)//2]:.6g} n={len(v)}")
PY
