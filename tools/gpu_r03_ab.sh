#!/bin/bash
# Round 3 A/B: the in-tree library against earlier builds (exp_*.so given as arguments), interleaved in
# one process on full-size C3/C4 histories and C2/C5 (all + final planes), then the full C5 sweep with each.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_ab}
shift
LIBS=$(echo "$@" | tr ' ' ',')
mkdir -p $OUT
timeout -k 10 900 python3 tools/ab_variants.py --libs "$LIBS" \
  --configs c4:1.0,c3:1.0,c2,c5:0.5 --modes all,final --rounds 5 --reps 3 > $OUT/ab.log 2>&1 || exit $?
echo ab done
for lib in "" "$@"; do
  timeout -k 10 300 python3 tools/c5_sweep.py ${lib:+--lib $lib} >> $OUT/c5.log 2>&1 || exit $?
done
echo c5 done
