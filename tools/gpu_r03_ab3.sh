#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_ab3}
mkdir -p $OUT
timeout -k 10 600 python3 tools/ab_variants.py --knobs aos_staging=1,2 --configs c4:1.0,c3:1.0 --modes all,final --rounds 7 --reps 3 > $OUT/ab_xchg.log 2>&1 || exit $?
echo ab done
