#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_ab2}
mkdir -p $OUT
timeout -k 10 600 python3 tools/ab_variants.py --libs ray_trace_pb_amd/exp_prev.so,ray_trace_pb_amd/exp_oldkill.so,ray_trace_pb_amd/exp_oldchk.so,ray_trace_pb_amd/exp_noratio.so \
  --configs c5:0.5,c3:0.5,c4:0.5,c2 --modes final,all --rounds 5 --reps 3 > $OUT/ab.log 2>&1 || exit $?
echo ab done
