#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03_diag
mkdir -p $OUT
timeout -k 10 600 python3 tools/ab_variants.py \
  --libs ray_trace_pb_amd/exp_l2input.so,ray_trace_pb_amd/exp_persist.so,ray_trace_pb_amd/exp_noinput.so \
  --configs c4:1.0,c3:1.0 --modes all --rounds 5 --reps 3 > $OUT/ab_diag2.log 2>&1 || exit $?
echo done
