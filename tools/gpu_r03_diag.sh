#!/bin/bash
# Round 3: where the C3 / C4 history kernels spend their time -- interleaved A/B of the shipped kernel
# against its memory path alone (nocomp), its compute side alone (nostore), no input reads (noinput) and
# the pre-round-3 build (prev), full-size C3 and C4.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03_diag
mkdir -p $OUT
timeout -k 10 600 python3 tools/ab_variants.py \
  --libs ray_trace_pb_amd/exp_prev.so,ray_trace_pb_amd/exp_nocomp.so,ray_trace_pb_amd/exp_nostore.so,ray_trace_pb_amd/exp_noinput.so \
  --configs c4:1.0,c3:1.0 --modes all --rounds 5 --reps 3 > $OUT/ab_diag.log 2>&1 || exit $?
echo done
