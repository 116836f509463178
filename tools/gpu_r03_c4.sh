#!/bin/bash
# Round 3: C4 (BASELINE configs[3]) history kernel evidence on one MI355X -- kernel trace, PMC passes
# (incl. TCC write-path counters) and a no-compute A/B, each step under its own time limit.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03_c4
mkdir -p $OUT
timeout -k 10 60 rocprofv3 -L > $OUT/counters_avail.txt 2>&1 || true
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ktrace -o c4 -- \
    python3 tools/configs_full.py --which c4 --reps 10 --check 2000 > $OUT/ktrace.log 2>&1 || exit $?
echo "ktrace done"
timeout -k 10 600 bash tools/pmc_kernel.sh $OUT/pmc trace_kernel python3 tools/configs_full.py --which c4 --reps 1 --check 100 \
    > $OUT/pmc_summary.txt 2>&1 || exit $?
echo "pmc done"
timeout -k 10 300 python3 tools/ab_variants.py --libs ray_trace_pb_amd/exp_nocomp.so --configs c4:1.0 --modes all,final \
    --rounds 5 --reps 3 > $OUT/ab_nocomp.log 2>&1 || exit $?
echo "ab done"
