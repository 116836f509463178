#!/bin/bash
# Round 3: where the history kernels' memory path loses against a fill -- store-pattern probes at full
# C3/C4 size and TLB / write-path PMC of the real C4 kernel, its no-compute build and the probes.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03_mem
mkdir -p $OUT
C4B=73607360000
C3B=30404274240
{
for args in "$C4B 1 2" "$C4B 23 2" "$C4B 23 2 10 4096" "$C4B 23 4" "$C4B 23 8" "$C4B 23 16" "$C4B 1 16" \
            "$C3B 19 2 10 4096" "$C3B 1 2" "$C4B 12 4" "$C4B 6 8"; do
  timeout -k 10 120 tools/store_probe $args || exit $?
done
} > $OUT/store_probe.log 2>&1 || exit $?
echo probes done
timeout -k 10 900 bash tools/pmc_groups.sh $OUT/pmc_fill probe_kernel tools/pmc/mempath.txt tools/store_probe $C4B 1 2 3 > $OUT/pmc_fill.txt 2>&1 || exit $?
timeout -k 10 900 bash tools/pmc_groups.sh $OUT/pmc_p23 probe_kernel tools/pmc/mempath.txt tools/store_probe $C4B 23 2 3 4096 > $OUT/pmc_p23.txt 2>&1 || exit $?
echo pmc probes done
timeout -k 10 900 bash tools/pmc_groups.sh $OUT/pmc_c4 trace_kernel tools/pmc/mempath.txt python3 tools/run_variant.py --config c4:1.0 --reps 2 > $OUT/pmc_c4.txt 2>&1 || exit $?
timeout -k 10 900 bash tools/pmc_groups.sh $OUT/pmc_c4nocomp trace_kernel tools/pmc/mempath.txt python3 tools/run_variant.py --config c4:1.0 --reps 2 --lib ray_trace_pb_amd/exp_nocomp.so > $OUT/pmc_c4nocomp.txt 2>&1 || exit $?
echo pmc c4 done
