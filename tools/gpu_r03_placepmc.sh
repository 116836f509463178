#!/bin/bash
# Round 3: why some placements of the C3 history trace slower -- per-buffer timing (sequential, in
# allocation order), then TLB / write-path PMC per dispatch of the same sequence.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P=gpurun_out/${1:-r03_placepmc}
mkdir -p $P
ARGS="--buffers 6 --pads= --sequential --rounds 1 --reps 2"
timeout -k 10 300 python3 tools/placement_c3.py $ARGS > $P/timing.log 2>&1 || exit $?
echo timing done
timeout -k 10 700 bash tools/pmc_groups.sh $P/pmc trace_kernel tools/pmc/tlb_write.txt python3 tools/placement_c3.py $ARGS > $P/pmc_summary.txt 2>&1 || exit $?
python3 tools/pmc_dispatches.py $P/pmc trace_kernel > $P/pmc_dispatches.txt 2>&1
echo pmc done
