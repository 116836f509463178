#!/bin/bash
# Round 3: contiguous / torch / shuffled-chunk (VMM) allocations of C3 histories, quarter and full size.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P=gpurun_out/${1:-r03_alloc}
mkdir -p $P
timeout -k 10 600 python3 tools/placement_alloc.py --pairs 5 --scale 0.5 --kinds contig,torch,s2,s64 > $P/alloc_q.log 2>&1 || exit $?
echo q done
timeout -k 10 600 python3 tools/placement_alloc.py --pairs 2 --kinds torch,s2,s64 > $P/alloc_full.log 2>&1 || exit $?
echo full done
