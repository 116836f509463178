#!/bin/bash
# Round 3: shuffled-chunk (VMM) histories allocated FIRST in the process vs torch ones, full size, two orders.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P=gpurun_out/${1:-r03_alloc}
mkdir -p $P
timeout -k 10 600 python3 tools/placement_alloc.py --pairs 3 --kinds s64,torch > $P/alloc_s64_first.log 2>&1 || exit $?
echo a done
timeout -k 10 600 python3 tools/placement_alloc.py --pairs 3 --kinds torch,s64 > $P/alloc_torch_first.log 2>&1 || exit $?
echo b done
timeout -k 10 600 python3 tools/placement_alloc.py --pairs 3 --kinds s2,torch > $P/alloc_s2_first.log 2>&1 || exit $?
echo c done
