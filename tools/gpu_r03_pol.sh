#!/bin/bash
# Round 3: store cache policy nt (exp_pol2) vs the shipped nt|sc1 over several C3 history placements, and
# on C4 / C2 in one process.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P=gpurun_out/${1:-r03_pol}
mkdir -p $P
timeout -k 10 600 python3 tools/placement_c3.py --buffers 6 --pads= --libs ray_trace_pb_amd/exp_pol2.so > $P/placement.log 2>&1 || exit $?
echo placement done
timeout -k 10 600 python3 tools/ab_variants.py --libs ray_trace_pb_amd/exp_pol2.so --configs c4:1.0,c2 --modes all --rounds 7 --reps 3 > $P/ab_c4_c2.log 2>&1 || exit $?
echo ab done
