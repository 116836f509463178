#!/bin/bash
# Round 3: store cache policy nt (exp_pol2) vs the shipped nt|sc1 over many placements: 16 quarter-size C3
# histories (7.6 GB each), then 6 full-size ones.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P=gpurun_out/${1:-r03_pol}
mkdir -p $P
timeout -k 10 600 python3 tools/placement_c3.py --scale 0.5 --buffers 16 --pads= --libs ${LIBS:-ray_trace_pb_amd/exp_pol2.so} > $P/placement_q16.log 2>&1 || exit $?
echo placement q done
timeout -k 10 600 python3 tools/placement_c3.py --buffers 6 --pads= --libs ${LIBS:-ray_trace_pb_amd/exp_pol2.so} > $P/placement.log 2>&1 || exit $?
echo placement done
