#!/bin/bash
# Round 3: is a slow history placement a property of the output buffer or of its position relative to the
# input rays?  24 quarter-size C3 histories traced from the original rays and from a copy allocated after
# them; then 6 full-size ones.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P=gpurun_out/${1:-r03_rays}
mkdir -p $P
timeout -k 10 600 python3 tools/placement_c3.py --scale 0.5 --buffers 24 --pads= --rays-copy > $P/placement_q24.log 2>&1 || exit $?
echo q done
timeout -k 10 600 python3 tools/placement_c3.py --buffers 6 --pads= --rays-copy > $P/placement_full.log 2>&1 || exit $?
echo full done
