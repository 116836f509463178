#!/bin/bash
# Round 3: store patterns vs history placement (tools/store_multi.py): 24 quarter-size, then 6 full-size buffers.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P=gpurun_out/${1:-r03_storemulti}
mkdir -p $P
timeout -k 10 600 python3 tools/store_multi.py --buffers 24 --scale 0.5 > $P/store_multi_q24.log 2>&1 || exit $?
echo q done
timeout -k 10 600 python3 tools/store_multi.py --buffers 6 --scale 1.0 > $P/store_multi_full.log 2>&1 || exit $?
echo full done
