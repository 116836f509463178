#!/bin/bash
# Round 3: placement of the C3 history (several separately allocated / plane-stride-padded buffers in one
# process), then two bench runs in fresh processes (is a slow headline a property of the process's first
# allocations?).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P=gpurun_out/${1:-r03_place}
mkdir -p $P
timeout -k 10 400 python3 tools/placement_c3.py --buffers 4 --pads 64,4096,65537 > $P/placement_c3.log 2>&1 || exit $?
echo placement done
for i in 1 2; do
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --cpu-baseline off --traffic off > $P/bench$i.log 2>&1 || exit $?
  echo bench$i done
done
