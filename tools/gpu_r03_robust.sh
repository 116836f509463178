#!/bin/bash
# Round 3: the C3 headline in three fresh bench processes (history_buffer vs torch.empty beside it).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P=gpurun_out/${1:-r03_robust}
mkdir -p $P
for i in 1 2 3; do
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --cpu-baseline off --traffic off --configs none > $P/bench_fresh$i.log 2>&1 || exit $?
  echo bench$i done
done
