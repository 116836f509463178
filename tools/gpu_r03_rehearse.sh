#!/bin/bash
# Round 3: power / clock under the final kernels and the 2-rank torchrun rehearsal of bench.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P=gpurun_out/${1:-r03_rehearse}
mkdir -p $P
bash tools/gpu_r03_power.sh ${1:-r03_rehearse}/power || exit $?
echo power done
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
  bench.py --gpus 2 --steps 20 --warmup 3 > $P/bench_2ranks_1gpu.log 2>&1 || exit $?
echo bench2 done
