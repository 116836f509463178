#!/bin/bash
# Round-2 GPU session on one MI355X: parity tests, smoke, the C3 headline bench (+C2 secondary, PMC
# traffic, CPU baseline), the rocprofv3 kernel-trace summary of the same bench command, PMC passes of the
# C3 trace kernel, a 2-rank torchrun rehearsal sharing the GPU, and the C3/C4 full-size configs.  Every GPU
# step has its own time limit; a crash/abort/timeout stops the script, test failures (exit 1) do not.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r02}
P=gpurun_out/$TAG
mkdir -p $P
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a $P/steps.log
  timeout -k 10 "$to" "$@" > "$P/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $P/steps.log
  tail -3 "$P/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
if [ -z "$SKIP_TESTS" ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:warnings --timeout 300 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
step bench 900 python bench.py
step rocprof_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d $P/rocprof -o bench -- python3 bench.py --cpu-baseline off --traffic off
if [ -z "$SKIP_EXTRA" ]; then
  step pmc_c3 900 bash tools/pmc_kernel.sh $P/pmc_c3 trace_kernel python3 bench.py --pmc-child --config c3
  step bench_2ranks_1gpu 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 20 --warmup 3
  step configs_c3_c4_full 900 python tools/configs_full.py
fi
exit 0
