#!/bin/bash
# Round 3 check on one MI355X: GPU tests, smoke, the full bench line (C3 headline + C2/C4/C5 configs + PMC +
# CPU baseline), a 2-rank torchrun rehearsal sharing the GPU, and rocprofv3 kernel stats of the bench.
# Every GPU step has its own time limit; a crash/abort/timeout stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P=gpurun_out/${1:-r03_check}
mkdir -p $P
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a $P/steps.log
  timeout -k 10 "$to" "$@" > "$P/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $P/steps.log
  tail -3 "$P/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
shift
for s in "$@"; do
  case $s in
    pytest) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:warnings --timeout 300 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 900 python bench.py --steps 20 --warmup 5 ;;
    bench2) step bench_2ranks_1gpu 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 20 --warmup 3 ;;
    rocprof) step rocprof_stats 900 rocprofv3 --kernel-trace --stats --output-format csv -d $P/rocprof -o bench -- python3 bench.py --cpu-baseline off --traffic off --steps 20 --warmup 5 ;;
  esac
done
exit 0
