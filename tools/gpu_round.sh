#!/bin/bash
# Round artifacts on one MI355X: parity tests, smoke, bench (+PMC traffic), a 2-rank torchrun rehearsal
# sharing the GPU, rocprofv3 kernel-trace stats of the bench, PMC passes, and the variant sweep.
# Every GPU step has its own time limit; a crash/abort/timeout stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r01}
P=gpurun_out/profiles_$TAG
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
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:warnings --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py
step bench_2ranks_1gpu 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 20 --warmup 3
step rocprof_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d $P/rocprof -o bench -- python3 bench.py --cpu-baseline off --traffic off
step pmc_all 900 bash tools/pmc_profile.sh $P/pmc_all --planes all
step pmc_final 900 bash tools/pmc_profile.sh $P/pmc_final --planes final
step sweep 600 python tools/perf_sweep.py --configs c2,c5,c4
step bench_aux 300 python tools/bench_aux.py
step rocprof_aux 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/rocprof_aux -o aux -- python3 tools/bench_aux.py
step configs_c3_c4_full 900 python tools/configs_full.py
step c5_sweep_full 900 python tools/c5_sweep.py
exit 0
