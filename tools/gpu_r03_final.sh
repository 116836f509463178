#!/bin/bash
# Round 3 final artefacts on one MI355X: GPU tests, smoke, the bench line (C3 headline + C2/C4/C5 + PMC +
# CPU baseline), rocprofv3 kernel stats of the bench, PMC passes of the C4 and C3 history kernels and the
# C5 sweep, power/clock samples, 2-rank rehearsal.  Each GPU step has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P=gpurun_out/${1:-r03_final}
mkdir -p $P
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a $P/steps.log
  timeout -k 10 "$to" "$@" < /dev/null > "$P/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $P/steps.log
  tail -2 "$P/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:warnings --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
# the in-tree build against the previous commit's (when tools/ built it as exp_prev.so): histories, then the C5 sweep
if [ -f ray_trace_pb_amd/exp_prev.so ]; then
  step ab_prev 900 python3 tools/ab_variants.py --libs ray_trace_pb_amd/exp_prev.so --configs c4:1.0,c3:1.0,c2 --modes all,final --rounds 7 --reps 3
  step c5_new 300 python3 tools/c5_sweep.py
  step c5_prev 300 python3 tools/c5_sweep.py --lib ray_trace_pb_amd/exp_prev.so
fi
step bench 900 python bench.py --steps 20 --warmup 5
step rocprof_stats 900 rocprofv3 --kernel-trace --stats --output-format csv -d $P/rocprof -o bench -- python3 bench.py --cpu-baseline off --traffic off --steps 20 --warmup 5
step pmc_c4 900 bash tools/pmc_kernel.sh $P/pmc_c4 trace_kernel python3 tools/run_variant.py --config c4:1.0 --reps 2
step pmc_c3 900 bash tools/pmc_kernel.sh $P/pmc_c3 trace_kernel python3 tools/run_variant.py --config c3:1.0 --reps 2
step pmc_c5 900 bash tools/pmc_kernel.sh $P/pmc_c5 sweep_kernel python3 tools/c5_sweep.py --fields 1 --warmup 0
step power 600 bash tools/gpu_r03_power.sh ${1:-r03_final}/power
step bench2 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 20 --warmup 3
exit 0
