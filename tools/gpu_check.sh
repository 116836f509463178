#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprof kernel-trace summary.  Each GPU step has its own
# time limit; a crash/abort/timeout (exit >= 124 or signal) stops the script, test failures (exit 1) do not.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r01}
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/steps.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:warnings --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 50 --warmup 5
step sweep 600 python tools/perf_sweep.py --configs c2,c5,c4
step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o bench -- python3 bench.py --steps 20 --warmup 3 --cpu-baseline off --traffic off
exit 0
