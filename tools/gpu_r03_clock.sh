#!/bin/bash
# Effective shader clock of the C4 history kernel, its final-plane-only form and its memory path alone:
# GRBM_GUI_ACTIVE per dispatch (one --pmc pass, kernel trace in the same run for the durations).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_clock}
mkdir -p $OUT
run() {  # tag args...
  local tag=$1; shift
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/$tag -o $tag -- \
    python3 tools/run_variant.py "$@" --reps 3 < /dev/null > $OUT/$tag.log 2>&1 || exit $?
  echo "$tag done"
}
run c4all --config c4:1.0 --planes all
run c4final --config c4:1.0 --planes final
run c4nocomp --config c4:1.0 --planes all --lib ray_trace_pb_amd/exp_nocomp.so
run c3all --config c3:1.0 --planes all
run c3final --config c3:1.0 --planes final
