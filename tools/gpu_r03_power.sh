#!/bin/bash
# Socket power and shader clock (read-only rocm-smi samples) while the C3/C4 history kernels, their
# final-plane forms and the memory path alone run back to back.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_power}
mkdir -p $OUT
timeout -k 10 30 rocm-smi --showmaxpower --showpower --showgpuclocks --json > $OUT/smi_idle.json 2>&1 || true
for args in "--config c4:1.0 --planes all" "--config c4:1.0 --planes final" "--config c4:1.0 --planes all --lib ray_trace_pb_amd/exp_nocomp.so" \
            "--config c3:1.0 --planes all" "--config c3:1.0 --planes final"; do
  lib=$(echo "$args" | sed -n 's/.*--lib \([^ ]*\).*/\1/p')
  if [ -n "$lib" ] && [ ! -f "$lib" ]; then echo "$args skipped ($lib not built)"; continue; fi
  timeout -k 10 120 python3 tools/power_probe.py $args --seconds 6 >> $OUT/power.log 2>&1 || exit $?
  echo "$args done"
done
