#!/bin/bash
# The one GPU runner (replaces round 3's per-experiment gpu_r03_*.sh scripts): runs the named steps on one
# MI355X, each under its own time limit, output under gpurun_out/OUT/; any step that fails, aborts or times out
# ends the script (nothing more runs on the GPU after a fault).
#
#   tools/gpu_run.sh OUT STEP [STEP ...]
#
# steps:
#   tests            all GPU tests (pytest -m gpu)
#   tests:EXPR       GPU tests selected by a pytest path or -k expression (tests:tests/test_gpu_buffers.py,
#                    tests:k=writer)
#   smoke            __graft_entry__.smoke()
#   bench            python bench.py --steps 20 --warmup 5 (the bench line; PMC traffic child runs included)
#   bench2           the N>1 path rehearsed: python bench.py --gpus 2 --oversubscribe (2 ranks, one GPU)
#   bench2pmc        the same with rank 0's PMC child runs (C4 traffic of its shard, C5 FLOP roofline)
#   rocprof          rocprofv3 --kernel-trace --stats of the headline loop alone (--extras off: the csv
#                    average is the timed launches' average) + the timed-launch split
#   pmc_c3|pmc_c4    PMC passes (tools/pmc_kernel.sh) of the C3 / C4 history kernel
#   pmc_c5           PMC passes of the fused C5 sweep kernel (1 field)
#   e2e              host phases of the drop-in call (tools/e2e_phases.py)
#   power            socket power / clock under the history kernels (tools/power_probe.py)
#   placement        per-channel TCC write requests / stalls of the slowest and fastest of 6 C3 history buffers
#                    (tools/placement_channels.py under rocprofv3 --pmc, JSON output: one value per instance)
#   counters         rocprofv3 -L (the PMC counters and their dimensions on this box)
#   vmm              tests/native/vmm_remap_check (HIP virtual-memory remapping, no torch; built in-tree)
#   vmmtorch         the same check on torch's HIP runtime (tools/vmm_torch_runtime.py)
#   e2e:CONFIG       host phases of the drop-in call for one bench config (e2e:c2)
#   dangling         round 5's MemPool crash reproduced in child processes (tools/mempool_dangling.py): a child
#                    killed by SIGSEGV is the expected result of one case, so this must be the LAST step
#   valu             issue cost of the kernels' VALU instructions (tools/valu/valu_rates.hip, built in-tree)
#   ab:LIB[,LIB..]   A/B of the in-tree library against experiment builds (tools/ab_variants.py, histories;
#                    C5 sweep per library, the in-tree one before and after)
#   py:SCRIPT[:ARGS] python3 tools/SCRIPT.py ARGS (ARGS with ',' for spaces)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P=gpurun_out/${1:?usage: tools/gpu_run.sh OUT STEP...}
shift
mkdir -p "$P"
step() {  # name timeout cmd...  (a repeated name gets a suffix: _2, _3, ...)
  local name=$1 to=$2; shift 2
  local base=$name k=2
  while [ -e "$P/$name.log" ]; do name="${base}_$k"; k=$((k+1)); done
  echo "=== $name: $*" | tee -a "$P/steps.log"
  timeout -k 10 "$to" "$@" < /dev/null > "$P/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a "$P/steps.log"
  tail -3 "$P/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
PYTEST="python -u -m pytest -m gpu -x -v -p no:warnings --tb=short --timeout 600 --timeout-method thread"
for s in "$@"; do
  case "$s" in
    tests) step pytest_gpu 1500 $PYTEST tests ;;
    tests:k=*) step "pytest_${s#tests:k=}" 900 $PYTEST tests -k "${s#tests:k=}" ;;
    tests:*) step "pytest_$(basename "${s#tests:}" .py)" 900 $PYTEST "${s#tests:}" ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 900 python bench.py --steps 20 --warmup 5 ;;
    bench2) step bench2 900 python bench.py --gpus 2 --oversubscribe --steps 20 --warmup 3 --cpu-baseline off --traffic off ;;
    bench2pmc) step bench2pmc 900 python bench.py --gpus 2 --oversubscribe --steps 10 --warmup 3 --cpu-baseline off ;;
    rocprof)
      step rocprof_c3 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$P/rocprof" -o c3 -- \
        python3 bench.py --configs none --extras off --cpu-baseline off --traffic off --steps 20 --warmup 5
      trace=$(find "$P/rocprof" -name 'c3_kernel_trace.csv' | sort | tail -n 1)
      if [ -n "$trace" ]; then
        python3 tools/rocprof_timed_launches.py "$trace" trace_kernel --warmup 5 --steps 20 > "$P/rocprof_c3_timed_launches.txt"
        cat "$P/rocprof_c3_timed_launches.txt"
      fi ;;
    pmc_c3) step pmc_c3 900 bash tools/pmc_kernel.sh "$P/pmc_c3" trace_kernel python3 tools/run_variant.py --config c3:1.0 --reps 2 ;;
    pmc_c4) step pmc_c4 900 bash tools/pmc_kernel.sh "$P/pmc_c4" trace_kernel python3 tools/run_variant.py --config c4:1.0 --reps 2 ;;
    pmc_c5) step pmc_c5 900 bash tools/pmc_kernel.sh "$P/pmc_c5" sweep_kernel python3 tools/c5_sweep.py --fields 1 --warmup 0 ;;
    e2e) step e2e 600 python3 tools/e2e_phases.py ;;
    e2e:*) step "e2e_${s#e2e:}" 600 python3 tools/e2e_phases.py --config "${s#e2e:}" --reps 31 ;;
    vmmtorch) step vmm_torch_runtime 300 python3 tools/vmm_torch_runtime.py 10 ;;
    dangling) step mempool_dangling 300 python3 tools/mempool_dangling.py ;;
    valu) step valu 300 tools/valu/_build/valu_rates ;;
    vmm) step vmm 300 tests/native/_build/vmm_remap_check 10 ;;
    counters) step counters 120 rocprofv3 -L ;;
    placement)
      step placement 900 rocprofv3 --pmc TCC_EA0_WRREQ TCC_EA0_WRREQ_DRAM_CREDIT_STALL TCC_EA0_WRREQ_STALL \
        --output-format csv json -d "$P/placement" -o pmc -- python3 tools/placement_channels.py --buffers 6
      python3 tools/placement_channels.py --analyze "$P/placement" --log "$P/placement.log" > "$P/placement_analysis.txt" 2>&1
      cat "$P/placement_analysis.txt" ;;
    power)
      for args in "--config c4:1.0 --planes all" "--config c4:1.0 --planes final" "--config c3:1.0 --planes all" \
                  "--config c3:1.0 --planes final"; do
        step "power_$(echo $args | tr -c 'a-z0-9' '_')" 120 python3 tools/power_probe.py $args --seconds 6
      done ;;
    ab:*)
      libs="${s#ab:}"
      step ab_hist 900 python3 tools/ab_variants.py --libs "$libs" --configs c4:1.0,c3:1.0,c2 --modes all,final --rounds 5 --reps 3
      step c5_new 300 python3 tools/c5_sweep.py
      for lib in $(echo "$libs" | tr ',' ' '); do
        step "c5_$(basename "$lib" .so)" 300 python3 tools/c5_sweep.py --lib "$lib"
      done
      step c5_new_again 300 python3 tools/c5_sweep.py ;;
    py:*)
      spec="${s#py:}"; script="${spec%%:*}"; args=""
      [ "$spec" != "$script" ] && args="$(echo "${spec#*:}" | tr ',' ' ')"
      step "py_$script" 900 python3 "tools/$script.py" $args ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
exit 0
