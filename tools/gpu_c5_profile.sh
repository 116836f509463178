export TMPDIR=/tmp
P=gpurun_out/r02_c5
mkdir -p $P
timeout -k 10 300 python -u -m pytest tests/test_gpu_analysis.py -q -x -p no:warnings --timeout 200 --timeout-method thread > $P/pytest_analysis.log 2>&1 || exit 1
tail -2 $P/pytest_analysis.log
timeout -k 10 300 python tools/c5_sweep.py > $P/c5_sweep_full.log 2>&1 || exit 1
tail -1 $P/c5_sweep_full.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/rocprof -o c5 -- python3 tools/c5_sweep.py --warmup 0 > $P/rocprof.log 2>&1 || exit 1
timeout -k 10 900 bash tools/pmc_kernel.sh $P/pmc sweep_kernel python3 tools/c5_sweep.py --fields 16 --warmup 0 > $P/pmc_summary.txt 2>&1
tail -25 $P/pmc_summary.txt
