# bench.py kernel time vs warm-up length (clock ramp / steady state probe)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/warm
for w in 5 20 2000 5 2000 20; do
  timeout -k 10 120 python bench.py --warmup $w --steps 200 --cpu-baseline off --traffic off > gpurun_out/warm/w$w.$RANDOM.log 2>&1 || exit $?
done
grep -ho '"warmup": [0-9]*\|"kernel_ms_avg": [0-9.]*' gpurun_out/warm/*.log | paste - - > gpurun_out/warm/summary.txt
