# PMC counters per output buffer (placement_probe in allocation order, 1 warm + 3 timed dispatches per buffer)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/plpmc
mkdir -p $O
ARGS="--configs c2 --buffers 16 --kinds torch --rounds 1 --reps 3 --order seq"
timeout -k 10 200 python -u tools/placement_probe.py $ARGS > $O/plain.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_HIT_sum --output-format csv -d $O/p1 -o pmc -- python3 tools/placement_probe.py $ARGS > $O/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum --output-format csv -d $O/p2 -o pmc -- python3 tools/placement_probe.py $ARGS > $O/p2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python3 tools/placement_probe.py $ARGS > $O/kt.log 2>&1 || exit $?
