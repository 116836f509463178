#!/bin/bash
# Per-channel PMC of the placement study (tools/placement_channels.py): derived counters selecting one TCC channel /
# one XCD (tools/placement_counters.py, ROCPROFILER_METRICS_PATH), checked on a tiny workload first.
# usage: tools/placement_pmc.sh OUTDIR
OUT=$1
export TMPDIR=/tmp
mkdir -p "$OUT"
python3 tools/placement_counters.py "$OUT/counter_defs.yaml" > "$OUT/custom_counters.txt" || exit 1
# rocprofiler-sdk reads counter_defs.yaml from the directory ROCPROFILER_METRICS_PATH names (a file path is not
# accepted: round-5 run r05_j listed none of the derived counters); the file form is tried second
ok=0
for path in "$OUT" "$OUT/counter_defs.yaml"; do
  export ROCPROFILER_METRICS_PATH="$path"
  timeout -s KILL 120 rocprofv3 -L > "$OUT/list.txt" 2>&1
  echo "ROCPROFILER_METRICS_PATH=$path: custom counters listed: $(grep -c 'RTPB_' "$OUT/list.txt")"
  if grep -q RTPB_WR_CH00 "$OUT/list.txt"; then ok=1; break; fi
done
[ $ok = 1 ] || { echo "derived counters not accepted"; exit 3; }
run() {  # tag limit counters...
  local tag=$1 lim=$2; shift 2
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/probe_$tag" -o pmc -- \
    python3 -c "import torch; x = torch.ones(1 << 24, device='cuda'); y = x * 2; torch.cuda.synchronize()" \
    > "$OUT/probe_$tag.log" 2>&1 || { echo "probe $tag failed rc=$?"; return 1; }
  timeout -s KILL "$lim" rocprofv3 --pmc "$@" --output-format csv -d "$OUT/pmc_$tag" -o pmc -- \
    python3 tools/placement_channels.py --buffers 6 > "$OUT/run_$tag.log" 2>&1 || { echo "run $tag failed rc=$?"; return 1; }
  python3 tools/placement_channels.py --analyze "$OUT/pmc_$tag" --log "$OUT/run_$tag.log" > "$OUT/analysis_$tag.txt" 2>&1
  cat "$OUT/analysis_$tag.txt"
}
CH_WR=$(for k in $(seq -w 0 15); do printf "RTPB_WR_CH%s " "$k"; done)
CH_ST=$(for k in $(seq -w 0 15); do printf "RTPB_ST_CH%s " "$k"; done)
XCC=$(for x in 0 1 2 3 4 5 6 7; do printf "RTPB_WR_XCC%s RTPB_ST_XCC%s " "$x" "$x"; done)
run ch_wr 600 $CH_WR && run ch_st 600 $CH_ST && run xcc 600 $XCC
