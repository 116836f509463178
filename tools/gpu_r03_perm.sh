#!/bin/bash
# Round 3: block-order permutations of the history kernel judged over several placements of the C3 history.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P=gpurun_out/${1:-r03_perm}
mkdir -p $P
timeout -k 10 600 python3 tools/placement_c3.py --buffers ${NBUF:-4} --pads=${PADS-4096,65537} \
  --libs ${LIBS:-ray_trace_pb_amd/exp_perm1.so,ray_trace_pb_amd/exp_perm16.so,ray_trace_pb_amd/exp_perm256.so} > $P/placement_${TAG:-perm}.log 2>&1 || exit $?
echo placement done
