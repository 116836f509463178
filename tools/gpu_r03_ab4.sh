#!/bin/bash
# Round 3: the GPU test suite, then an in-process A/B of the in-tree library against the given
# experiment builds on the full-size C3/C4 histories (all planes) and C2.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_ab4}
shift
LIBS=$(echo "$@" | tr ' ' ',')
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:warnings --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
echo pytest done
timeout -k 10 900 python3 tools/ab_variants.py --libs "$LIBS" \
  --configs c4:1.0,c3:1.0,c2,c5:0.5 --modes all,final --rounds 7 --reps 3 > $OUT/ab.log 2>&1 || exit $?
echo ab done
