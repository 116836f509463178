#!/bin/bash
# Round 3: the GPU test suite, an in-process A/B of the in-tree library against the given builds on the C4
# / C3 / C2 histories and final planes, then the full C5 sweep with each library.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_ab5}
shift
LIBS=$(echo "$@" | tr ' ' ',')
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:warnings --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
echo pytest done
timeout -k 10 900 python3 tools/ab_variants.py --libs "$LIBS" \
  --configs c4:1.0,c3:1.0,c2 --modes all,final --rounds 7 --reps 3 > $OUT/ab.log 2>&1 || exit $?
echo ab done
for lib in "" "$@"; do
  timeout -k 10 300 python3 tools/c5_sweep.py ${lib:+--lib $lib} >> $OUT/c5.log 2>&1 || exit $?
done
echo c5 done
