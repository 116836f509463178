#!/bin/bash
# Round 3: placement-robust history buffers -- GPU tests, then the bench line (history_buffer vs torch.empty).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P=gpurun_out/${1:-r03_buffers}
mkdir -p $P
timeout -k 10 300 python -u -m pytest tests/test_gpu_buffers.py -x -v -p no:warnings --timeout 120 --timeout-method thread > $P/pytest_buffers.log 2>&1 || exit $?
echo buffers tests done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:warnings --timeout 300 --timeout-method thread > $P/pytest_gpu.log 2>&1 || exit $?
echo gpu tests done
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > $P/bench.log 2>&1 || exit $?
echo bench done
