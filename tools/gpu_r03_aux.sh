#!/bin/bash
# Round 3: the SURVEY 8(f) kernels around the trace (device generators, intersect_rays, spot statistics,
# propagate_ray2plane, hook kernels), the streaming writer and the PSF pipeline, each under its own limit,
# plus rocprofv3 kernel stats of the aux bench.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_aux}
mkdir -p $OUT
timeout -k 10 300 python3 tools/bench_aux.py > $OUT/bench_aux.log 2>&1 || exit $?
echo aux done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rocprof -o aux -- python3 tools/bench_aux.py > $OUT/rocprof_aux.log 2>&1 || exit $?
echo rocprof done
timeout -k 10 300 python3 tools/bench_writer.py --dir /tmp/rtpb_writer > $OUT/bench_writer.log 2>&1 || exit $?
echo writer done
timeout -k 10 600 python3 tools/bench_psf.py > $OUT/bench_psf.log 2>&1 || exit $?
echo psf done
