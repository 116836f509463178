# GPU check + A/B of the exact division / sqrt fast paths (experiment builds next to the in-tree library)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/fd
timeout -k 10 300 python -u -m pytest tests/test_gpu_fastdiv.py -x -v -p no:warnings --timeout 120 --timeout-method thread > gpurun_out/fd/pytest_fastdiv.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:warnings --timeout 120 --timeout-method thread > gpurun_out/fd/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 600 python -u tools/ab_libs.py ray_trace_pb_amd/exp_nofastsqrt.so ray_trace_pb_amd/exp_nofastdiv.so --configs c5,c4,c2 --dtypes f32,f64 --rounds 11 > gpurun_out/fd/ab_fastsqrt.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/c5_sweep.py > gpurun_out/fd/c5_sweep_sqrt.log 2>&1 || exit $?
