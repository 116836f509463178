# GPU tests + A/B of the in-tree library against an experiment build (tools/ab_libs.py)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/fd
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:warnings --timeout 120 --timeout-method thread > gpurun_out/fd/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 600 python -u tools/ab_libs.py ray_trace_pb_amd/exp_prev.so --configs c4,c5 --dtypes f32,f64 --rounds 9 > gpurun_out/fd/ab_lens.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/c5_sweep.py > gpurun_out/fd/c5_sweep_lens.log 2>&1 || exit $?
