# A/B of the shared-divisor quotient variants (experiment builds next to the in-tree library)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/fd
timeout -k 10 600 python -u tools/ab_libs.py ray_trace_pb_amd/exp_nofastdiv.so ray_trace_pb_amd/exp_fd_nowl.so ray_trace_pb_amd/exp_fd_nolens.so --configs c5,c4,c2 --dtypes f32,f64 --rounds 11 > gpurun_out/fd/ab_fastdiv2.log 2>&1 || exit $?
