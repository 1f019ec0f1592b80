set -u
mkdir -p gpurun_out
ROOT=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_backward_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/bwd_tests.log 2>&1; rc=$?
echo "bwd tests rc=$rc"; tail -3 gpurun_out/bwd_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/prof_bwd2 -o run -- python -u $ROOT/tools/bench_configs.py --only bwd --iters 8 > $ROOT/gpurun_out/prof_bwd2.log 2>&1; rc=$?
grep config $ROOT/gpurun_out/prof_bwd2.log
exit $rc
