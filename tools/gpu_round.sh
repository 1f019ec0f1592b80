set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r02b.log 2>&1; rc=$?
echo "tests rc=$rc" ; tail -3 gpurun_out/gpu_tests_r02b.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r02b.json 2> gpurun_out/bench_r02b.err; rc=$?
echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench_r02b.json
