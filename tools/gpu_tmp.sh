set -u
mkdir -p gpurun_out
ROOT=$(pwd)
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r02e.json 2> gpurun_out/bench_r02e.err; rc=$?
echo "bench rc=$rc"; tail -c 2500 gpurun_out/bench_r02e.json
exit $rc
