set -u
mkdir -p gpurun_out
TAG=r02b timeout -k 10 900 bash tools/profile.sh > gpurun_out/profile.log 2>&1; rc=$?; tail -3 gpurun_out/profile.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r02d.json 2> gpurun_out/bench_r02d.err; rc=$?; tail -c 1500 gpurun_out/bench_r02d.json; exit $rc
