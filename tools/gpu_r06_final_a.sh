# Round-6 final evidence, part A: GPU parity tests (default and with the A/B-variant tests), smoke(),
# the default bench line and the 2-rank gloo rehearsal.  Every GPU step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rs > $OUT/r06d_final_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/r06d_final_tests.log; [ $rc -eq 0 ] || exit $rc
MPIV_AB_TESTS=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/r06d_final_tests_ab.log 2>&1
rc=$?; echo "tests (A/B incl.) rc=$rc"; tail -2 $OUT/r06d_final_tests_ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/r06d_final_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/r06d_final_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py > $OUT/r06d_final_bench.json 2> $OUT/r06d_final_bench.err
rc=$?; echo "bench rc=$rc"; tail -c 300 $OUT/r06d_final_bench.err; [ $rc -eq 0 ] || exit $rc
MPIV_BENCH_BACKEND=gloo MPIV_BENCH_ONE_DEVICE=1 timeout -k 10 400 python3 -u bench.py --gpus 2 --steps 3 --warmup 1 \
    --cpu-seconds 0 > $OUT/r06d_final_bench2.json 2> $OUT/r06d_final_bench2.err
rc=$?; echo "bench --gpus 2 rc=$rc"; tail -c 300 $OUT/r06d_final_bench2.err
