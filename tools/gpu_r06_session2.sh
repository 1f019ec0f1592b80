set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_assemble_gpu.py tests/test_u8_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/r06_tests2a.log 2>&1
rc=$?; echo "assemble/u8 tests rc=$rc"; tail -3 $OUT/r06_tests2a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/r06_tests2.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/r06_tests2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py > $OUT/r06_bench2.json 2> $OUT/r06_bench2.err
rc=$?; echo "bench rc=$rc"; tail -c 400 $OUT/r06_bench2.err
