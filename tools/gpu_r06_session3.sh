set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_backward_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/r06_tests3a.log 2>&1
rc=$?; echo "backward tests rc=$rc"; tail -3 $OUT/r06_tests3a.log; [ $rc -eq 0 ] || exit $rc
MPIV_AB_TESTS=1 timeout -k 10 400 python -u -m pytest tests/test_backward_gpu.py -x -q --timeout 200 --timeout-method thread -k "abort or fold or fallback" > $OUT/r06_tests3b.log 2>&1
rc=$?; echo "backward A/B tests rc=$rc"; tail -3 $OUT/r06_tests3b.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/probes/nb_train_probe.py > $OUT/nb_probe2.json 2> $OUT/nb_probe2.err
rc=$?; echo "probe rc=$rc"; cat $OUT/nb_probe2.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/r06_tests3.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/r06_tests3.log
