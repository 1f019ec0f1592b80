set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out; mkdir -p $OUT
MPIV_AB_TESTS=1 timeout -k 10 500 python -u -m pytest tests/test_backward_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/r06_tests4a.log 2>&1
rc=$?; echo "backward tests (A/B incl.) rc=$rc"; tail -3 $OUT/r06_tests4a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/probes/autograd_floor_probe.py > $OUT/autograd_probe3.json 2> $OUT/autograd_probe3.err
rc=$?; echo "probe rc=$rc"; cat $OUT/autograd_probe3.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/probes/nb_train_probe.py > $OUT/nb_probe3.json 2> $OUT/nb_probe3.err
rc=$?; echo "probe rc=$rc"; cat $OUT/nb_probe3.json
