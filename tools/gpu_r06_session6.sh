set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 200 python tools/probes/bwd_fold_probe.py > $OUT/bwd_fold3.json 2> $OUT/bwd_fold3.err
rc=$?; echo "fold probe rc=$rc"; cat $OUT/bwd_fold3.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/r06_tests6.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/r06_tests6.log; [ $rc -eq 0 ] || exit $rc
MPIV_AB_TESTS=1 timeout -k 10 500 python -u -m pytest tests/test_backward_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/r06_tests6b.log 2>&1
rc=$?; echo "backward A/B tests rc=$rc"; tail -2 $OUT/r06_tests6b.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --legs nb,netout,train --steps 3 --warmup 1 > $OUT/r06_bench6.json 2> $OUT/r06_bench6.err
rc=$?; echo "bench rc=$rc"; python3 -c "import json;d=json.loads(open('$OUT/r06_bench6.json').read().splitlines()[-1]);print(d['notebook']['train_step_ms'], d['net_output_render']['training']['fused']['step_ms'], d['net_output_render']['training']['two_step']['step_ms'], d['training_render_backward']['backward_ms'])"
