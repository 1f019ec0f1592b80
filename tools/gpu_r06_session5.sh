set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 200 python tools/probes/autograd_floor_probe.py > $OUT/autograd_probe4.json 2> $OUT/autograd_probe4.err
rc=$?; echo "probe rc=$rc"; cat $OUT/autograd_probe4.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/r06_tests5.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/r06_tests5.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --legs nb,netout --steps 3 --warmup 1 > $OUT/r06_bench5.json 2> $OUT/r06_bench5.err
rc=$?; echo "bench rc=$rc"; python3 -c "import json;d=json.loads(open('$OUT/r06_bench5.json').read().splitlines()[-1]);print(d['notebook']['train_step_ms'], d['net_output_render']['training']['fused']['step_ms'], d['net_output_render']['training']['two_step']['step_ms'])"
