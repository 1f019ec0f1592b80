set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_backward_gpu.py -x -q --timeout 200 --timeout-method thread -k "graph" > $OUT/r06_tests7a.log 2>&1
rc=$?; echo "graph test rc=$rc"; tail -3 $OUT/r06_tests7a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --legs nb --steps 3 --warmup 1 > $OUT/r06_bench7.json 2> $OUT/r06_bench7.err
rc=$?; echo "bench rc=$rc"; python3 -c "import json;d=json.loads(open('$OUT/r06_bench7.json').read().splitlines()[-1]);nb=d['notebook'];print({k:v for k,v in nb.items() if 'train' in k})"
