set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rs > $OUT/r06_tests1.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/r06_tests1.log; [ $rc -eq 0 ] || exit $rc
MPIV_BENCH_FAULT=c5_hang MPIV_BENCH_LEG_DEADLINE=40 MPIV_BENCH_BACKEND=gloo MPIV_BENCH_ONE_DEVICE=1 timeout -k 10 300 python3 -u bench.py --gpus 2 --steps 3 --warmup 1 --legs c4,c5 > $OUT/r06_fault_hang.json 2> $OUT/r06_fault_hang.err
rc=$?; echo "fault hang rc=$rc"; tail -c 300 $OUT/r06_fault_hang.err; [ $rc -eq 0 ] || exit $rc
MPIV_BENCH_FAULT=c5_raise MPIV_BENCH_LEG_DEADLINE=40 MPIV_BENCH_BACKEND=gloo MPIV_BENCH_ONE_DEVICE=1 timeout -k 10 300 python3 -u bench.py --gpus 2 --steps 3 --warmup 1 --legs c4,c5 > $OUT/r06_fault_raise.json 2> $OUT/r06_fault_raise.err
rc=$?; echo "fault raise rc=$rc"; tail -c 300 $OUT/r06_fault_raise.err
