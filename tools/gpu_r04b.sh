#!/bin/bash
# round-4 session: GPU tests, backward gather A/B, bench line.  Each step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r04b}
timeout -k 10 200 python3 -u tools/bwd_ab.py 0 3 > $OUT/bwd_ab_$TAG.jsonl 2> $OUT/bwd_ab_$TAG.err
rc=$?; echo "bwd_ab rc=$rc"; cat $OUT/bwd_ab_$TAG.jsonl; tail -3 $OUT/bwd_ab_$TAG.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py ${BENCH_ARGS:-} > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; tail -c 400 $OUT/bench_$TAG.err; [ $rc -eq 0 ] || exit $rc
echo "session done"
