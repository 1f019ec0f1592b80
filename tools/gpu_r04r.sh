#!/bin/bash
# Round 4 session r: full GPU suite + bench on the plane-group build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $OUT/r04r_tests.log 2>&1
rc=$?; tail -4 $OUT/r04r_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $OUT/bench_r04r.json 2> $OUT/bench_r04r.err
rc=$?; tail -2 $OUT/bench_r04r.err; exit $rc
