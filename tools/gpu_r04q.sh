#!/bin/bash
# Round 4 session q: plane-grouped backward -- full GPU suite, then backward timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $OUT/r04q_tests.log 2>&1
rc=$?; tail -4 $OUT/r04q_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 120 python -u tools/bwd_ab.py 0 > $OUT/r04q_bwd.jsonl 2> $OUT/r04q_bwd.err
rc=$?; cat $OUT/r04q_bwd.jsonl; exit $rc
