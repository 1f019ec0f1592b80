#!/bin/bash
# Round 4 session j: strip kernel tests + A/B timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_render_gpu.py tests/test_backward_gpu.py tests/test_u8_gpu.py -k "chunk or native or training_forward or u8" > $OUT/r04j_tests.log 2>&1
rc=$?; tail -3 $OUT/r04j_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab.py --only strips,u8f > $OUT/r04j_ab.jsonl 2> $OUT/r04j_ab.err
rc=$?; cat $OUT/r04j_ab.jsonl; exit $rc
