#!/bin/bash
# Round 4 session s: backward GPU tests after the workspace layout fix.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_backward_gpu.py tests/test_render_gpu.py > $OUT/r04s_tests.log 2>&1
rc=$?; tail -3 $OUT/r04s_tests.log; exit $rc
