#!/bin/bash
# focused debug session: one test file, verbose, short per-test timeout (thread method prints stacks)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
T=${T:-tests/test_backward_gpu.py}
K=${K:-}
timeout -k 10 240 python -u -m pytest $T ${K:+-k "$K"} -m gpu -x -v --timeout 60 --timeout-method thread > $OUT/dbg.log 2>&1
rc=$?; echo "rc=$rc"; tail -60 $OUT/dbg.log
