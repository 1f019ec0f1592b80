#!/bin/bash
# Round 4 session m: u8 ring-depth tests + A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_u8_gpu.py > $OUT/r04m_tests.log 2>&1
rc=$?; tail -3 $OUT/r04m_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab.py --only u8f > $OUT/r04m_ab.jsonl 2> $OUT/r04m_ab.err
rc=$?; cat $OUT/r04m_ab.jsonl; exit $rc
