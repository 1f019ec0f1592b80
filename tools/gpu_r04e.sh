#!/bin/bash
# round-4 session: GPU tests, bench line, backward A/B (MPIV_LIB variants), ticket diagnosis last
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r04e}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; tail -c 300 $OUT/bench_$TAG.err; [ $rc -eq 0 ] || exit $rc
for v in default gtr3c gtr4c gtr2s3; do
  if [ $v = default ]; then lib=""; else lib="build/ab_$v.so"; fi
  echo "== bwd $v"
  MPIV_LIB=$lib timeout -k 5 60 python3 -u tools/bwd_ab.py 0 > $OUT/bwdab_${v}_$TAG.jsonl 2>&1
  rc=$?; tail -1 $OUT/bwdab_${v}_$TAG.jsonl; [ $rc -eq 0 ] || break
done
for a in "1 9 4" "4 9 4" "1024 9 1024"; do
  echo "== tickets $a"; timeout -k 5 25 python3 -u tools/ticket_selftest.py $a; rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || break
done
echo "session done"
