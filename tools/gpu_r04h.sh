#!/bin/bash
# backward A/B (default vs MPIV_LIB variants), then GPU tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r04h}
for rep in 1 2; do
for v in default gpf2; do
  if [ $v = default ]; then lib=""; else lib="build/ab_$v.so"; fi
  echo "== bwd $v $rep"
  MPIV_LIB=$lib timeout -k 5 60 python3 -u tools/bwd_ab.py 0 > $OUT/bwdab_${v}_${TAG}_$rep.jsonl 2>&1
  rc=$?; tail -1 $OUT/bwdab_${v}_${TAG}_$rep.jsonl; [ $rc -eq 0 ] || exit $rc
done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/gpu_tests_$TAG.log
echo "session done"
