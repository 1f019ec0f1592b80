#!/bin/bash
# Round 4 session t: backward tests (non-checkpoint path through the strip forward) + A/B of
# non-temporal d MPI stores (build/ab_*.so) + bench training leg timings.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_backward_gpu.py > $OUT/r04t_tests.log 2>&1
rc=$?; tail -3 $OUT/r04t_tests.log; [ $rc = 0 ] || exit $rc
: > $OUT/r04t_ab.jsonl
for rep in 0 1; do for so in build/ab_*.so; do
  n=$(basename $so .so)
  MPIV_LIB=$(pwd)/$so timeout -k 10 120 python -u tools/bwd_ab.py 0 > $OUT/r04t_$n.jsonl 2> $OUT/r04t_$n.err || { echo "$n failed"; tail -3 $OUT/r04t_$n.err; exit 1; }
  sed "s/^{/{\"lib\": \"$n\", /" $OUT/r04t_$n.jsonl >> $OUT/r04t_ab.jsonl
done; done
cat $OUT/r04t_ab.jsonl
