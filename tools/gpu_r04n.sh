#!/bin/bash
# Round 4 session n: u8 A/B across builds (build/ab_*.so); bit identity across ring depths inside each build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
: > $OUT/r04n_ab.jsonl
for rep in 0 1; do for so in build/ab_*.so; do
  n=$(basename $so .so)
  MPIV_LIB=$(pwd)/$so timeout -k 10 200 python -u tools/ab.py --only u8f > $OUT/r04n_$n.jsonl 2> $OUT/r04n_$n.err || { echo "$n failed"; tail -3 $OUT/r04n_$n.err; exit 1; }
  sed "s/^{/{\"lib\": \"$n\", /" $OUT/r04n_$n.jsonl >> $OUT/r04n_ab.jsonl
done; done
grep '"1 views\|u8 render, 1 views' $OUT/r04n_ab.jsonl
