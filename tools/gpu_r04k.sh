#!/bin/bash
# Round 4 session k: backward A/B across builds (build/ab_*.so), bit identity by sha.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
: > $OUT/r04p_ab.jsonl
for rep in 0 1; do
for so in build/ab_*.so; do
  n=$(basename $so .so)
  MPIV_LIB=$(pwd)/$so timeout -k 10 120 python -u tools/bwd_ab.py 0 > $OUT/r04p_$n.jsonl 2> $OUT/r04p_$n.err \
    || { echo "$n failed"; tail -3 $OUT/r04p_$n.err; exit 1; }
  sed "s/^{/{\"lib\": \"$n\", /" $OUT/r04p_$n.jsonl >> $OUT/r04p_ab.jsonl
done
done
cat $OUT/r04p_ab.jsonl
