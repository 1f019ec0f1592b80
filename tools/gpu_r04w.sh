#!/bin/bash
# Round 4 session w: in-place strip block shape A/B across builds (build/ab_*.so); each build's
# strip frames / checkpoints compared bit for bit with its 64 x 1 row kernel (tools/ab.py strip).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
: > $OUT/r04w_ab.jsonl
for rep in 0 1; do for so in build/ab_*.so; do
  n=$(basename $so .so)
  MPIV_LIB=$(pwd)/$so timeout -k 10 200 python -u tools/ab.py --only strip > $OUT/r04w_$n.jsonl 2> $OUT/r04w_$n.err || { echo "$n failed"; tail -3 $OUT/r04w_$n.err; exit 1; }
  sed "s/^{/{\"lib\": \"$n\", /" $OUT/r04w_$n.jsonl >> $OUT/r04w_ab.jsonl
done; done
grep -v backward $OUT/r04w_ab.jsonl
