#!/bin/bash
# tools/ab.py experiments (ONLY=...) across build/ab_*.so, then (optional) the default build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for so in build/ab_*.so; do
  n=$(basename $so .so)
  MPIV_LIB=$(pwd)/$so timeout -k 10 200 python -u tools/ab.py --only ${ONLY:-bwd} > $OUT/$n.jsonl 2> $OUT/$n.err \
    || { echo "$n failed"; tail -3 $OUT/$n.err; exit 1; }
  echo "== $n"; cat $OUT/$n.jsonl
done
