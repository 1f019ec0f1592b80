#!/bin/bash
# tools/ab.py experiments (ONLY=...) across build/ab_*.so, each under rocprofv3 --kernel-trace --stats
# (per-kernel averages in gpurun_out/abprof_<build>/), then EXTRA experiments on the in-tree libraries.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
for so in build/ab_*.so; do
  n=$(basename $so .so)
  (cd /tmp && TMPDIR=/tmp MPIV_LIB=$ROOT/$so timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $OUT/abprof_$n -o run -- python3 -u $ROOT/tools/ab.py --only ${ONLY:-bwdg} > $OUT/$n.jsonl 2> $OUT/$n.err) \
    || { echo "$n failed"; tail -3 $OUT/$n.err; exit 1; }
  echo "== $n"; cat $OUT/$n.jsonl
done
if [ -n "${EXTRA:-}" ]; then
  timeout -k 10 300 python3 -u tools/ab.py --only $EXTRA > $OUT/extra.jsonl 2> $OUT/extra.err \
    || { echo "extra failed"; tail -3 $OUT/extra.err; exit 1; }
  echo "== extra"; cat $OUT/extra.jsonl
fi
