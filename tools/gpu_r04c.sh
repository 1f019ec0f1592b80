#!/bin/bash
# fallback debug cases, then the backward A/B across build variants (MPIV_LIB)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
bash tools/gpu_fbdbg.sh
for rep in 1; do
  for v in default nt gtr2 gtr2l4 gtr2nt; do
    if [ $v = default ]; then lib=""; else lib="build/ab_$v.so"; fi
    echo "== $v rep $rep"
    MPIV_LIB=$lib timeout -k 5 60 python3 -u tools/bwd_ab.py 0 > $OUT/bwdab_${v}_$rep.jsonl 2>&1
    rc=$?; tail -2 $OUT/bwdab_${v}_$rep.jsonl; [ $rc -eq 0 ] || exit $rc
  done
done
