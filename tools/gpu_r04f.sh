#!/bin/bash
# ticket-schedule diagnosis (uniform control flow), backward A/B, GPU tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r04f}
ok=1
for a in "1 9 4" "4 9 4" "1024 9 1024" "20000 9 1024"; do
  echo "== tickets $a"; timeout -k 5 25 python3 -u tools/ticket_selftest.py $a; rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { ok=0; break; }
done
if [ $ok = 1 ]; then
  for c in "ga tk_one" "ga tk_fixed4" "ga tk" "gbig tk" "ga tk_many"; do
    echo "== $c"; timeout -k 5 25 python3 -u tools/fb_dbg.py $c; rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || break
  done
fi
for v in default; do
  echo "== bwd $v"
  timeout -k 5 60 python3 -u tools/bwd_ab.py 0 > $OUT/bwdab_${v}_$TAG.jsonl 2>&1
  rc=$?; tail -1 $OUT/bwdab_${v}_$TAG.jsonl; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/gpu_tests_$TAG.log
echo "session done"
