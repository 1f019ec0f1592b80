#!/bin/bash
# Kernel A/B across builds of libmpiv.so (build/ab_*.so): config timings per build.
#   ONLY=c3 bash tools/gpu_ab_lib.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for so in build/ab_*.so; do
  n=$(basename $so .so)
  MPIV_LIB=$(pwd)/$so timeout -k 10 200 python -u tools/bench_configs.py --only ${ONLY:-c3} > $OUT/$n.jsonl 2> $OUT/$n.err \
    || { echo "$n failed"; tail -3 $OUT/$n.err; exit 1; }
  echo "== $n"; python -c "
import json,sys
for l in open('$OUT/$n.jsonl'):
    d=json.loads(l); print(f\"{d['config'][:70]:70s} {d['ms_median']:9.4f} {d['roofline_frac']:.3f}\")"
done
# headline kernel per build: bench.py lines for VIEWS (default 125 8 1)
[ "${BENCH:-0}" = 1 ] || exit 0
for so in build/ab_*.so; do
  n=$(basename $so .so)
  for v in ${VIEWS:-125 8 1}; do
    MPIV_LIB=$(pwd)/$so timeout -k 10 180 python -u bench.py --views $v --steps 5 --warmup 1 --cpu-seconds 0 > $OUT/${n}_b$v.log 2>&1 \
      || { echo "$n bench failed"; tail -3 $OUT/${n}_b$v.log; exit 1; }
    python -c "
import json
l=[x for x in open('$OUT/${n}_b$v.log') if x.startswith('{')][-1]; d=json.loads(l)
print('$n', $v, d['value'], d['roofline']['kernel_ms_per_launch'], d['roofline']['frac'])"
  done
done
