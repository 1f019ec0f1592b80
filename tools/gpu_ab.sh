#!/bin/bash
# Render-kernel A/B on the GPU box, headline config (config 4): KERNELS x VIEWS bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for k in ${KERNELS:-packed packed_mv}; do
  for v in ${VIEWS:-125 8 1}; do
    timeout -k 10 180 python -u bench.py --kernel $k --views $v --steps 5 --warmup 1 --cpu-seconds 0 \
      > $OUT/ab_${k}_$v.log 2>&1 || { echo "ab $k $v failed"; tail -5 $OUT/ab_${k}_$v.log; exit 1; }
    python - $OUT/ab_${k}_$v.log <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{')][-1]; d=json.loads(l)
print(d['config']['kernel'], d['config']['views_per_gpu_per_step'], d['value'], d['roofline']['kernel_ms_per_launch'], d['roofline']['frac'])
PY
  done
done
