#!/bin/bash
# bench.py lines under several environment settings (kernel A/B at the headline config):
#   ENVS="MPIV_RENDER_PAIR=0 MPIV_RENDER_PAIR=1" VIEWS="125 1" bash tools/gpu_env_bench.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for e in ${ENVS}; do
  for v in ${VIEWS:-125 8 1}; do
    env $e timeout -k 10 180 python -u bench.py --views $v --steps 5 --warmup 1 --cpu-seconds 0 > $OUT/eb_${e}_$v.log 2>&1 \
      || { echo "$e $v failed"; tail -3 $OUT/eb_${e}_$v.log; exit 1; }
    python -c "
import json
l=[x for x in open('$OUT/eb_${e}_$v.log') if x.startswith('{')][-1]; d=json.loads(l)
print('$e', $v, d['value'], d['roofline']['kernel_ms_per_launch'], d['roofline']['frac'])"
  done
done
