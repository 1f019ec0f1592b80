#!/bin/bash
# Headline bench (config 4, --no-extras) across abbuild/ab_*.so, alternating builds twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out; mkdir -p $OUT
for rep in 1 2; do
  for so in abbuild/ab_*.so; do
    n=$(basename $so .so)
    MPIV_LIB=$(pwd)/$so timeout -k 10 240 python -u bench.py --views ${VIEWS:-125} --steps ${STEPS:-10} --warmup 2 \
        --cpu-seconds 0 --no-extras > $OUT/${n}_$rep.log 2>&1 || { echo "$n failed"; tail -5 $OUT/${n}_$rep.log; exit 1; }
    python -c "
import json
l=[x for x in open('$OUT/${n}_$rep.log') if x.startswith('{')][-1]; d=json.loads(l)
print(json.dumps({'lib':'$n','rep':$rep,'value':d['value'],'ms_per_step':d['ms_per_step'],'kernel_ms':d['roofline']['kernel_ms_per_launch'],'frac':d['roofline']['frac'],'check':d.get('timed_frame_check')}))"
  done
done
