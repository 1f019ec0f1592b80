#!/bin/bash
# Config timings under several environment settings (A/B of env-selected kernels):
#   ENVS="MPIV_RENDER_SV=0 MPIV_RENDER_SV=1" ONLY=c4,c5 bash tools/gpu_env_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for e in ${ENVS}; do
  env $e timeout -k 10 300 python -u tools/bench_configs.py --only ${ONLY:-c4} > $OUT/env_$e.jsonl 2> $OUT/env_$e.err \
    || { echo "$e failed"; tail -3 $OUT/env_$e.err; exit 1; }
  echo "== $e"; python -c "
import json
for l in open('$OUT/env_$e.jsonl'):
    d=json.loads(l); print(f\"{d['config'][:72]:72s} {d['ms_median']:9.4f} {d['roofline_frac']:.3f}\")"
done
