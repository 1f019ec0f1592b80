#!/bin/bash
# Sweep parity tests + config-3 kernel A/B timings (run on the GPU box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_sweep_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/sweep_tests.log 2>&1
rc=$?
tail -5 gpurun_out/sweep_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_configs.py --only ${ONLY:-c3} > gpurun_out/ab.jsonl 2> gpurun_out/ab.err
rc=$?
python - <<'PY'
import json
for l in open("gpurun_out/ab.jsonl"):
    d = json.loads(l)
    print(f"{d['config'][:90]:90s} {d['ms_median']:9.4f} {d.get('roofline_frac', 0):.3f}")
PY
exit $rc
