#!/bin/bash
# One GPU-box session for a round: GPU parity tests, the default bench line, the
# one-device 2-rank rehearsal of bench.py --gpus 2 (gloo), and the rocprofv3 passes.
# Every GPU step has its own limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r04}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_$TAG.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 $OUT/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 python3 -u bench.py ${BENCH_ARGS:-} > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; tail -c 400 $OUT/bench_$TAG.err; [ $rc -eq 0 ] || exit $rc
if [ "${SKIP_MULTI:-0}" != 1 ]; then
  MPIV_BENCH_BACKEND=gloo MPIV_BENCH_ONE_DEVICE=1 timeout -k 10 400 python3 -u bench.py --gpus 2 --steps 3 --warmup 1 \
      --cpu-seconds 0 > $OUT/bench2_$TAG.json 2> $OUT/bench2_$TAG.err
  rc=$?; echo "bench --gpus 2 rc=$rc"; tail -c 400 $OUT/bench2_$TAG.err; [ $rc -eq 0 ] || exit $rc
fi
if [ "${SKIP_PROF:-0}" != 1 ]; then
  bash tools/profile.sh || exit 1
fi
echo "round script done"
