#!/bin/bash
# One GPU-box session: parity tests, a bench line, a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash/timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
TESTS=${TESTS:-tests}
timeout -k 10 ${PYTEST_LIMIT:-420} python -u -m pytest $TESTS -m gpu -x -v --timeout 180 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 "$OUT/pytest_gpu.log"
if [ $rc -gt 1 ]; then exit $rc; fi
[ "${SKIP_BENCH:-0}" = 1 ] && exit 0
timeout -k 10 ${BENCH_LIMIT:-300} python -u bench.py ${BENCH_ARGS:---steps 5 --warmup 1 --cpu-seconds 8} > "$OUT/bench.log" 2>&1
rc=$?
echo "bench rc=$rc"; tail -3 "$OUT/bench.log"
if [ $rc -ne 0 ]; then exit $rc; fi
[ "${SKIP_PROF:-0}" = 1 ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 ${PROF_LIMIT:-300} rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run \
    -- python -u "$ROOT/bench.py" --steps 3 --warmup 1 --cpu-seconds 0 --no-training > "$OUT/prof.log" 2>&1
rc=$?
echo "rocprof rc=$rc"; tail -3 "$OUT/prof.log"
find "$OUT/prof" -name "*stats*" | head
exit $rc
