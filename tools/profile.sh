#!/bin/bash
# rocprofv3 evidence for every bench.py leg (run on the GPU box):
#   1. kernel-trace --stats of bench.py (all legs but the CPU baseline)
#   2-6. separate --pmc passes (FETCH_SIZE | WRITE_SIZE | TCC_HIT,TCC_MISS | VALU | TA busy)
# then, locally in the same tree: python tools/parse_prof.py gpurun_out/prof <tag>
# (groups the dispatches by kernel and grid size -> profiles/prof_summary.json).
# Each pass has its own time limit; any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof
# the trace pass runs the driver's own bench command (--steps 20 --warmup 5), so every timed leg
# has as many dispatches in the summary as in the driver's line; the counter passes only need the
# per-dispatch shapes and stay short
TRACE_ARGS=${PROF_TRACE_ARGS:---steps 20 --warmup 5 --cpu-seconds 0}
ARGS=${PROF_ARGS:---steps 3 --warmup 1 --cpu-seconds 0}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
    -- python3 -u "$ROOT/bench.py" $TRACE_ARGS > "$OUT/trace.log" 2>&1 || { echo "trace pass failed"; tail -5 "$OUT/trace.log"; exit 1; }
echo "trace pass ok"
for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE" \
            "TA_BUSY_avr GRBM_GUI_ACTIVE"; do
    name=$(echo "$pass" | tr ' ' '_')
    [ "$pass" = "SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE" ] && name=VALU
    [ "$pass" = "TA_BUSY_avr GRBM_GUI_ACTIVE" ] && name=TA
    timeout -s KILL 300 rocprofv3 --pmc $pass --output-format csv -d "$OUT/$name" -o run \
        -- python3 -u "$ROOT/bench.py" $ARGS > "$OUT/$name.log" 2>&1 || { echo "pmc pass $pass failed"; tail -5 "$OUT/$name.log"; exit 1; }
    echo "pmc pass $name ok"
done
echo "profile passes done; summarise locally: python tools/parse_prof.py gpurun_out/prof <tag>"
