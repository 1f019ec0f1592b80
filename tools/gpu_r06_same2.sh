#!/bin/bash
# round 6: the whole GPU suite on the same-row reuse build, then its A/B against render_same=-1
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/same2_tests.log 2>&1 || { tail -40 gpurun_out/same2_tests.log; exit 1; }
tail -3 gpurun_out/same2_tests.log
timeout -k 10 240 python -u tools/ab.py --only same --iters 15 > gpurun_out/same2_ab.jsonl 2>&1 || { tail -20 gpurun_out/same2_ab.jsonl; exit 1; }
echo done
