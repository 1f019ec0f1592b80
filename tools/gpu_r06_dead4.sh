#!/bin/bash
# round 6: dead tiles in the backward chain -- backward / assembly GPU tests (default and A/B), then timings
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_backward_gpu.py tests/test_assemble_gpu.py > gpurun_out/dead4_tests.log 2>&1 || { tail -40 gpurun_out/dead4_tests.log; exit 1; }
tail -n 1 gpurun_out/dead4_tests.log
MPIV_AB_TESTS=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_backward_gpu.py > gpurun_out/dead4_tests_ab.log 2>&1 || { tail -40 gpurun_out/dead4_tests_ab.log; exit 1; }
tail -n 1 gpurun_out/dead4_tests_ab.log
timeout -k 10 300 python -u tools/bench_configs.py --only bwd --iters 20 > gpurun_out/dead4_bwd.jsonl 2>&1 || { tail -20 gpurun_out/dead4_bwd.jsonl; exit 1; }
cut -c1-160 gpurun_out/dead4_bwd.jsonl
echo done
