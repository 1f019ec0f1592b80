#!/bin/bash
# round 6: dead-tile (border-only) skipping -- render GPU tests, then the stretched-config A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_render_gpu.py tests/test_config5_gpu.py tests/test_u8_gpu.py tests/test_assemble_gpu.py tests/test_helpers_gpu.py > gpurun_out/dead_tests.log 2>&1 || { tail -40 gpurun_out/dead_tests.log; exit 1; }
tail -2 gpurun_out/dead_tests.log
MPIV_AB_TESTS=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_render_gpu.py -k "dead or same or sharing or ring or census" > gpurun_out/dead_tests_ab.log 2>&1 || { tail -40 gpurun_out/dead_tests_ab.log; exit 1; }
tail -2 gpurun_out/dead_tests_ab.log
timeout -k 10 240 python -u tools/ab.py --only same,same1 --iters 15 > gpurun_out/dead_ab.jsonl 2>&1 || { tail -20 gpurun_out/dead_ab.jsonl; exit 1; }
echo done
