#!/bin/bash
# round 6: dead tiles in the fused net-output render -- its GPU tests, then the netout A/B (pose 5 / 20)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_assemble_gpu.py tests/test_render_gpu.py tests/test_backward_gpu.py > gpurun_out/dead2_tests.log 2>&1 || { tail -40 gpurun_out/dead2_tests.log; exit 1; }
tail -2 gpurun_out/dead2_tests.log
timeout -k 10 300 python -u tools/bench_configs.py --only net --iters 30 > gpurun_out/dead2_net.jsonl 2>&1 || { tail -20 gpurun_out/dead2_net.jsonl; exit 1; }
cat gpurun_out/dead2_net.jsonl
echo done
