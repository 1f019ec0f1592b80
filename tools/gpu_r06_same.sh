#!/bin/bash
# round 6: same-row tap reuse A/B (3-wave and forced 4-wave builds) + the render/config-5/u8/assembly GPU tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_render_gpu.py tests/test_config5_gpu.py tests/test_assemble_gpu.py tests/test_u8_gpu.py > gpurun_out/same_tests.log 2>&1 || { tail -30 gpurun_out/same_tests.log; exit 1; }
tail -3 gpurun_out/same_tests.log
timeout -k 10 240 python -u tools/ab.py --only same --iters 15 > gpurun_out/same_ab.jsonl 2>&1 || { tail -20 gpurun_out/same_ab.jsonl; exit 1; }
MPIV_LIB=$PWD/mpi_vision_amd/libmpiv_w4.so timeout -k 10 240 python -u tools/ab.py --only same --iters 15 > gpurun_out/same_ab_w4.jsonl 2>&1 || { tail -20 gpurun_out/same_ab_w4.jsonl; exit 1; }
echo done
