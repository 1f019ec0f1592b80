#!/bin/bash
# round 6: out-of-range south loads (OOB) routed for <= 2-view same-row launches -- render / config-5
# GPU tests (default and A/B), then the bench legs' routes against the previous build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_render_gpu.py tests/test_config5_gpu.py tests/test_u8_gpu.py > gpurun_out/oob_tests.log 2>&1 || { tail -30 gpurun_out/oob_tests.log; exit 1; }
tail -n 1 gpurun_out/oob_tests.log
MPIV_AB_TESTS=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_render_gpu.py tests/test_config5_gpu.py > gpurun_out/oob_tests_ab.log 2>&1 || { tail -30 gpurun_out/oob_tests_ab.log; exit 1; }
tail -n 1 gpurun_out/oob_tests_ab.log
bash tools/gpu_ab_libs.sh mpi_vision_amd/libmpiv_prev.so
