set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_u8_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_u8.log 2>&1; rc=$?; tail -15 gpurun_out/t_u8.log; exit $rc
