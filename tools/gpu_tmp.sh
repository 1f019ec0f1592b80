set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_assemble_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_asm.log 2>&1; rc=$?; tail -5 gpurun_out/t_asm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_configs.py --only net --iters 20 > gpurun_out/cfg_net.jsonl 2>&1; rc=$?; cut -c1-160 gpurun_out/cfg_net.jsonl; exit $rc
