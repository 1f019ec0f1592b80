set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?; tail -2 gpurun_out/t_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/sv_poses.py --poses 0,500 > gpurun_out/sv_poses.jsonl 2>&1; rc=$?; grep pose gpurun_out/sv_poses.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_configs.py --only c4 --iters 10 > gpurun_out/cfg_rows.jsonl 2>&1; rc=$?; grep -E "packed" gpurun_out/cfg_rows.jsonl | grep -E "rows|direct|default" | cut -c1-130; exit $rc
