# Round-6 final evidence, part C: the bench line again (it quotes the rocprof summary of this build) and the
# 2-rank gloo rehearsal.  Every GPU step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python3 -u bench.py > $OUT/r06d_final_bench_prof.json 2> $OUT/r06d_final_bench_prof.err
rc=$?; echo "bench rc=$rc"; tail -c 300 $OUT/r06d_final_bench_prof.err; [ $rc -eq 0 ] || exit $rc
MPIV_BENCH_BACKEND=gloo MPIV_BENCH_ONE_DEVICE=1 timeout -k 10 400 python3 -u bench.py --gpus 2 --steps 3 --warmup 1 \
    --cpu-seconds 0 > $OUT/r06d_final_bench2.json 2> $OUT/r06d_final_bench2.err
rc=$?; echo "bench --gpus 2 rc=$rc"; tail -c 300 $OUT/r06d_final_bench2.err
