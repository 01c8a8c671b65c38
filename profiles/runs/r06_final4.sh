set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_f4_bench_a.json 2> gpurun_out/r06_f4_bench_a.err || exit 6
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_f4_bench_b.json 2> gpurun_out/r06_f4_bench_b.err || exit 6
timeout -k 10 300 python -u -m pytest tests/test_gpu_dp.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06_f4_dp.log 2>&1 || exit 7
