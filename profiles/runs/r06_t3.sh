set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_text.py tests/test_gpu_text_dp.py > gpurun_out/r06_t3_tests.log 2>&1 || exit 1
B="python bench.py --steps 20 --warmup 5 --modes text --no-eval --no-cpu-baseline --no-f32-probe"
timeout -k 10 200 $B > gpurun_out/r06_t3_a.json 2> gpurun_out/r06_t3_a.err || exit 3
timeout -k 10 200 $B > gpurun_out/r06_t3_b.json 2> gpurun_out/r06_t3_b.err || exit 3
