set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_text.py tests/test_gpu_text_dp.py > gpurun_out/r06_c_tests.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --modes text --no-eval --no-cpu-baseline --no-f32-probe > gpurun_out/r06_c_text.json 2>/dev/null || exit 2
bash profiles/gpu_only_timeline.sh r06_c || exit 3
