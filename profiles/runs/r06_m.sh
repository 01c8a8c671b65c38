set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_races.py tests/test_gpu_plan.py tests/test_gpu_schedule.py tests/test_gpu_deferred.py tests/test_gpu_benchshape.py tests/test_gpu_text.py > gpurun_out/r06_m_tests.log 2>&1 || exit 1
B="python bench.py --steps 20 --warmup 5 --modes inbatch --no-eval --no-cpu-baseline --no-f32-probe"
for i in 1 2 3; do
  timeout -k 10 200 $B > gpurun_out/r06_m_b_$i.json 2>/dev/null || exit 3
done
timeout -k 10 200 $B --gpu-only > gpurun_out/r06_m_go.json 2>/dev/null || exit 4
