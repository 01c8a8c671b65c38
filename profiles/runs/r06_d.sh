set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_deferred.py tests/test_gpu_adam_exact.py > gpurun_out/r06_d_tests.log 2>&1 || exit 1
B="python bench.py --steps 20 --warmup 5 --modes inbatch --no-eval --no-cpu-baseline --no-f32-probe"
for i in 1 2; do
  for w in 100000 64 32 128; do
    timeout -k 10 200 env DCUE_SLICE_WGS=$w $B > gpurun_out/r06_d_w${w}_$i.json 2>/dev/null || exit 2
  done
done
