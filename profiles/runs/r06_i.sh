set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_deferred.py > gpurun_out/r06_i_tests.log 2>&1 || exit 1
B="python bench.py --steps 20 --warmup 5 --modes inbatch --no-eval --no-cpu-baseline --no-f32-probe"
for i in 1 2; do
  timeout -k 10 200 env DCUE_FROZEN_ROWS=0 $B > gpurun_out/r06_i_off_$i.json 2>/dev/null || exit 2
  timeout -k 10 200 $B > gpurun_out/r06_i_on_$i.json 2>/dev/null || exit 3
  timeout -k 10 200 env DCUE_SLICE_WGS=512 $B > gpurun_out/r06_i_w512_$i.json 2>/dev/null || exit 3
  timeout -k 10 200 env DCUE_SLICE_WGS=256 $B > gpurun_out/r06_i_w256_$i.json 2>/dev/null || exit 3
done
