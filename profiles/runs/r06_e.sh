set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 400 env DCUE_SLICE_STREAM=w1 DCUE_SLICE_WGS=256 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_deferred.py tests/test_gpu_races.py -k "deferred or delays_bit_identical" > gpurun_out/r06_e_tests.log 2>&1 || exit 1
B="python bench.py --steps 20 --warmup 5 --modes inbatch --no-eval --no-cpu-baseline --no-f32-probe"
for i in 1 2; do
  for v in "u:1073741824" "w1:1073741824" "w1:512" "w1:256" "w0:512"; do
    ss=${v%%:*}; w=${v##*:}
    timeout -k 10 200 env DCUE_SLICE_STREAM=$ss DCUE_SLICE_WGS=$w $B > gpurun_out/r06_e_${ss}_${w}_$i.json 2>/dev/null || exit 2
  done
done
