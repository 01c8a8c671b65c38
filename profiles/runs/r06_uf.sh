set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_deferred.py tests/test_gpu_races.py tests/test_gpu_schedule.py tests/test_gpu_adam_exact.py > gpurun_out/r06_uf_tests.log 2>&1 || exit 1
B="python bench.py --steps 20 --warmup 5 --modes inbatch --no-eval --no-cpu-baseline --no-f32-probe --gpu-only"
timeout -k 10 200 $B > gpurun_out/r06_uf_a.json 2> gpurun_out/r06_uf_a.err || exit 3
timeout -k 10 200 $B > gpurun_out/r06_uf_b.json 2> gpurun_out/r06_uf_b.err || exit 3
DCUE_HIP_LIB=$GRAFT_REPO_ROOT/ktrace_tmp/libdcue_hip.so KT_STEPS=400 timeout -k 10 300 python profiles/tools/ktrace.py > gpurun_out/r06_ktu2.txt 2>&1 || exit 2
