set -o pipefail
cd $GRAFT_REPO_ROOT
B="python bench.py --steps 20 --warmup 5 --modes inbatch --no-eval --no-cpu-baseline --no-f32-probe --gpu-only"
timeout -k 10 200 $B > gpurun_out/r06_x_a.json 2> gpurun_out/r06_x_a.err || exit 3
DCUE_HIP_LIB=$GRAFT_REPO_ROOT/ktrace_tmp/libdcue_hip.so timeout -k 10 200 python profiles/tools/ktrace.py > gpurun_out/r06_kt5.txt 2>&1 || exit 2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06_x_tests.log 2>&1 || exit 4
