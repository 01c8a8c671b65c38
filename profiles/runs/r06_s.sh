set -o pipefail
cd $GRAFT_REPO_ROOT
DCUE_HIP_LIB=$GRAFT_REPO_ROOT/ktrace_tmp/libdcue_hip.so timeout -k 10 200 python profiles/tools/ktrace.py > gpurun_out/r06_kt1.txt 2>&1 || exit 2
B="python bench.py --steps 20 --warmup 5 --modes inbatch --no-eval --no-cpu-baseline --no-f32-probe --gpu-only"
timeout -k 10 200 $B > gpurun_out/r06_s_a.json 2> gpurun_out/r06_s_a.err || exit 3
timeout -k 10 200 $B > gpurun_out/r06_s_b.json 2> gpurun_out/r06_s_b.err || exit 4
