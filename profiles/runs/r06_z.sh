set -o pipefail
cd $GRAFT_REPO_ROOT
B="python bench.py --steps 20 --warmup 5 --modes inbatch --no-eval --no-cpu-baseline --no-f32-probe --gpu-only"
timeout -k 10 200 $B > gpurun_out/r06_z_a.json 2> gpurun_out/r06_z_a.err || exit 3
DCUE_HIP_LIB=$GRAFT_REPO_ROOT/ktrace_tmp/libdcue_hip.so timeout -k 10 200 python profiles/tools/ktrace.py > gpurun_out/r06_kt6.txt 2>&1 || exit 2
timeout -k 10 200 $B > gpurun_out/r06_z_b.json 2> gpurun_out/r06_z_b.err || exit 3
timeout -k 10 200 env DCUE_W1K=1 $B > gpurun_out/r06_z_c.json 2> gpurun_out/r06_z_c.err || exit 3
