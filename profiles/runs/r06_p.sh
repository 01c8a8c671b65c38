set -o pipefail
cd $GRAFT_REPO_ROOT
B="python bench.py --steps 20 --warmup 5 --modes inbatch --no-eval --no-cpu-baseline --no-f32-probe --host-trace"
timeout -k 10 200 $B > gpurun_out/r06_p_a.json 2> gpurun_out/r06_p_a.err || exit 3
timeout -k 10 200 $B > gpurun_out/r06_p_b.json 2> gpurun_out/r06_p_b.err || exit 4
timeout -k 10 200 env DCUE_HOST_PROFILE=2 $B > gpurun_out/r06_p_hp.json 2> gpurun_out/r06_p_hp.err || exit 5
