set -o pipefail
cd $GRAFT_REPO_ROOT
B="python bench.py --steps 20 --warmup 5 --modes inbatch --no-eval --no-cpu-baseline --no-f32-probe --host-trace"
timeout -k 10 200 env DCUE_HOST_PROFILE=2 $B > gpurun_out/r06_hp5.json 2> gpurun_out/r06_hp5.err || exit 3
