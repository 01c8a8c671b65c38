set -o pipefail
cd $GRAFT_REPO_ROOT
B="python bench.py --steps 20 --warmup 5 --modes inbatch --no-eval --no-cpu-baseline --no-f32-probe --gpu-only"
for i in 1 2; do
timeout -k 10 200 $B > gpurun_out/r06_fo_d$i.json 2> gpurun_out/r06_fo_d$i.err || exit 3
timeout -k 10 200 env DCUE_FORK_ONCE=1 $B > gpurun_out/r06_fo_o$i.json 2> gpurun_out/r06_fo_o$i.err || exit 3
done
