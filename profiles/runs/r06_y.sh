set -o pipefail
cd $GRAFT_REPO_ROOT
B="python bench.py --steps 20 --warmup 5 --modes inbatch --no-eval --no-cpu-baseline --no-f32-probe --gpu-only"
for S in 2 4 16; do
timeout -k 10 200 env DCUE_W1K_MIN_STAGES=$S $B > gpurun_out/r06_y_$S.json 2> gpurun_out/r06_y_$S.err || exit 3
done
timeout -k 10 200 env DCUE_W1K=0 $B > gpurun_out/r06_y_off.json 2> gpurun_out/r06_y_off.err || exit 3
