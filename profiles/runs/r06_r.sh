set -o pipefail
cd $GRAFT_REPO_ROOT
B="python bench.py --steps 20 --warmup 5 --modes inbatch --no-eval --no-cpu-baseline --no-f32-probe --gpu-only"
for S in 4 8 12 16; do
timeout -k 10 200 env DCUE_W16T_MIN_STAGES=$S $B > gpurun_out/r06_r_$S.json 2> gpurun_out/r06_r_$S.err || exit 3
done
