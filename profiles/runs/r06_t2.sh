set -o pipefail
cd $GRAFT_REPO_ROOT
B="python bench.py --steps 20 --warmup 5 --modes text --no-eval --no-cpu-baseline --no-f32-probe --gpu-only"
for S in 128 32 16; do
timeout -k 10 200 env DCUE_TEXT_WGRAD_ITEMS=$S $B > gpurun_out/r06_t2_$S.json 2> gpurun_out/r06_t2_$S.err || exit 3
done
