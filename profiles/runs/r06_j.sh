set -o pipefail
cd $GRAFT_REPO_ROOT
B="python bench.py --steps 20 --warmup 5 --modes inbatch --no-eval --no-cpu-baseline --no-f32-probe"
for i in 1 2; do
  timeout -k 10 200 env DCUE_FROZEN_ROWS=0 $B > gpurun_out/r06_j_off_$i.json 2>/dev/null || exit 2
  timeout -k 10 200 $B > gpurun_out/r06_j_on_$i.json 2>/dev/null || exit 3
done
