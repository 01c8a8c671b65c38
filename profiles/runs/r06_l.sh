set -o pipefail
cd $GRAFT_REPO_ROOT
B="python bench.py --steps 20 --warmup 5 --modes inbatch --no-eval --no-cpu-baseline --no-f32-probe"
for i in 1 2 3; do
  timeout -k 10 200 env DCUE_SIDE_THREAD=0 $B > gpurun_out/r06_l_st0_$i.json 2>/dev/null || exit 2
  timeout -k 10 200 $B > gpurun_out/r06_l_st1_$i.json 2>/dev/null || exit 3
done
timeout -k 10 200 $B --steps 100 > gpurun_out/r06_l_s100.json 2>/dev/null || exit 4
