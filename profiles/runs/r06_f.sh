set -o pipefail
cd $GRAFT_REPO_ROOT
B="python bench.py --steps 20 --warmup 5 --modes inbatch --no-eval --no-cpu-baseline --no-f32-probe"
for i in 1 2; do
  timeout -k 10 200 $B > gpurun_out/r06_f_base_$i.json 2>/dev/null || exit 2
  timeout -k 10 200 env DCUE_SLICE_SKIP=1 $B > gpurun_out/r06_f_skip_$i.json 2>/dev/null || exit 2
  timeout -k 10 200 $B --flush-every 24 > gpurun_out/r06_f_fe24_$i.json 2>/dev/null || exit 2
  timeout -k 10 200 $B --flush-every 48 > gpurun_out/r06_f_fe48_$i.json 2>/dev/null || exit 2
done
