set -o pipefail
cd $GRAFT_REPO_ROOT
B="python bench.py --steps 20 --warmup 5 --modes inbatch --no-eval --no-cpu-baseline --no-f32-probe"
for i in 1 2 3; do
  timeout -k 10 200 $B > gpurun_out/r06_k_plain_$i.json 2>/dev/null || exit 2
  timeout -k 10 200 $B --gpu-only > gpurun_out/r06_k_gpuonly_$i.json 2>/dev/null || exit 3
done
timeout -k 10 200 env DCUE_HOST_PROFILE=1 $B > gpurun_out/r06_k_hostprof.json 2> gpurun_out/r06_k_hostprof.err || exit 4
