set -o pipefail
cd $GRAFT_REPO_ROOT
B="python bench.py --steps 20 --warmup 5 --modes inbatch --no-eval --no-cpu-baseline --no-f32-probe --host-trace"
for i in 1 2 3; do
timeout -k 10 200 $B --spin-sync 0 > gpurun_out/r06_ss_0_$i.json 2> gpurun_out/r06_ss_0_$i.err || exit 3
timeout -k 10 200 $B --spin-sync 1 > gpurun_out/r06_ss_1_$i.json 2> gpurun_out/r06_ss_1_$i.err || exit 3
done
