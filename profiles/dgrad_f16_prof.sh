set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for V in 0 1; do
  DCUE_DGRAD_F16=$V timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d /tmp/dg$V -o run -- python3 $ROOT/bench.py --no-cpu-baseline --no-eval --steps 50 --warmup 10 --modes catalogue --profile-phase catalogue > $ROOT/gpurun_out/dgprof_$V.log 2>&1 || exit 1
  f=$(find /tmp/dg$V -name '*kernel_stats.csv' | head -n 1)
  grep -E 'k_conv_rows<1' "$f" | cut -c1-160 > $ROOT/gpurun_out/dgprof_$V.txt
done
cat $ROOT/gpurun_out/dgprof_0.txt $ROOT/gpurun_out/dgprof_1.txt
