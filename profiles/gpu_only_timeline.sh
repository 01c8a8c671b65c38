#!/bin/bash
# The in-batch step's GPU-only schedule: bench.py --gpu-only parks the GPU behind a sleep kernel
# while the host enqueues every timed step, so the kernel trace shows the GPU's own dependencies
# (no host pacing).   gpurun -- 'bash profiles/gpu_only_timeline.sh <tag>'
set -uo pipefail
TAG=${1:-rNN}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/gpuonly_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d "$OUT/trace" -o run -- python3 $ROOT/bench.py \
  --no-cpu-baseline --no-eval --no-f32-probe --steps ${STEPS:-8} --warmup 3 --modes inbatch --gpu-only \
  --profile-phase ${PHASE:-inbatch} \
  > "$OUT/prof.log" 2>&1 || exit 1
python3 $ROOT/profiles/timeline.py "$OUT/trace" "k_conv_rows<0, 0," > "$OUT/timeline.txt" 2>&1
python3 $ROOT/profiles/phase_kernels.py "$OUT/trace" 40 > "$OUT/kernels.txt"
rm -rf "$OUT/trace"
