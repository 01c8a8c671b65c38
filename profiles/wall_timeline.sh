#!/bin/bash
# The in-batch step's schedule in the normal (host-paced) mode: rocprofv3 --kernel-trace over the
# steady-state phase's timed steps, cut at each conv-1 forward (profiles/timeline.py). Compare with
# gpu_only_timeline.sh, where the host enqueues everything before the GPU starts.
#   gpurun -- 'bash profiles/wall_timeline.sh <tag>'
set -uo pipefail
TAG=${1:-rNN}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/wall_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d "$OUT/trace" -o run -- python3 $ROOT/bench.py \
  --no-cpu-baseline --no-eval --no-f32-probe --steps ${STEPS:-40} --warmup 10 --modes inbatch --profile-phase inbatch \
  > "$OUT/prof.log" 2>&1 || exit 1
python3 $ROOT/profiles/timeline.py "$OUT/trace" "k_conv_rows<0, 0," > "$OUT/timeline.txt" 2>&1
python3 $ROOT/profiles/phase_kernels.py "$OUT/trace" 40 > "$OUT/kernels.txt"
rm -rf "$OUT/trace"
