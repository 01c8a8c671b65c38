#!/bin/bash
# One catalogue step's kernel timeline (rocprofv3 --kernel-trace of the catalogue phase; host-paced,
# the step is GPU-bound there).   gpurun -- 'bash profiles/cat_timeline.sh <tag>'
set -uo pipefail
TAG=${1:-rNN}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/cattl_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d "$OUT/trace" -o run -- python3 $ROOT/bench.py \
  --no-cpu-baseline --no-eval --steps ${STEPS:-12} --warmup 4 --modes catalogue --profile-phase catalogue \
  > "$OUT/prof.log" 2>&1 || exit 1
python3 $ROOT/profiles/timeline.py "$OUT/trace" "k_conv_rows<0, 0," > "$OUT/timeline.txt" 2>&1
rm -rf "$OUT/trace"
