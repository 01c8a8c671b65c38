#!/bin/bash
# One bench phase under rocprofv3 --kernel-trace, summarised per kernel inside the phase's marker
# window (profiles/phase_kernels.py). Run on the GPU box from the repo root:
#   gpurun -- 'bash profiles/phase_prof.sh <tag> <phase> [steps] [extra bench args...]'
set -euo pipefail
TAG=$1; PH=$2; STEPS=${3:-100}; shift 3 || shift $#
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/stats_$PH" -o run \
  -- python3 $ROOT/bench.py --no-cpu-baseline --no-eval --steps $STEPS --warmup 10 --profile-phase $PH "$@" \
  > "$OUT/stats_$PH.log" 2>&1
python3 "$ROOT/profiles/phase_kernels.py" "$OUT/stats_$PH" 40 > "$OUT/${TAG}_${PH}_kernels.txt"
cat "$OUT/${TAG}_${PH}_kernels.txt"
