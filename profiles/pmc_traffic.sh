#!/bin/bash
# HBM traffic (FETCH_SIZE, WRITE_SIZE: two --pmc passes) of the roofline kernels in one bench phase,
# summarised per launch by summarize_pmc.py.   gpurun -- 'bash profiles/pmc_traffic.sh <tag> <phase>'
set -uo pipefail
TAG=${1:-rNN}; PH=${2:-catalogue}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $C --kernel-include-regex 'k_conv1_wgrad|k_conv_wgrad16|k_emb_flush_rows|k_conv_rows|spin_kernel' \
    -f csv -d "$OUT/pmc_${PH}_$C" -o run -- python3 $ROOT/bench.py --no-cpu-baseline --no-eval --steps 40 \
    --warmup 5 --modes $([ "$PH" = catalogue ] && echo catalogue || echo inbatch) --profile-phase $PH \
    > "$OUT/pmc_${PH}_$C.log" 2>&1 || exit 1
done
python3 "$ROOT/profiles/summarize_pmc.py" "$OUT" "$TAG"
