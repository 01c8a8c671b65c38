#!/bin/bash
# HBM traffic (FETCH_SIZE, WRITE_SIZE: two --pmc passes) of the roofline kernels in one bench phase,
# summarised per launch by summarize_pmc.py.   gpurun -- 'bash profiles/pmc_traffic.sh <tag> <phase>'
# <phase>: inbatch | inbatch_cold | catalogue | text
set -uo pipefail
TAG=${1:-rNN}; PH=${2:-catalogue}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
case "$PH" in catalogue) MODES=catalogue;; text) MODES=text;; *) MODES=inbatch;; esac
KRE='k_conv1_wgrad|k_conv_wgrad16|k_conv_wgrad1k|k_emb_flush_rows|k_conv_rows|k_user_fwd|k_text_wgrad|k_text_fwd|spin_kernel'
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $C --kernel-include-regex "$KRE" \
    -f csv -d "$OUT/pmc_${PH}_$C" -o run -- python3 $ROOT/bench.py --no-cpu-baseline --no-eval --no-f32-probe \
    --steps 40 --warmup 5 --modes $MODES --profile-phase $PH \
    > "$OUT/pmc_${PH}_$C.log" 2>&1 || exit 1
done
python3 "$ROOT/profiles/summarize_pmc.py" "$OUT" "$TAG"
