#!/bin/bash
# Row-tile sweep of the conv row-GEMMs (DCUE_ROWS_TW forces tiles per workgroup; 0 = the chooser):
#   gpurun -- 'bash profiles/tw_sweep.sh <phase> <tw...>'
# per TW value: the plain bench phase's ms/step, then the phase's kernels under rocprofv3.
set -uo pipefail
PH=${1:-catalogue}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/tw_$PH
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
MODES=$([ "$PH" = catalogue ] && echo catalogue || echo inbatch)
for TW in "$@"; do
  export DCUE_ROWS_TW=$TW
  timeout -k 10 200 python3 $ROOT/bench.py --no-cpu-baseline --no-eval --steps 60 --warmup 10 --modes $MODES \
    > "$OUT/plain_$TW.log" 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d "$OUT/trace_$TW" -o run -- python3 $ROOT/bench.py \
    --no-cpu-baseline --no-eval --steps 30 --warmup 5 --modes $MODES --profile-phase $PH > "$OUT/prof_$TW.log" 2>&1 || exit 1
  python3 $ROOT/profiles/phase_kernels.py "$OUT/trace_$TW" 14 > "$OUT/kernels_$TW.txt"
  python3 $ROOT/profiles/timeline.py "$OUT/trace_$TW" "k_conv_rows<0, 0," > "$OUT/timeline_$TW.txt" 2>&1
  python3 - "$OUT/plain_$TW.log" "$PH" <<'PY' >> "$OUT/kernels_$TW.txt"
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
ph = d["catalogue"] if sys.argv[2] == "catalogue" else (d["inbatch_cold"] if sys.argv[2] == "inbatch_cold" else d)
print("ms_per_step", ph["ms_per_step"])
PY
  rm -rf "$OUT/trace_$TW"
done
