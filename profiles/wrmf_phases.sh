#!/bin/bash
# WRMF ALS iteration time per variant (env settings, "-" = none) from bench.py's dcbr phase.
#   gpurun -- 'bash profiles/wrmf_phases.sh <tag> "<env 1>" ...'
set -uo pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/wrmf_$TAG
mkdir -p "$OUT"
i=0
for E in "$@"; do
  i=$((i + 1))
  EV=$([ "$E" = "-" ] && echo "DCUE_AB_VARIANT=$i" || echo "$E")
  env $EV timeout -k 10 300 python3 $ROOT/bench.py --no-cpu-baseline --no-eval --no-f32-probe --steps 2 --warmup 1 \
    --modes dcbr > "$OUT/v$i.log" 2>&1; [ $? -ge 124 ] && exit 1
  python3 - "$OUT/v$i.log" "$EV" >> "$OUT/summary.txt" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
w = d.get("dcbr", {})
print("%-28s wrmf %.2f ms/iteration (first %.1f)" % (sys.argv[2], w.get("wrmf_ms_per_iteration", -1),
                                                     w.get("wrmf_first_iteration_ms_incl_csr_build", -1)))
PY
done
cat "$OUT/summary.txt"
