#!/bin/bash
# A/B/C... of runtime environment switches in one GPU session: alternating bench runs, one per
# variant per round (variant "-" = no extra environment). STEPS / WARMUP (default: the driver's
# 20 / 5) and BENCH_EXTRA pass through to bench.py.
#   gpurun -- 'bash profiles/ab_env.sh <tag> <rounds> <modes> "<env 1>" "<env 2>" ...'
set -uo pipefail
TAG=$1; ROUNDS=$2; MODES=$3; shift 3
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/ab_$TAG
mkdir -p "$OUT"
for r in $(seq 1 $ROUNDS); do
  i=0
  for E in "$@"; do
    i=$((i + 1))
    EV=$([ "$E" = "-" ] && echo "DCUE_AB_VARIANT=$i" || echo "$E")
    env $EV timeout -k 10 200 python3 $ROOT/bench.py --no-cpu-baseline --no-eval --no-f32-probe --steps ${STEPS:-20} --warmup ${WARMUP:-5} \
      --modes $MODES ${BENCH_EXTRA:-} > "$OUT/v${i}_$r.log" 2>&1 || exit 1
    python3 - "$OUT/v${i}_$r.log" "$EV" <<'PY' >> "$OUT/summary.txt"
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
cat = d.get("catalogue", {})
cold = d.get("inbatch_cold", {})
print(sys.argv[2], "warm %.4f (host %.4f, gpu-only %s) cold %s cat %s (host %s)" % (
    d["ms_per_step"], d.get("host_enqueue_ms_per_step", 0), d.get("gpu_only_ms_per_step"), cold.get("ms_per_step"),
    cat.get("ms_per_step"), cat.get("host_enqueue_ms_per_step")))
PY
  done
done
cat "$OUT/summary.txt"
