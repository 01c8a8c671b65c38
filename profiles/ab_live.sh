#!/bin/bash
# Plain-bench A/B (no profiler) of the driver's in-batch command per variant (env settings, "-" =
# none): step times and the bench's live HIP-event kernel timings.
#   gpurun -- 'bash profiles/ab_live.sh <tag> <rounds> "<env 1>" "<env 2>" ...'
set -uo pipefail
TAG=$1; ROUNDS=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/live_$TAG
mkdir -p "$OUT"
for r in $(seq 1 $ROUNDS); do
  i=0
  for E in "$@"; do
    i=$((i + 1))
    EV=$([ "$E" = "-" ] && echo "DCUE_AB_VARIANT=$i" || echo "$E")
    env $EV timeout -k 10 200 python3 $ROOT/bench.py --no-cpu-baseline --no-eval --no-f32-probe --steps 20 --warmup 5 \
      --modes ${MODES:-inbatch} > "$OUT/v${i}_$r.log" 2>&1 || exit 1
    python3 - "$OUT/v${i}_$r.log" "$EV" <<'PY' >> "$OUT/summary.txt"
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
ph = d.get("text", d)  # (MODES=text: the text phase's block)
ks = " ".join("%s %.1f/%.1f" % (k["kernel"].split()[0], k["avg_ms"] * 1e3, k.get("median_ms", 0) * 1e3)
              for k in ph.get("kernels", []))
print("%-26s step %.4f host %.4f cold %.4f | avg/median us: %s" % (sys.argv[2], ph["ms_per_step"],
      ph.get("host_enqueue_ms_per_step", 0), d.get("inbatch_cold", {}).get("ms_per_step", -1), ks))
PY
  done
done
cat "$OUT/summary.txt"
