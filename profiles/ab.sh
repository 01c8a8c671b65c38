#!/bin/bash
# A/B of an environment switch in one GPU session: alternating runs of the in-batch bench phases.
#   gpurun -- 'bash profiles/ab.sh <tag> "<env A>" "<env B>" [rounds] [modes]'
set -uo pipefail
TAG=$1; A=$2; B=$3; ROUNDS=${4:-2}; MODES=${5:-inbatch}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/ab_$TAG
mkdir -p "$OUT"
for r in $(seq 1 $ROUNDS); do
  for V in A B; do
    E=$([ $V = A ] && echo "$A" || echo "$B")
    env $E timeout -k 10 200 python3 $ROOT/bench.py --no-cpu-baseline --no-eval --steps 200 --warmup 20 \
      --modes $MODES > "$OUT/${V}_$r.log" 2>&1 || exit 1
    python3 - "$OUT/${V}_$r.log" "$V" "$E" <<'PY' >> "$OUT/summary.txt"
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
ks = {k["kernel"].split(" ")[0]: round(k["avg_ms"] * 1e3, 2) for k in d["kernels"]}
cat = d.get("catalogue", {}).get("ms_per_step")
print(sys.argv[2], sys.argv[3], "warm %.4f cold %.4f cat %s" % (d["ms_per_step"], d["inbatch_cold"]["ms_per_step"], cat), ks)
PY
  done
done
