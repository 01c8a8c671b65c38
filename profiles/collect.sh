#!/bin/bash
# Round profile collection, run on the GPU box from the repo root:
#   gpurun -- 'bash profiles/collect.sh r01_c'
# 1. rocprofv3 --kernel-trace --stats of the default bench command (csv kernel stats)
# 2. two --pmc passes (FETCH_SIZE, then WRITE_SIZE: they do not fit one TCC pass) restricted to the
#    roofline kernel, summarised (gfx950 FETCH_SIZE x2 correction, KB -> B) by summarize_pmc.py into
#    profiles/pmc_conv1_wgrad.json, which bench.py reports as roofline.traffic.
set -euo pipefail
TAG=${1:-rNN}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
BENCH="$ROOT/bench.py --no-cpu-baseline --steps 200 --warmup 20"
# the same command without the profiler: its live roofline timing is the one bench.py reports
(cd "$ROOT" && timeout -k 10 240 python3 $BENCH > "$OUT/plain.log" 2>&1)
grep '^{' "$OUT/plain.log" | tail -n 1 > "$OUT/${TAG}_bench_plain.json"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/stats" -o run -- python3 $BENCH \
  > "$OUT/stats.log" 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c --kernel-include-regex 'k_conv1_wgrad' -f csv \
    -d "$OUT/pmc_$c" -o run -- python3 $ROOT/bench.py --no-cpu-baseline --no-eval --steps 40 --warmup 5 \
    > "$OUT/pmc_$c.log" 2>&1
done
# catalogue mode (M = B(1+N) distinct items per step): kernel stats only
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/stats_cat" -o run -- python3 $ROOT/bench.py \
  --mode catalogue --no-cpu-baseline --no-eval --steps 40 --warmup 5 > "$OUT/stats_cat.log" 2>&1
cp "$OUT/stats_cat/run_kernel_stats.csv" "$OUT/${TAG}_cat_kernel_stats.csv"
grep '^{' "$OUT/stats_cat.log" | tail -n 1 > "$OUT/${TAG}_cat_bench.json"
python3 "$ROOT/profiles/summarize_pmc.py" "$OUT" "$TAG"
