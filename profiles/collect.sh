#!/bin/bash
# Round profile collection, run on the GPU box from the repo root:
#   gpurun -- 'bash profiles/collect.sh r02_a [steps] [warmup]'
# (round 5 on: the driver's shape, --steps 20 --warmup 5, unless given)
# 1. the bench command without the profiler (its live HIP-event kernel timings are what the bench
#    line reports; compared against 2.)
# 2. per timed phase (cold in-batch, steady-state in-batch, catalogue): rocprofv3 --kernel-trace
#    --stats; bench.py --profile-phase brackets that phase's timed steps with a marker kernel and
#    summarize_pmc.py keeps only the dispatches between the marks (<tag>_<phase>_kernel_stats.csv)
# 3. per mode, two --pmc passes (FETCH_SIZE, then WRITE_SIZE: they do not fit one TCC pass) over
#    the conv-1 forward, the conv weight gradients (conv 1; layers 2-5 + fc) and the rolling
#    user-table flush (+ the marker), summarised by
#    summarize_pmc.py (gfx950 FETCH_SIZE x2 correction, KB -> B) into pmc_<kernel>_<mode>.json
set -euo pipefail
TAG=${1:-rNN}
STEPS=${2:-20}
WARMUP=${3:-5}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
BENCH="$ROOT/bench.py --no-cpu-baseline --no-eval --no-f32-probe --steps $STEPS --warmup $WARMUP"
(cd "$ROOT" && timeout -k 10 300 python3 $BENCH > "$OUT/plain.log" 2>&1)
grep '^{' "$OUT/plain.log" | tail -n 1 > "$OUT/${TAG}_bench_plain.json"
for PH in inbatch catalogue inbatch_cold text; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/stats_$PH" -o run \
    -- python3 $BENCH --profile-phase $PH > "$OUT/stats_$PH.log" 2>&1
done
for PH in inbatch catalogue text; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $C --kernel-include-regex 'k_conv1_wgrad|k_conv_wgrad16|k_emb_flush_rows|k_conv_rows|k_text_fwd|spin_kernel' \
      -f csv -d "$OUT/pmc_${PH}_$C" -o run -- python3 $ROOT/bench.py --no-cpu-baseline --no-eval --steps 40 \
      --warmup 5 --profile-phase $PH > "$OUT/pmc_${PH}_$C.log" 2>&1
  done
done
python3 "$ROOT/profiles/summarize_pmc.py" "$OUT" "$TAG"
# keep the summaries and rocprofv3's own --stats tables; drop the raw traces (gpurun copies back at
# most 64 MiB of gpurun_out/)
for PH in inbatch catalogue inbatch_cold text; do
  f=$(find "$OUT/stats_$PH" -name '*kernel_stats.csv' | head -n 1)
  [ -n "$f" ] && cp "$f" "$OUT/${TAG}_${PH}_rocprof_kernel_stats.csv"
done
rm -rf "$OUT"/stats_inbatch "$OUT"/stats_catalogue "$OUT"/stats_inbatch_cold "$OUT"/stats_text "$OUT"/pmc_*_FETCH_SIZE "$OUT"/pmc_*_WRITE_SIZE
