#!/bin/bash
# Stall breakdown of the step's kernels in one bench phase: one rocprofv3 --pmc pass (8 SQ counters
# + GRBM_GUI_ACTIVE) over bench.py --profile-phase <phase>, summarised per kernel (averages per
# dispatch inside the phase window).   gpurun -- 'bash profiles/pmc_kernels.sh <tag> <phase>'
set -uo pipefail
TAG=${1:-rNN}; PH=${2:-inbatch}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_${TAG}_$PH
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
MODES=$([ "$PH" = catalogue ] && echo catalogue || echo inbatch)
COUNTERS=${PMC_COUNTERS:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE}
timeout -s KILL 240 rocprofv3 --pmc $COUNTERS \
  -f csv -d "$OUT/raw" -o run -- python3 $ROOT/bench.py --no-cpu-baseline --no-eval --steps 20 --warmup 5 \
  --modes $MODES --profile-phase $PH > "$OUT/run.log" 2>&1 || exit 1
python3 - "$OUT" > "$OUT/summary.txt" <<'PY'
import csv, glob, os, sys, collections
d = sys.argv[1]
rows = []
for f in glob.glob(os.path.join(d, "raw", "**", "*counter_collection.csv"), recursive=True):
    rows += list(csv.DictReader(open(f)))
marks = sorted(int(r["Dispatch_Id"]) for r in rows if "spin_kernel" in r["Kernel_Name"])
lo, hi = (marks[0], marks[-1]) if len(marks) >= 2 else (0, 1 << 62)
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in rows:
    i = int(r["Dispatch_Id"])
    if not (lo < i < hi) or "spin_kernel" in r["Kernel_Name"]:
        continue
    k = r["Kernel_Name"].split("(")[0][:90]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(i)
order = sorted(agg, key=lambda k: -agg[k].get("GRBM_GUI_ACTIVE", 0))
for k in order:
    n = len(disp[k]); a = {c: v / n for c, v in agg[k].items()}
    wc = a.get("SQ_WAVE_CYCLES", 0) or 1
    print("%-90s n=%d gui=%.0f waveQ=%.0f wait=%.2f waitinst=%.2f active=%.2f mfma_busy=%.0f valu=%.0f lds=%.0f" % (
        k, n, a.get("GRBM_GUI_ACTIVE", 0), wc, a.get("SQ_WAIT_ANY", 0) / wc, a.get("SQ_WAIT_INST_ANY", 0) / wc,
        a.get("SQ_ACTIVE_INST_ANY", 0) / wc, a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0), a.get("SQ_INSTS_VALU", 0),
        a.get("SQ_INSTS_LDS", 0)),
          " ".join("%s=%.0f" % (c, v) for c, v in sorted(a.items()) if c not in (
              "GRBM_GUI_ACTIVE", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
              "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_VALU", "SQ_INSTS_LDS")))
PY
rm -rf "$OUT/raw"
