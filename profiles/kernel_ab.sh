#!/bin/bash
# One kernel's A/B across environment variants: per variant (env settings, "-" = none) a kernel-trace
# pass and FETCH_SIZE / WRITE_SIZE passes over one bench phase, summarised as the kernel's average
# duration and HBM bytes per launch inside the phase window (FETCH_SIZE x2, the gfx950 correction).
#   gpurun -- 'KERNEL=k_conv_wgrad16t PHASE=inbatch bash profiles/kernel_ab.sh <tag> "<env 1>" ...'
set -uo pipefail
TAG=$1; shift
KERNEL=${KERNEL:-k_text_fwd}; PHASE=${PHASE:-text}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/kab_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
MODES=$([ "$PHASE" = catalogue ] && echo catalogue || ([ "$PHASE" = text ] && echo text || echo inbatch))
BENCH="python3 $ROOT/bench.py --no-cpu-baseline --no-eval --no-f32-probe --steps 20 --warmup 5 --modes $MODES --profile-phase $PHASE"
i=0
for E in "$@"; do
  i=$((i + 1))
  EV=$([ "$E" = "-" ] && echo "DCUE_AB_VARIANT=$i" || echo "$E")
  for kv in $EV; do export "$kv"; done
  timeout -s KILL 180 rocprofv3 --kernel-trace --kernel-include-regex "$KERNEL|spin_kernel" -f csv \
    -d "$OUT/v${i}_trace" -o run -- $BENCH > "$OUT/v${i}_trace.log" 2>&1 || exit 1
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $C --kernel-include-regex "$KERNEL|spin_kernel" -f csv \
      -d "$OUT/v${i}_$C" -o run -- $BENCH > "$OUT/v${i}_$C.log" 2>&1 || exit 1
  done
  for kv in $EV; do unset "${kv%%=*}"; done
  python3 - "$OUT" "$i" "$EV" "$KERNEL" >> "$OUT/summary.txt" <<'PY'
import csv, glob, os, re, sys
d, i, ev, kern = sys.argv[1:5]
def rows(kind, pat):
    out = []
    for f in glob.glob(os.path.join(d, "v%s_%s" % (i, kind), "**", pat), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out
tr = rows("trace", "*kernel_trace.csv")
marks = sorted(int(r["Start_Timestamp"]) for r in tr if "spin_kernel" in r["Kernel_Name"])
lo, hi = (marks[0], marks[-1]) if len(marks) >= 2 else (0, 1 << 62)
sel = [r for r in tr if re.search(kern, r["Kernel_Name"]) and lo < int(r["Start_Timestamp"]) < hi]
durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in sel]
def pmc(c):
    pm = rows(c, "*counter_collection.csv")
    ids = sorted(int(r["Dispatch_Id"]) for r in pm if "spin_kernel" in r["Kernel_Name"])
    plo, phi = (ids[0], ids[-1]) if len(ids) >= 2 else (0, 1 << 62)
    v = [float(r["Counter_Value"]) for r in pm if re.search(kern, r["Kernel_Name"]) and plo < int(r["Dispatch_Id"]) < phi]
    return sum(v) / max(1, len(v)) * 1024
name = sel[0]["Kernel_Name"][:70] if sel else "?"
print("%-34s %s n=%d avg %.2f us min %.2f us  read %.2f MB write %.2f MB /launch" % (
    ev, name, len(durs), sum(durs) / max(1, len(durs)) / 1e3, min(durs or [0]) / 1e3,
    2 * pmc("FETCH_SIZE") / 1e6, pmc("WRITE_SIZE") / 1e6))
PY
  rm -rf "$OUT/v${i}_trace" "$OUT/v${i}_FETCH_SIZE" "$OUT/v${i}_WRITE_SIZE"
done
cat "$OUT/summary.txt"
