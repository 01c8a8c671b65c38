#!/bin/bash
# Text-forward shape A/B: per variant (env settings, "-" = none) one kernel-trace pass and one
# FETCH_SIZE pass over bench.py's text phase, summarised as k_text_fwd* average duration and HBM
# read bytes per launch (FETCH_SIZE x2, the gfx950 correction).
#   gpurun -- 'bash profiles/text_fwd_ab.sh <tag> "<env 1>" "<env 2>" ...'
set -uo pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/textab_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="python3 $ROOT/bench.py --no-cpu-baseline --no-eval --no-f32-probe --steps 20 --warmup 5 --modes text --profile-phase text"
i=0
for E in "$@"; do
  i=$((i + 1))
  EV=$([ "$E" = "-" ] && echo "DCUE_AB_VARIANT=$i" || echo "$E")
  export $EV
  timeout -s KILL 180 rocprofv3 --kernel-trace --kernel-include-regex 'k_text_fwd|spin_kernel' -f csv \
    -d "$OUT/v${i}_trace" -o run -- $BENCH > "$OUT/v${i}_trace.log" 2>&1 || exit 1
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'k_text_fwd|spin_kernel' -f csv \
    -d "$OUT/v${i}_pmc" -o run -- $BENCH > "$OUT/v${i}_pmc.log" 2>&1 || exit 1
  unset ${EV%%=*}
  python3 - "$OUT" "$i" "$EV" >> "$OUT/summary.txt" <<'PY'
import csv, glob, os, sys
d, i, ev = sys.argv[1], sys.argv[2], sys.argv[3]
def rows(kind, pat):
    out = []
    for f in glob.glob(os.path.join(d, "v%s_%s" % (i, kind), "**", pat), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out
tr = rows("trace", "*kernel_trace.csv")
marks = sorted(int(r["Start_Timestamp"]) for r in tr if "spin_kernel" in r["Kernel_Name"])
lo, hi = (marks[0], marks[-1]) if len(marks) >= 2 else (0, 1 << 62)
durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tr
        if "k_text_fwd" in r["Kernel_Name"] and lo < int(r["Start_Timestamp"]) < hi]
pm = rows("pmc", "*counter_collection.csv")
ids = sorted(int(r["Dispatch_Id"]) for r in pm if "spin_kernel" in r["Kernel_Name"])
plo, phi = (ids[0], ids[-1]) if len(ids) >= 2 else (0, 1 << 62)
fs = [float(r["Counter_Value"]) for r in pm if "k_text_fwd" in r["Kernel_Name"] and plo < int(r["Dispatch_Id"]) < phi]
name = next((r["Kernel_Name"][:60] for r in tr if "k_text_fwd" in r["Kernel_Name"]), "?")
print("%-28s %s n=%d avg %.2f us min %.2f us  hbm_read %.2f MB/launch (n=%d)" % (
    ev, name, len(durs), sum(durs) / max(1, len(durs)) / 1e3, min(durs or [0]) / 1e3,
    2 * 1024 * sum(fs) / max(1, len(fs)) / 1e6, len(fs)))
PY
  rm -rf "$OUT/v${i}_trace" "$OUT/v${i}_pmc"
done
cat "$OUT/summary.txt"
