#!/bin/bash
# PMC of the WRMF solve (bench.py --modes dcbr, BASELINE config 5): one rocprofv3 --pmc pass per
# counter group (SQ stall/instruction counters; FETCH_SIZE; WRITE_SIZE), mean per k_wrmf_solve
# dispatch, written to gpurun_out/pmcw_<tag>/ as <tag>_pmc_wrmf_solve.txt and pmc_wrmf_solve.json
# (copied into profiles/ after review; HBM bytes per launch with
# MI355X_MICROARCH.md's corrections: FETCH_SIZE doubled, KB x 1024).
#   gpurun -- 'bash profiles/pmc_wrmf.sh <tag>'
set -uo pipefail
TAG=${1:-rNN}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmcw_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" FETCH_SIZE WRITE_SIZE; do
  i=$((i + 1))
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-include-regex 'k_wrmf' -f csv -d "$OUT/p$i" -o run \
    -- python3 $ROOT/bench.py --no-cpu-baseline --no-eval --no-f32-probe --steps 5 --warmup 2 --modes dcbr \
    > "$OUT/p$i.log" 2>&1 || exit 1
done
python3 - "$OUT" "$TAG" "$OUT" <<'PY'
import collections, csv, glob, json, os, sys
d, tag, prof = sys.argv[1], sys.argv[2], sys.argv[3]
agg = collections.defaultdict(float)
n = collections.defaultdict(set)
for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_wrmf_solve" not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        n[r["Counter_Name"]].add(r["Dispatch_Id"])
mean = {c: v / max(1, len(n[c])) for c, v in agg.items()}
with open(os.path.join(prof, "%s_pmc_wrmf_solve.txt" % tag), "w") as fh:
    fh.write("k_wrmf_solve, bench.py --modes dcbr (100k users x 200k tracks, d=128): mean per dispatch "
             "(users and items half-steps)\n")
    for c in sorted(mean):
        fh.write("%s %.1f\n" % (c, mean[c]))
hbm = None
if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
    hbm = 2 * mean["FETCH_SIZE"] * 1024 + mean["WRITE_SIZE"] * 1024
json.dump({"kernel": "k_wrmf_solve", "hbm_bytes": hbm, "fetch_kb": mean.get("FETCH_SIZE"),
           "write_kb": mean.get("WRITE_SIZE"), "correction": "FETCH_SIZE x2 (gfx950), KB x1024", "tag": tag},
          open(os.path.join(prof, "pmc_wrmf_solve.json"), "w"), indent=1)
print(json.dumps(mean, indent=1))
PY
