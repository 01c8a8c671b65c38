"""Summarise one collect.sh run into profile files (copied into profiles/ after review).

  python3 profiles/summarize_pmc.py <collect output dir> <tag>

bench.py --profile-phase <phase> brackets that phase's timed steps with two marker kernels
(torch's spin_kernel); only the dispatches between the marks count here.

Writes
  <tag>_<phase>_kernel_stats.csv  per kernel: calls, total/avg/min/max ns inside the phase window
                                  (rocprofv3's own --stats cover the whole process)
  <tag>_kernels_per_step.json     each kernel's time per timed step, per phase
  pmc_<kernel>_<mode>.json        per-launch HBM bytes of the kernels the bench line reports a
                                  roofline for (bench.py reads roofline.traffic from them)

HBM bytes follow MI355X_MICROARCH.md "HBM [CDNA4]": FETCH_SIZE / WRITE_SIZE are in KB; on gfx950
FETCH_SIZE reports half the bytes of a wide coalesced read, so it is doubled; WRITE_SIZE is exact.
"""
import csv
import glob
import json
import os
import sys

# conv-1 weight gradient: the tap-fused kernel (k_conv_wgrad16t, round 3) is the default, the one-tap
# k_conv_wgrad1k (round 6) an A/B under DCUE_W1K=1; layer 2's tap-fused weight gradient runs beside
# the dgrad chain on a side stream
KERNELS = {"conv1_wgrad": "k_conv1_wgrad", "conv1_wgrad16": "k_conv_wgrad16t<0,", "conv1_wgrad1k": "k_conv_wgrad1k<",
           "wgrad16t_layer2": "k_conv_wgrad16t<2,", "wgrad16_multi": "k_conv_wgrad16_multi", "emb_flush_rows": "k_emb_flush_rows",
           "conv1_fwd": "k_conv_rows<0, 0,", "text_fwd": "k_text_fwd", "user_fwd": "k_user_fwd",
           "text_wgrad": "k_text_wgrad"}
MARK = "spin_kernel"


def _rows(d, pattern):
    rows = []
    for f in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    return rows


def _window_by_dispatch(rows):
    """(first, last) dispatch ids strictly between the two marker kernels, or None."""
    ids = sorted({int(r["Dispatch_Id"]) for r in rows if MARK in r.get("Kernel_Name", "")})
    return (ids[0], ids[-1]) if len(ids) >= 2 else None


def phase_stats(d):
    rows = _rows(d, "*kernel_trace.csv")
    marks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if MARK in r["Kernel_Name"])
    if len(marks) < 2:
        return None
    lo, hi = marks[0][1], marks[-1][0]
    agg = {}
    for r in rows:
        if MARK in r["Kernel_Name"]:
            continue
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s < lo or e > hi:
            continue
        a = agg.setdefault(r["Kernel_Name"], [])
        a.append(e - s)
    return agg


def per_dispatch(d, counter, kernel):
    """mean over the kernel's dispatches inside the marker window of the counter's value (summed
    over its dimensions per dispatch)"""
    rows = _rows(d, "*counter_collection.csv")
    win = _window_by_dispatch(rows)
    by = {}
    for r in rows:
        if r.get("Counter_Name") != counter or kernel not in r.get("Kernel_Name", ""):
            continue
        did = int(r["Dispatch_Id"])
        if win and not (win[0] < did < win[1]):
            continue
        by[did] = by.get(did, 0.0) + float(r["Counter_Value"])
    if not by:
        return None, 0
    return sum(by.values()) / len(by), len(by)


def main():
    d, tag = sys.argv[1], sys.argv[2]
    out = {}
    for mode in ("inbatch", "catalogue", "text"):
        for short, kname in KERNELS.items():
            fetch_kb, n_f = per_dispatch(os.path.join(d, "pmc_%s_FETCH_SIZE" % mode), "FETCH_SIZE", kname)
            write_kb, n_w = per_dispatch(os.path.join(d, "pmc_%s_WRITE_SIZE" % mode), "WRITE_SIZE", kname)
            if fetch_kb is None or write_kb is None:
                continue
            rd, wr = 2.0 * fetch_kb * 1024.0, write_kb * 1024.0
            rec = {"kernel": kname, "mode": mode, "fetch_size_kb_raw": fetch_kb, "write_size_kb": write_kb,
                   "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
                   "hbm_bytes_per_launch": rd + wr, "dispatches": [n_f, n_w], "tag": tag,
                   "correction": "FETCH_SIZE x2 (gfx950 half-count on wide reads), KB x1024"}
            name = "pmc_%s_%s.json" % (short, mode)
            with open(os.path.join(d, name), "w") as fh:
                json.dump(rec, fh, indent=1)
            out[name] = rec["hbm_bytes_per_launch"]
    steps = None
    plain = os.path.join(d, "%s_bench_plain.json" % tag)
    if os.path.exists(plain):
        steps = json.load(open(plain)).get("steps")
    per_step = {}
    for ph in ("inbatch", "catalogue", "inbatch_cold", "text"):
        agg = phase_stats(os.path.join(d, "stats_%s" % ph))
        if not agg or not steps:
            continue
        tot = sum(sum(v) for v in agg.values())
        rows = sorted(agg.items(), key=lambda kv: -sum(kv[1]))
        with open(os.path.join(d, "%s_%s_kernel_stats.csv" % (tag, ph)), "w", newline="") as fh:
            w = csv.writer(fh)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
            for k, v in rows:
                w.writerow([k, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / tot, min(v), max(v)])
        per_step[ph] = {"steps": steps, "kernel_ms_per_step": tot / steps / 1e6,
                        "kernels": [{"name": k.split("(")[0][:120], "calls_per_step": len(v) / steps,
                                     "avg_us": sum(v) / len(v) / 1e3, "us_per_step": sum(v) / steps / 1e3}
                                    for k, v in rows]}
    with open(os.path.join(d, "%s_kernels_per_step.json" % tag), "w") as fh:
        json.dump(per_step, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
