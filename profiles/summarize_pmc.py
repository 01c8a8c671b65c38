"""Summarise one collect.sh run into committed profile files.

  python3 profiles/summarize_pmc.py <collect output dir> <tag>

Writes (under gpurun_out/<dir>, copied into profiles/ by hand after review):
  <tag>_kernel_stats.csv     rocprofv3 --stats kernel summary of the bench command
  <tag>_bench.json           the bench JSON line printed under the profiler
  pmc_conv1_wgrad.json       per-launch HBM bytes of the roofline kernel (k_conv_wgrad layer 1)

HBM bytes follow MI355X_MICROARCH.md "HBM [CDNA4]": FETCH_SIZE / WRITE_SIZE are in KB; on gfx950
FETCH_SIZE reports half the bytes of a wide coalesced read, so it is doubled; WRITE_SIZE is exact.
"""
import csv
import glob
import json
import os
import sys


def _counter_rows(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    return rows


def per_dispatch(d, counter):
    """mean over dispatches of the counter's value (summed over its dimensions per dispatch)"""
    by = {}
    for r in _counter_rows(d):
        if r.get("Counter_Name") != counter:
            continue
        key = r.get("Dispatch_Id") or r.get("Correlation_Id")
        by[key] = by.get(key, 0.0) + float(r["Counter_Value"])
    if not by:
        return None, 0
    return sum(by.values()) / len(by), len(by)


def main():
    d, tag = sys.argv[1], sys.argv[2]
    out = {}
    fetch_kb, n_f = per_dispatch(os.path.join(d, "pmc_FETCH_SIZE"), "FETCH_SIZE")
    write_kb, n_w = per_dispatch(os.path.join(d, "pmc_WRITE_SIZE"), "WRITE_SIZE")
    if fetch_kb is not None and write_kb is not None:
        rd = 2.0 * fetch_kb * 1024.0
        wr = write_kb * 1024.0
        out = {"kernel": "k_conv1_wgrad (conv layer 1 weight gradient)",
               "fetch_size_kb_raw": fetch_kb, "write_size_kb": write_kb,
               "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
               "hbm_bytes_per_launch": rd + wr, "dispatches": [n_f, n_w],
               "correction": "FETCH_SIZE x2 (gfx950 half-count on wide reads), KB x1024"}
        with open(os.path.join(d, "pmc_conv1_wgrad.json"), "w") as fh:
            json.dump(out, fh, indent=1)
    stats = glob.glob(os.path.join(d, "stats", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        with open(stats[0]) as src, open(os.path.join(d, "%s_kernel_stats.csv" % tag), "w") as dst:
            dst.write(src.read())
    log = os.path.join(d, "stats.log")
    if os.path.exists(log):
        lines = [ln for ln in open(log) if ln.startswith("{")]
        if lines:
            with open(os.path.join(d, "%s_bench.json" % tag), "w") as fh:
                fh.write(lines[-1])
    print(json.dumps(out))


if __name__ == "__main__":
    main()
