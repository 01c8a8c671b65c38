"""One timed step's kernel timeline from a rocprofv3 --kernel-trace run of bench.py --profile-phase.

  python3 profiles/timeline.py <dir with *kernel_trace.csv> [anchor kernel substring]

Steps are cut at each dispatch of the anchor kernel (default k_input_stats: the first kernel of
the item tower on the caller's stream). Prints the median step period, then the kernels of the
step whose period is the median: start offset, duration and queue, and the critical stream's busy
fraction (union of its kernels' intervals over the period).
"""
import csv
import glob
import os
import statistics
import sys

MARK = "spin_kernel"


def main():
    d = sys.argv[1]
    anchor = sys.argv[2] if len(sys.argv) > 2 else "k_input_stats"
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", "?"))
                 for r in rows), key=lambda x: x[0])
    marks = [k for k in ks if MARK in k[2]]
    if len(marks) >= 2:
        lo, hi = marks[0][1], marks[-1][0]
        ks = [k for k in ks if k[0] >= lo and k[1] <= hi and MARK not in k[2]]
    starts = [k[0] for k in ks if anchor in k[2]]
    periods = [(starts[i + 1] - starts[i], i) for i in range(len(starts) - 1)]
    if not periods:
        print("no anchor dispatches")
        return
    med = statistics.median(p for p, _ in periods)
    print("steps %d  period median %.1f us  min %.1f  max %.1f" % (
        len(periods), med / 1e3, min(periods)[0] / 1e3, max(periods)[0] / 1e3))
    per, i = min(periods, key=lambda x: abs(x[0] - med))
    t0, t1 = starts[i], starts[i + 1]
    step = [k for k in ks if t0 <= k[0] < t1]
    q_anchor = next(k[3] for k in step if anchor in k[2])
    busy = {}
    for s, e, n, q in step:
        busy.setdefault(q, []).append((s, min(e, t1)))
    print("%8s %8s %6s  %s" % ("start", "dur", "queue", "kernel"))
    for s, e, n, q in step:
        short = n.split("(")[0].replace("void ", "").replace("dcue::", "")
        print("%8.1f %8.1f %6s%s %s" % ((s - t0) / 1e3, (e - s) / 1e3, q, "*" if q == q_anchor else " ", short[:90]))
    for q, iv in busy.items():
        iv.sort()
        tot, cs, ce = 0, None, None
        for s, e in iv:
            if cs is None or s > ce:
                if cs is not None:
                    tot += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        tot += ce - cs
        print("queue %s busy %.1f us of %.1f (%.0f%%)" % (q, tot / 1e3, per / 1e3, 100.0 * tot / per))
    # the anchor queue over every step: median gap before each of its kernels (by position in the
    # step) -- what cross-stream waits, event records and dispatch cost the critical chain
    gaps = {}
    for j in range(len(starts) - 1):
        a, b = starts[j], starts[j + 1]
        chain = [k for k in ks if a <= k[0] < b and k[3] == q_anchor]
        for n, (k0, k1) in enumerate(zip(chain, chain[1:])):
            name = k1[2].split("(")[0].replace("void ", "").replace("dcue::", "")[:60]
            gaps.setdefault((n, name), []).append((k1[0] - k0[1]) / 1e3)
    print("anchor-queue gaps (median over %d steps, us):" % (len(starts) - 1))
    tot = 0.0
    for (n, name), v in sorted(gaps.items()):
        g = statistics.median(v)
        tot += g
        print("  %6.1f  before %s" % (g, name))
    print("  %6.1f  total" % tot)


if __name__ == "__main__":
    main()
