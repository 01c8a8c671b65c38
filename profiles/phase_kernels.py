"""Print the kernels of one profiled bench phase (rocprofv3 --kernel-trace output dir of a
bench.py --profile-phase run): calls, average and total microseconds inside the marker window.

  python3 profiles/phase_kernels.py <dir> [top]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from summarize_pmc import phase_stats  # noqa: E402


def main():
    d = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    agg = phase_stats(d)
    if not agg:
        print("no marker window in", d)
        return 1
    rows = sorted(((sum(v), len(v), k) for k, v in agg.items()), reverse=True)
    for tot, n, k in rows[:top]:
        print("%9.1f us total %6d calls %8.2f us avg  %s" % (tot / 1e3, n, tot / n / 1e3, k[:110]))
    return 0


if __name__ == "__main__":
    sys.exit(main())
