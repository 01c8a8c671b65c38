"""Host-side pieces of bench.py that need no GPU."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_fail_flag_failures():
    import bench
    assert bench.fail_flag_failures(0) == []
    f = bench.fail_flag_failures(1)
    assert len(f) == 1 and "bit 0" in f[0]
    f = bench.fail_flag_failures(2)
    assert len(f) == 1 and "bit 1" in f[0]
    f = bench.fail_flag_failures(5)
    assert len(f) == 2 and "0x4" in f[1]
