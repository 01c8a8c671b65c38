"""The deferred user-table Adam replay's long-idle shortcut (csrc/adam_replay.h), checked on the host.

The deferred replay must stay bit-identical to the dense per-step sweep the reference's dense
embedding gradient implies (nn/dcue.py:143-147,209). replay_run switches an element to the m/v
recurrence once its parameter update can no longer move p; tests/native/adam_replay_check.cpp
compiles the same header for the CPU and compares replay_run with the plain step-by-step replay on
random and adversarial states (binade-edge p, thresholds, subnormals, zeros, huge magnitudes),
bit for bit, and checks the margin the shortcut leaves below half a float spacing of p.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path_factory.mktemp("arc") / "adam_replay_check")
    subprocess.check_call([gxx, "-O2", "-std=c++17", "-ffp-contract=off",
                           "-I", os.path.join(ROOT, "amplifai-deepcontentrecommenders_amd", "csrc"),
                           "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "native", "adam_replay_check.cpp"), "-o", exe])
    return exe


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_replay_shortcut_bit_exact(checker, seed):
    r = subprocess.run([checker, "60000", str(seed)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    fields = r.stdout.split()
    stats = dict(zip(fields[::2], fields[1::2]))
    assert int(stats["mismatches"]) == 0
    assert int(stats["shortcut-steps"]) > 0.1 * int(stats["element-steps"])  # the shortcut is exercised
    assert float(stats["worst-margin"]) < 1.0
    # frozen rows (round 6): the epoch-bounded freeze test and the history-free recurrence
    assert int(stats["frozen-mismatches"]) == 0
    assert int(stats["frozen-elements"]) > 1000
