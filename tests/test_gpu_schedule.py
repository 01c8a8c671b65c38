"""The step's issue schedule does not change its bits: five in-batch plan steps (tests/
schedule_worker.py, one process per variant, run one after another) give bit-identical losses,
dense parameters and user table with the side-issue thread on and off (DCUE_SIDE_THREAD, csrc/side.hip)
and under each scheduling A/B knob of DESIGN.md §4.7 round 4 (a fork event after the score kernel,
the prologue before the forward, one late wait before conv 1, the lookahead at the dgrad fork, the
user tower's forward as three launches) and the fused user-tower forward.
Every variant orders the same kernels by the same data
dependencies, so any difference would be a missing order."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VARIANTS = [
    {},
    {"DCUE_SIDE_THREAD": "0"},
    {"DCUE_SCORE_FORK": "1"},
    {"DCUE_PROLOGUE_FIRST": "1"},
    {"DCUE_LATE_WAIT": "conv1"},
    {"DCUE_AHEAD_AT": "fork"},
    {"DCUE_USER_FWD": "split"},
    {"DCUE_USER_FWD": "split", "DCUE_SIDE_THREAD": "0"},
]
# (the fused user tower, the default since round 5: its round-4 non-finite runs were the plan's
# cross-stream races, not the kernel -- DESIGN.md §4.7 round 5, tests/test_gpu_races.py)


def test_schedule_variants_bit_identical(tmp_path):
    res = []
    for i, extra in enumerate(VARIANTS):
        out = os.path.join(tmp_path, "v%d.pt" % i)
        env = dict(os.environ, OUT=out, **extra)
        for k in ("DCUE_SIDE_THREAD", "DCUE_SCORE_FORK", "DCUE_PROLOGUE_FIRST", "DCUE_LATE_WAIT",
                  "DCUE_AHEAD_AT", "DCUE_USER_FWD"):
            if k not in extra:
                env.pop(k, None)
        p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "schedule_worker.py")], env=env,
                           stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=100)
        assert p.returncode == 0, "variant %s failed:\n%s" % (extra, p.stdout[-3000:])
        res.append(torch.load(out, weights_only=True))
    base = res[0]
    for extra, r in zip(VARIANTS, res):
        assert torch.isfinite(r["loss"]).all(), "non-finite loss under %s" % extra
        assert r["fail_flags"] == 0, "fused user forward gave up a wait under %s" % extra
    for extra, r in zip(VARIANTS[1:], res[1:]):
        for k in ("loss", "P", "emb"):
            assert torch.equal(r[k], base[k]), "%s differs under %s" % (k, extra)
