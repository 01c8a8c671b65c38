"""Cross-stream orders of the plan step, tested by schedule perturbation (include/dcue.h
dcue_debug_delay, tests/race_worker.py).

A plan step runs on four streams (the caller's, the user stream, two weight-gradient streams) and
steps follow each other without a host synchronisation, so the previous step's side-stream work
overlaps the next step's start. Every buffer must be ordered by the streams' events, not by how the
timing usually falls. Here a spin kernel of several milliseconds is injected ahead of the work at one
site at a time -- far longer than the host's lead over the GPU -- and the five steps must come out
bit-identical to the undelayed run (losses, dense parameters, user table). A missing wait shows as a
difference, deterministically, on every run.

Round 4's intermittent divergence was two such missing waits (DESIGN.md §4.7,
round 5): the next step's prologue cleared the accumulator slot that the layer-2 weight gradient of
the previous step was still reading on wgrad stream 1 (its split-f16 range words read as "no value",
a NaN operand scale), and the late Adam rewrote conv 2's packed weights while the caller's stream
could still be in conv 2's input gradient. test_legacy_orders_fail runs round 4's orders
(DCUE_LEGACY_ORDERS=1) under the same delays and requires the detector to catch both."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))

DELAY_US = 5000
SITES = ["user_fwd", "user_bwd", "wgrad_hi", "wgrad_2", "late_adam", "prologue", "lookahead", "conv2", "dgrad_2",
         "wgrad_1"]


def _check(base, r, what):
    import race_worker as W
    assert W.finite(r), "%s: non-finite (probes: %s)" % (what, r["probes"])
    for k in ("loss", "P", "emb"):
        assert torch.equal(r[k], base[k]), "%s: %s differs from the undelayed run" % (what, k)


@pytest.mark.parametrize("tower", ["bn", "text", "res"])
def test_delays_bit_identical(tower):
    import race_worker as W
    from dcrecommend import _native as nat
    base = W.run(tower)
    assert W.finite(base)
    sites = SITES + (["fc_wgrad"] if tower in ("text", "res") else []) + (["text_fwd"] if tower == "text" else [])
    for site in sites:
        _check(base, W.run(tower, {site: DELAY_US}), "%s tower, delay at %s" % (tower, site))
    # every side stream late at once
    _check(base, W.run(tower, {s: 2000 for s in ("user_bwd", "wgrad_hi", "wgrad_2", "late_adam")}),
           "%s tower, all side streams delayed" % tower)
    assert nat.debug_fail_flags() == 0


def test_catalogue_plan_delays():
    import race_worker as W
    base = W.run("bn", inbatch=False)
    for site in ("user_bwd", "wgrad_2", "late_adam", "prologue", "dgrad_2"):
        _check(base, W.run("bn", {site: DELAY_US}, inbatch=False), "catalogue plan, delay at %s" % site)


def test_poisoned_scratch_and_probes():
    """Workspace and plan scratch filled with NaN bytes before use (DCUE_POISON): no kernel reads a
    word it did not write first -- the run equals the unpoisoned one and every probe stays finite."""
    import race_worker as W
    from dcrecommend import _native as nat
    base = W.run("bn")
    os.environ["DCUE_POISON"] = "1"
    nat.lib().dcue_debug_poison(1)
    try:
        r = W.run("bn", check="probe")
        rt = W.run("text", check="probe")
    finally:
        os.environ.pop("DCUE_POISON", None)
        nat.lib().dcue_debug_poison(0)
    assert r["probes"] == [] and rt["probes"] == [], (r["probes"], rt["probes"])
    _check(base, r, "poisoned scratch")
    assert W.finite(rt)


def test_legacy_orders_fail():
    """The detector has teeth: with round 4's orders (DCUE_LEGACY_ORDERS=1) a delayed layer-2 weight
    gradient and a delayed conv-2 input gradient both change the run; the probes name the first
    kernel that went non-finite."""
    env = dict(os.environ, DCUE_LEGACY_ORDERS="1")
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "race_worker.py"), "bn",
                        "wgrad_2,dgrad_2", str(DELAY_US)], env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True, timeout=100)
    assert p.returncode == 0, p.stdout[-3000:]
    res = json.loads(p.stdout.strip().splitlines()[-1])
    print(res)
    assert res["legacy_orders"] == "1" and res["base_finite"]
    assert not res["wgrad_2"]["identical"], res
    assert not res["dgrad_2"]["identical"], res


def test_text_position_parts_delays():
    """the text branch runs on a side stream; with position parts (DCUE_TEXT_PARTS=2) its
    two workgroups per item merge through tickets in the accumulator block's forward part. The
    tickets are cleared in the text stream's own order (the plan's prologue, or the branch's own clear
    in eager launches), never by the caller stream's accumulator clear. Delays at the text forward, the
    user tower and conv 2 must leave the run bit-identical."""
    env = dict(os.environ, DCUE_TEXT_PARTS="2")
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "race_worker.py"), "text32",
                        "text_fwd,user_fwd,conv2", str(DELAY_US)], env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True, timeout=100)
    assert p.returncode == 0, p.stdout[-3000:]
    res = json.loads(p.stdout.strip().splitlines()[-1])
    print(res)
    assert res["base_finite"]
    for site in ("text_fwd", "user_fwd", "conv2"):
        assert res[site]["identical"] and res[site]["finite"], (site, res[site])
