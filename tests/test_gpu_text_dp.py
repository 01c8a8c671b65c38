"""BASELINE config 4 (mixed audio + text item tower, d = 256) data parallel, on two ranks of one GPU
(gloo host transport; tests/text_dp_worker.py): plan.step with the native split exchange is bit-exact
with launch + an explicit all-reduce mean + NativeAdam on a twin, over back-to-back steps, with the
text segments (text.conv.*, the widened fc) inside the exchange buckets. Parity unpinned against the
reference (its text encoder was never published, reference datasets/dcuelmitemset.py:8)."""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_text_tower_world2(tmp_path):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    world, procs = 2, []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), OUT=str(tmp_path))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "text_dp_worker.py")],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out)
    for r, p in enumerate(procs):
        assert p.returncode == 0, "rank %d failed:\n%s" % (r, outs[r][-3000:])
    print("\n".join(o.strip() for o in outs))
    res = [torch.load(os.path.join(tmp_path, "r%d.pt" % r), weights_only=True) for r in range(world)]
    for r in res:
        assert r["bad"] == [] and r["finite"] and r["replicas"] and r["moved"], r
    assert torch.equal(res[0]["P"], res[1]["P"])
