"""BASELINE config 5 data parallel, on two ranks of one GPU (gloo; tests/dcbr_worker.py): the
row-sharded WRMF (each rank solves 1/world of the rows, dcue_comm_allgather hands every rank all of
them) bit-exact with a one-rank fit, and the DCBR regression with its dense gradient averaged over
the ranks bit-exact with an explicit all-reduce mean + NativeAdam on a twin model, one replica.
Parity unpinned against the reference (DCBR was never published, reference .gitignore:13)."""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_dcbr_world2(tmp_path):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    world, procs = 2, []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), OUT=str(tmp_path))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "dcbr_worker.py")],
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
        assert r["wrmf_ok"] and r["twin"] and r["replicas"], r
    assert torch.equal(res[0]["P"], res[1]["P"])
