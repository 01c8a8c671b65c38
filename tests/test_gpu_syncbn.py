"""Row e on two ranks of one GPU (gloo; tests/syncbn_worker.py): the plan's native data-parallel
exchange at world 2 over the library's host transport (distributed.HostComm -- RCCL refuses two
ranks on one GPU), and SyncBN (dcue_plan_set_sync_bn) against a one-rank run over the global batch.

Bars: part 1 bit-exact (launch + all-reduce mean + Adam on a twin model; replicas identical across
ranks); part 2 the SyncBN mean gradient and running statistics within 1e-4 of max of the one-rank
global-batch run, while per-replica BatchNorm misses it by more than 1e-3 of max.
"""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_native_exchange_world2_and_sync_bn(tmp_path):
    world, port = 2, _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), OUT=str(tmp_path))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "syncbn_worker.py")],
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
    assert torch.equal(res[0]["P"], res[1]["P"])  # part 1: one dense replica
    assert torch.equal(res[0]["G"], res[1]["G"])  # part 2: the exchanged mean is the same everywhere
    for r in res:
        assert r["err_sync"] <= 1e-4 * r["scale"], r
        assert r["bn_err"] <= 1e-4, r
        assert r["err_plain"] > 1e-3 * r["scale"], r  # the test has teeth: per-replica BN differs
