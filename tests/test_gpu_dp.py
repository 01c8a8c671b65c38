"""Data-parallel gradient exchange with overlap (row e, dcrecommend.distributed): two ranks on one
GPU (gloo), the bucketed all-reduce issued behind the step against a plain post-step all-reduce.

Bar: bit-exact (two addends per element either way). The ranks are child processes
(tests/dp_worker.py), started with subprocess like any other program.
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


def test_overlapped_allreduce_matches_plain(tmp_path):
    world, port = 2, _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), OUT=str(tmp_path))
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "dp_worker.py")], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
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
    parts = [torch.load(os.path.join(tmp_path, "r%d.pt" % r), weights_only=True) for r in range(world)]
    assert torch.equal(parts[0]["G"], parts[1]["G"])  # the mean is the same on every rank
    assert 0 < parts[0]["late"] < parts[0]["G"].numel()
