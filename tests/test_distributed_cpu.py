"""World-size-2 gloo tests of the data-parallel layout (dcrecommend.distributed, bench.py's N>1 path).

CPU only: the HIP step itself needs a GPU, but everything the ranks exchange or partition is host
logic -- user sharding, the dense-gradient mean, the max-over-ranks timing -- and runs here on gloo.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dcrecommend import distributed as D
        rs = np.random.RandomState(0)
        n_users, n_items, n_pairs = 101, 50, 1000
        users = torch.from_numpy(rs.randint(0, n_users, n_pairs))
        items = torch.from_numpy(rs.randint(0, n_items, n_pairs))
        lu, li = D.shard_interactions(users, items, rank, world)
        assert int(lu.max()) < D.local_user_count(n_users, rank, world)
        glob = D.to_global_user(lu, rank, world)
        assert bool(((glob % world) == rank).all())
        # replicated dense grad: every rank holds its own, the mean comes back everywhere
        g = torch.arange(8, dtype=torch.float32) * (rank + 1)
        D.allreduce_mean_(g)
        # the bucketed exchange (CPU branch: buckets in order) gives the same mean
        class _Plan:
            waits = 0

            def wait_side(self, stream):
                _Plan.waits += 1
        g2 = torch.arange(8, dtype=torch.float32) * (rank + 1)
        D.allreduce_mean_overlapped_(_Plan(), g2, 3)
        assert torch.equal(g2, g) and _Plan.waits == 1
        t = D.max_over_ranks(1.5 + rank, torch.device("cpu"))
        torch.save({"glob": glob, "items": li, "g": g, "t": t}, os.path.join(out_dir, "r%d.pt" % rank))
    finally:
        dist.destroy_process_group()


def test_user_sharding_and_grad_mean_world2(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    parts = [torch.load(os.path.join(tmp_path, "r%d.pt" % r), weights_only=True) for r in range(world)]
    rs = np.random.RandomState(0)
    users = rs.randint(0, 101, 1000)
    items = rs.randint(0, 50, 1000)
    # the shards partition the interaction set (each pair exactly once, on its user's rank)
    got = sorted(zip(torch.cat([p["glob"] for p in parts]).tolist(), torch.cat([p["items"] for p in parts]).tolist()))
    assert got == sorted(zip(users.tolist(), items.tolist()))
    expect = torch.arange(8, dtype=torch.float32) * 1.5
    for p in parts:
        assert torch.equal(p["g"], expect)
        assert p["t"] == 2.5


def test_local_user_counts_cover_table():
    from dcrecommend import distributed as D
    for n in (0, 1, 7, 100, 101):
        for w in (1, 2, 3, 8):
            assert sum(D.local_user_count(n, r, w) for r in range(w)) == n
