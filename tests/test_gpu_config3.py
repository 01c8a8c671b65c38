"""BASELINE.json configs[2] at its per-GPU shape: 1M users x 1M tracks, 50M interactions over 8
data-parallel replicas is, per rank, 125k local users (the user-sharded table), the whole 1M-track
table replicated in HBM (33.5 GB fp16) and 6.25M interactions.

Run on one MI355X as property tests (no oracle finishes these sizes):
  * addressing past 2^31 elements: the table holds 1M tracks tiled from a 65,536-track random
    block, so track t and t mod 65,536 carry identical spectrograms; features and train-mode
    scores/loss computed from the high ids equal those from their low twins bit for bit (every
    kernel that indexes the table must use 64-bit offsets: track 999,999 starts at element 1.68e10);
  * training: 300 in-batch TrainPlan steps (fused NativeAdam, deferred 125k-row user table): the
    loss stays finite and falls; after a flush the table and moments are finite;
  * the catalogue sampler at 1M tracks (datasets/dcuedataset.py:207-220): draws are split songs the
    user never interacted with, and catalogue steps train with finite loss.
"""
import os
import sys
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
N_USERS, N_TRACKS, N_PAIRS = 125_000, 1_000_000, 6_250_000
BLOCK = 65_536
B, N = 64, 20


@pytest.fixture(scope="module")
def world():
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import song_split
    t0 = time.perf_counter()
    gen = torch.Generator(device=DEV).manual_seed(5)
    tracks = torch.empty((N_TRACKS, 131, 128), dtype=torch.float16, device=DEV)
    tracks[:BLOCK] = torch.randn((BLOCK, 131, 128), generator=gen, device=DEV).half()
    for s in range(BLOCK, N_TRACKS, BLOCK):
        e = min(N_TRACKS, s + BLOCK)
        tracks[s:e] = tracks[:e - s]
    pair_user = torch.randint(0, N_USERS, (N_PAIRS,), generator=gen, device=DEV)
    pair_track = torch.randint(0, N_TRACKS, (N_PAIRS,), generator=gen, device=DEV)
    split = song_split(N_TRACKS)
    torch.cuda.synchronize()
    print("config-3 table %.1f GB built in %.1f s" % (tracks.numel() * 2 / 1e9, time.perf_counter() - t0))
    return tracks, pair_user, pair_track, split


def _net(lr):
    from dcrecommend.dcue.dcue import DCUENet
    from dcrecommend.optim import NativeAdam
    torch.manual_seed(0)
    net = DCUENet({"feature_dim": 128, "conv_hidden": 128, "user_embdim": 300, "user_count": N_USERS,
                   "model_type": "truedcuemel1dbn"}).to(DEV)
    net.train()
    opt = NativeAdam(net.parameters(), lr, (0.9, 0.99), 1e-8, 0, defer_embedding=True)
    return net, opt


def test_table_addressing_past_2_31(world):
    from dcrecommend import _native as nat
    tracks = world[0]
    assert tracks.numel() * tracks.element_size() >= 33.5e9
    net, _ = _net(1e-4)
    rs = np.random.RandomState(0)
    high = torch.from_numpy(rs.randint(N_TRACKS - BLOCK, N_TRACKS, B * (1 + N))).to(DEV, torch.int32)
    high[0] = N_TRACKS - 1  # the table's last element: 1.68e10 elements in
    low = high % BLOCK
    users = torch.from_numpy(rs.randint(0, N_USERS, B)).to(DEV)
    users[0] = N_USERS - 1
    out = {}
    # eval mode first: a train-mode forward moves the BN running statistics the eval forward reads
    for train in (False, True):
        for name, ids in (("high", high), ("low", low)):
            s, uf, f, loss = net.native_forward(users, tracks, ids, N, nat.LAYOUT_CATALOGUE, train=train)
            out[name, train] = (s, uf, f, loss)
    for train in (False, True):
        for a, b, what in zip(out["high", train], out["low", train], ("scores", "user feats", "item feats", "loss")):
            assert torch.isfinite(a).all(), what
            assert torch.equal(a, b), "%s differ between high track ids and their low twins (train=%s)" % (what, train)


def test_inbatch_training_at_config3(world):
    from dcrecommend import _native as nat
    from dcrecommend.dcue.plan import TrainPlan
    tracks, pair_user, pair_track, _ = world
    net, opt = _net(1e-3)
    mt = torch.empty(nat.MT_STATE_BYTES, dtype=torch.uint8, device=DEV)
    nat.check(nat.lib().dcue_mt_seed(nat.ptr(mt), 3, nat.stream_handle()), "mt_seed")
    plan = TrainPlan(net, tracks, B, N, mt_state=mt, optimizer=opt)
    steps = 300
    gen = torch.Generator(device=DEV).manual_seed(9)
    # a pool of 10 batches cycled: the loss must fall as the towers fit them (fresh random
    # interactions every step leave nothing to learn, and their loss only wanders)
    rows = torch.randint(0, N_PAIRS, (10, B), generator=gen, device=DEV).repeat(steps // 10, 1)
    ub = pair_user[rows].contiguous()
    ib = pair_track[rows].to(torch.int32).contiguous()
    losses = torch.empty(steps, device=DEV)
    t0 = time.perf_counter()
    for s in range(steps):
        plan.step(ub[s], ib[s])
        losses[s].copy_(plan.loss)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    plan.close()
    opt.flush()
    L = losses.cpu().numpy()
    print("config-3 in-batch: %.3f ms/step, loss %.4f (first 50) -> %.4f (last 50)"
          % (dt / steps * 1e3, L[:50].mean(), L[-50:].mean()))
    assert np.isfinite(L).all()
    assert L[-50:].mean() < L[:50].mean()
    st = opt._adam_state()
    for k in ("em", "ev"):
        assert torch.isfinite(st[k]).all(), k
    assert torch.isfinite(net.user_embd.embeddings.weight).all()
    assert torch.isfinite(net._flat["P"]).all()


def test_catalogue_sampler_and_steps_at_config3(world):
    from dcrecommend import _native as nat
    from dcrecommend.datasets.csr import check_catalogue_users, saturated_users, user_split_ranks
    from dcrecommend.dcue.plan import TrainPlan
    tracks, pair_user, pair_track, split = world
    t0 = time.perf_counter()
    pu, pt = pair_user.cpu().numpy(), pair_track.cpu().numpy()
    split_items = np.nonzero(split == 0)[0].astype(np.int64)
    indptr, ranks = user_split_ranks(pu, pt, N_USERS, split_items)
    t_csr = time.perf_counter() - t0
    sat = saturated_users(indptr, len(split_items))
    net, opt = _net(1e-4)
    plan = TrainPlan(net, tracks, B, N, optimizer=opt)
    split_d = torch.from_numpy(split_items).to(DEV)
    indptr_d = torch.from_numpy(indptr).to(DEV)
    ranks_d = torch.from_numpy(ranks).to(DEV)
    mt = torch.empty(nat.MT_STATE_BYTES, dtype=torch.uint8, device=DEV)
    nat.check(nat.lib().dcue_mt_seed(nat.ptr(mt), 11, nat.stream_handle()), "mt_seed")
    negs = torch.empty((B, N), dtype=torch.int64, device=DEV)
    gen = torch.Generator(device=DEV).manual_seed(4)
    steps = 20
    losses = torch.empty(steps, device=DEV)
    drawn = []
    for s in range(steps):
        rows = torch.randint(0, N_PAIRS, (B,), generator=gen, device=DEV)
        users, pos = pair_user[rows].contiguous(), pair_track[rows].contiguous()
        check_catalogue_users(users.cpu().numpy(), sat)
        nat.check(nat.lib().dcue_sample_catalogue(nat.ptr(mt), 0, 0, nat.ptr(split_d), split_d.numel(),
                                                  nat.ptr(indptr_d), nat.ptr(ranks_d), nat.ptr(users), B, N,
                                                  nat.ptr(negs), nat.stream_handle()), "dcue_sample_catalogue")
        drawn.append((users.cpu().numpy(), negs.cpu().numpy()))
        nat.check(nat.lib().dcue_build_catalogue_batch(nat.ptr(pos), nat.ptr(negs), B, N, nat.ptr(plan.item_track),
                                                       nat.stream_handle()), "dcue_build_catalogue_batch")
        plan.step(users, None)
        losses[s].copy_(plan.loss)
    torch.cuda.synchronize()
    plan.close()
    print("config-3 catalogue: host CSR over %d interactions in %.2f s; %d split songs" % (N_PAIRS, t_csr,
                                                                                           len(split_items)))
    assert torch.isfinite(losses).all()
    # every draw: a split song outside the user's interactions (all splits)
    order = np.argsort(pu, kind="stable")
    start = np.searchsorted(pu[order], np.arange(N_USERS + 1))
    for users, ng in drawn:
        assert (split[ng] == 0).all()
        for u, row in zip(users, ng):
            mine = pt[order[start[u]:start[u + 1]]]
            assert not np.isin(row, mine).any()
