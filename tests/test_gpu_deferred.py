"""Deferred user-table Adam (include/dcue.h dcue_emb_log) against the dense per-step sweep.

The reference's dense embedding gradient makes torch.optim.Adam step every user row each batch
(nn/dcue.py:143-147,209). NativeAdam(defer_embedding=True) performs the zero-gradient steps of rows
outside the batch later, replaying the recorded per-step scalars through the same fp32 operations.
Bar: BIT-EXACT -- after any flush every parameter, buffer and Adam moment equals the dense run's.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _pair(E, n_users, seed=3):
    from dcrecommend.dcue.dcue import DCUENet
    nets = []
    for _ in range(2):
        torch.manual_seed(seed)
        nets.append(DCUENet({"feature_dim": 32, "conv_hidden": 32, "user_embdim": E,
                             "user_count": n_users, "model_type": "truedcuemel1dbn"}).cuda())
    return nets


def _state(net, opt):
    out = {k: v.detach().clone() for k, v in net.state_dict().items()}
    st = opt._adam_state()
    for k in ("m", "v", "em", "ev"):
        out["adam." + k] = st[k].clone()
    return out


def _assert_equal_state(a, b):
    assert a.keys() == b.keys()
    for k in a:
        assert torch.equal(a[k], b[k]), "%s differs: max |diff| %.3e" % (k, float((a[k].double() - b[k].double()).abs().max()))


@pytest.mark.parametrize("E,wd,flush_every,steps,n_users,B", [
    (40, 0.0, 4, 13, 40, 8), (30, 1e-3, 5, 13, 40, 8), (300, 0.0, 64, 13, 40, 8),
    # > DCUE_MAX_LOG_CAP (256) steps between full flushes: only the rolling slices keep rows current
    (40, 0.0, 8, 300, 40, 8), (30, 1e-3, 16, 270, 40, 8),
    # users idle for hundreds of steps: the replay's long-idle shortcut (csrc/adam_replay.h) runs in
    # the rolling slices and in the forward's sync of returning users
    (300, 0.0, 64, 420, 600, 4), (64, 0.0, 16, 420, 600, 4)])
def test_deferred_matches_dense_bit_exact(E, wd, flush_every, steps, n_users, B):
    from dcrecommend import _native as nat
    from dcrecommend.optim import NativeAdam
    from dcrecommend.optim.cyclic_scheduler import CyclicLRWithRestarts
    N, n_tracks = 3, 48
    dense, lazy = _pair(E, n_users)
    gen = torch.Generator(device=DEV).manual_seed(7)
    tracks = torch.randn((n_tracks, 131, 128), generator=gen, device=DEV).half()
    opts, scheds = [], []
    for net, defer in ((dense, False), (lazy, True)):
        net.train()
        opt = NativeAdam(net.parameters(), 1e-3, (0.9, 0.99), 1e-8, wd, defer_embedding=defer,
                         flush_every=flush_every)
        sch = CyclicLRWithRestarts(opt, B, epoch_size=20 * B, restart_period=1, t_mult=2, policy="cosine")
        sch.step()
        opts.append(opt)
        scheds.append(sch)
    for s in range(steps):
        users = torch.randint(0, n_users, (B,), generator=gen, device=DEV)
        if s == 2:
            users[1] = users[0]  # a user twice in one batch
        items = torch.randint(0, n_tracks, (B,), generator=gen, device=DEV, dtype=torch.int64).to(torch.int32)
        neg = torch.randint(0, B, (B, N), generator=gen, device=DEV, dtype=torch.int64).to(torch.int32)
        losses = []
        for net, opt, sch in zip((dense, lazy), opts, scheds):
            if s and s % 20 == 0:
                sch.step()  # next epoch of 20 batches (batch_step raises past the epoch's count)
            _, _, _, loss = net.native_forward(users, tracks, items, N, nat.LAYOUT_GATHER, neg, train=True,
                                               margin=0.2)
            losses.append(loss.clone())
            net.native_backward(None)
            opt.step()
            sch.batch_step()
        assert torch.equal(losses[0], losses[1]), "step %d loss differs" % s
        if s == 6 and steps < 100:  # a flush between periodic ones (state_dict flushes)
            _assert_equal_state(_state(dense, opts[0]), _state(lazy, opts[1]))
    # eval-mode user features sync only the rows they read
    probe = torch.arange(n_users, device=DEV)
    dense.eval()
    lazy.eval()
    assert torch.equal(dense.user_features(probe), lazy.user_features(probe))
    _assert_equal_state(_state(dense, opts[0]), _state(lazy, opts[1]))
