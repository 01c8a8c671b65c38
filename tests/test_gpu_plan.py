"""Step plans (include/dcue.h dcue_plan_*, eager and HIP-graph replay) and live kernel timers.

Bar: a replayed plan is BIT-EXACT with the same step issued call by call (it runs the very same
kernels), in both batch layouts and both replay modes, with the deferred user-table Adam running
between replays.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _nets(n=2, E=40, n_users=40, seed=5):
    from dcrecommend.dcue.dcue import DCUENet
    out = []
    for _ in range(n):
        torch.manual_seed(seed)
        out.append(DCUENet({"feature_dim": 32, "conv_hidden": 32, "user_embdim": E, "user_count": n_users,
                            "model_type": "truedcuemel1dbn"}).cuda().train())
    return out


def _mt(seed):
    from dcrecommend import _native as nat
    st = torch.empty(nat.MT_STATE_BYTES, dtype=torch.uint8, device=DEV)
    nat.check(nat.lib().dcue_mt_seed(nat.ptr(st), seed, nat.stream_handle()), "mt_seed")
    return st


def _state(net, opt):
    out = {k: v.detach().clone() for k, v in net.state_dict().items()}
    for k, v in opt._adam_state().items():
        if k in ("m", "v", "em", "ev"):
            out["adam." + k] = v.clone()
    out["grad"] = net._flat["G"].clone()
    return out


@pytest.mark.parametrize("inbatch,graph,fused_adam,lookahead", [
    (True, False, False, False), (False, False, False, False), (True, True, False, False),
    (False, True, False, False), (True, False, True, False),
    # dcue_plan_set_next: bn0 statistics and the conv-1 wgrad input prepared one step ahead (a
    # withdrawn announcement and a mismatched one fall back to computing them in the step)
    (True, False, True, True), (True, False, False, True)])
def test_plan_replay_matches_eager(inbatch, graph, fused_adam, lookahead):
    from dcrecommend import _native as nat
    from dcrecommend.dcue.plan import TrainPlan
    from dcrecommend.optim import NativeAdam
    n_users, B, N, n_tracks, steps = 40, 8, 3, 48, 6
    eager, replayed = _nets()
    gen = torch.Generator(device=DEV).manual_seed(11)
    tracks = torch.randn((n_tracks, 131, 128), generator=gen, device=DEV).half()
    opts = [NativeAdam(n.parameters(), 1e-3, (0.9, 0.99), 1e-8, 0, defer_embedding=True, flush_every=4)
            for n in (eager, replayed)]
    mts = [_mt(21), _mt(21)]
    M = B if inbatch else B * (1 + N)
    plan = TrainPlan(replayed, tracks, B, N, mt_state=mts[1] if inbatch else None, graph=graph,
                     optimizer=opts[1] if fused_adam else None)
    neg = torch.zeros((B, N), dtype=torch.int32, device=DEV)
    all_users = [torch.randint(0, n_users, (B,), generator=gen, device=DEV) for _ in range(steps)]
    all_items = [torch.randint(0, n_tracks, (M,), generator=gen, device=DEV, dtype=torch.int64).to(torch.int32)
                 for _ in range(steps)]
    decoy = all_items[0].clone()
    for s in range(steps):
        users, items = all_users[s], all_items[s]
        if lookahead and s + 1 < steps:
            if s == 2:
                assert plan.set_next(None)  # withdrawn: step 3 computes its own
            elif s == 3:
                assert plan.set_next(decoy)  # step 4 passes another buffer: computed in the step
            else:
                assert plan.set_next(all_items[s + 1])
        if inbatch:
            nat.check(nat.lib().dcue_sample_inbatch(nat.ptr(mts[0]), B, N, nat.ptr(neg), nat.stream_handle()),
                      "sample")
            eager.native_forward(users, tracks, items, N, nat.LAYOUT_GATHER, neg, train=True, margin=0.2)
        else:
            eager.native_forward(users, tracks, items, N, nat.LAYOUT_CATALOGUE, None, train=True, margin=0.2)
        eager.native_backward(None)
        opts[0].step()
        if fused_adam:
            plan.step(users, items)  # launch + Adam in one call
        else:
            plan.launch(users, items)
            opts[1].step()
    if inbatch:
        assert torch.equal(neg, plan.neg_item)
    a, b = _state(eager, opts[0]), _state(replayed, opts[1])
    for k in a:
        assert torch.equal(a[k], b[k]), k
    plan.close()


def test_timer_counts_eager_and_plan_launches():
    from dcrecommend import _native as nat
    from dcrecommend.dcue.plan import TrainPlan
    net, = _nets(1)
    gen = torch.Generator(device=DEV).manual_seed(3)
    tracks = torch.randn((16, 131, 128), generator=gen, device=DEV).half()
    B, N = 8, 2
    users = torch.randint(0, 40, (B,), generator=gen, device=DEV)
    items = torch.randint(0, 16, (B * (1 + N),), generator=gen, device=DEV, dtype=torch.int64).to(torch.int32)
    nat.timer_read(nat.TIMED_CONV1_WGRAD)  # reset
    nat.timer_enable(nat.TIMED_CONV1_WGRAD, True)
    try:
        for _ in range(2):
            net.native_forward(users, tracks, items, N, nat.LAYOUT_CATALOGUE, None, train=True)
            net.native_backward(None)
        ms, n = nat.timer_read(nat.TIMED_CONV1_WGRAD)
        assert n == 2 and ms > 0.0
        for graph in (False, True):
            plan = TrainPlan(net, tracks, B, N, item_track=items, graph=graph)
            for _ in range(3):
                plan.launch(users)
            ms, n = nat.timer_read(nat.TIMED_CONV1_WGRAD)
            assert n == 3 and ms > 0.0
            plan.close()
        # the per-launch read (dcue_timer_samples): one positive duration per timed launch, then reset
        for _ in range(2):
            net.native_forward(users, tracks, items, N, nat.LAYOUT_CATALOGUE, None, train=True)
            net.native_backward(None)
        samples = nat.timer_samples(nat.TIMED_CONV1_WGRAD)
        assert len(samples) == 2 and all(v > 0.0 for v in samples)
        assert nat.timer_samples(nat.TIMED_CONV1_WGRAD) == []
    finally:
        nat.timer_enable(nat.TIMED_CONV1_WGRAD, False)


def test_destroy_right_after_step_keeps_deferred_table_exact():
    """A deferred-embedding plan closed straight after plan.step(): the rolling-flush slice the next
    launch would have issued runs at destruction, ordered after the last step's user-table Adam on
    the user stream. The table and its moments then equal a dense-sweep run bit for bit."""
    from dcrecommend.dcue.plan import TrainPlan
    from dcrecommend.optim import NativeAdam
    n_users, B, N, n_tracks = 40, 8, 3, 48
    deferred, dense = _nets()
    gen = torch.Generator(device=DEV).manual_seed(13)
    tracks = torch.randn((n_tracks, 131, 128), generator=gen, device=DEV).half()
    batches = [(torch.randint(0, n_users, (B,), generator=gen, device=DEV),
                torch.randint(0, n_tracks, (B,), generator=gen, device=DEV).to(torch.int32)) for _ in range(7)]
    outs = []
    for net, defer in ((deferred, True), (dense, False)):
        opt = NativeAdam(net.parameters(), 1e-3, (0.9, 0.99), 1e-8, 0, defer_embedding=defer, flush_every=4)
        plan = TrainPlan(net, tracks, B, N, mt_state=_mt(21), optimizer=opt)
        for u, it in batches:
            plan.step(u, it)
        plan.close()  # no synchronisation in between
        opt.flush() if defer else None
        torch.cuda.synchronize()
        outs.append(_state(net, opt))
    for k in outs[1]:
        if k == "grad":
            continue
        assert torch.equal(outs[0][k], outs[1][k]), k
