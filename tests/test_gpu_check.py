"""Check mode (a HIP bounds/NaN check mode; dcrecommend.check, include/dcue.h
dcue_check_*): the probes flag exactly what they should, and a TrainPlan in check mode refuses a
batch with an out-of-range track id before any kernel indexes the table with it, and raises on a
step whose outputs are not finite."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def test_probes():
    from dcrecommend.check import StepCheck
    ck = StepCheck(DEV)
    ok = torch.randn(1001, device=DEV)
    ck.finite(ok, "clean")
    ck.ids(torch.arange(10, device=DEV, dtype=torch.int32), 10, "ids in range")
    assert ck.failed() == []
    for v in (float("nan"), float("inf"), float("-inf")):
        bad = ok.clone()
        bad[997] = v  # in the scalar tail past the last float4
        ck.finite(bad, "tail %s" % v)
        bad = ok.clone()
        bad[5] = v
        ck.finite(bad, "body %s" % v)
    ck.ids(torch.tensor([0, 3, 10], device=DEV), 10, "id == limit")
    ck.ids(torch.tensor([-1, 3], device=DEV, dtype=torch.int32), 10, "negative id")
    assert set(ck.failed()) == {"tail nan", "body nan", "tail inf", "body inf", "tail -inf", "body -inf",
                                "id == limit", "negative id"}
    with pytest.raises(RuntimeError, match="DCUE check mode"):
        ck.raise_if_any()
    assert ck.failed() == []  # cleared by the raise


def test_plan_in_check_mode():
    from dcrecommend import _native as nat
    from dcrecommend.dcue.dcue import DCUENet
    from dcrecommend.dcue.plan import TrainPlan
    from dcrecommend.optim import NativeAdam
    torch.manual_seed(0)
    net = DCUENet({"feature_dim": 32, "conv_hidden": 32, "user_embdim": 40, "user_count": 30,
                   "model_type": "truedcuemel1dbn"}).to(DEV).train()
    opt = NativeAdam(net.parameters(), 1e-3, (0.9, 0.99), 1e-8, 0)
    gen = torch.Generator(device=DEV).manual_seed(2)
    tracks = torch.randn((40, 131, 128), generator=gen, device=DEV).half()
    mt = torch.empty(nat.MT_STATE_BYTES, dtype=torch.uint8, device=DEV)
    nat.check(nat.lib().dcue_mt_seed(nat.ptr(mt), 1, nat.stream_handle()), "mt_seed")
    B, N = 8, 3
    plan = TrainPlan(net, tracks, B, N, mt_state=mt, optimizer=opt, check=True)
    users = torch.randint(0, 30, (B,), generator=gen, device=DEV)
    items = torch.randint(0, 40, (B,), generator=gen, device=DEV).to(torch.int32)
    plan.step(users, items)  # a clean step passes
    bad = items.clone()
    bad[3] = 40
    with pytest.raises(RuntimeError, match="item ids outside the track table"):
        plan.step(users, bad)
    with pytest.raises(RuntimeError, match="user ids outside the table"):
        plan.step(users + 30, items)
    with torch.no_grad():
        net.conv.fc.weight[0, 0] = float("nan")
    with pytest.raises(RuntimeError, match="non-finite"):
        plan.step(users, items)
    plan.close()
