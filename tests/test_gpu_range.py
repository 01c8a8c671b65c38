"""Range of the split-f16 conv forwards.

Every forward conv multiplies its BN-applied (or raw) input as fp16 pairs, v*S = hi + lo, with a
power-of-two scale S per launch from the input layer's value range (conv.hip range_stage): the
largest |v| lands in [2^14, 2^15), so nothing overflows fp16 and small activations stay clear of
fp16's subnormals. The BatchNorm-free towers feed raw ReLU activations forward
(audiomodels/truedcuemel1d.py, truedcuemel1dres.py:74-97), so their magnitudes follow the input's.
Here the input spectrograms are scaled by 1e3 and 1e-3 (and 1e5, past fp16's 65504, on the fp32
table the module API builds), and one train step's scores, loss and every dense gradient are
checked against the fp64 oracle (oracle/dcue_oracle.py, the reference step restated): scores and
loss within 1e-4 of their max (north_star), gradients within 1e-3 of their max (as the golden tests).
The eval forward (running statistics; the ranges come from the batch itself) is checked the same way.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _step(model_type, scale, H=64, d=32, n_users=9, B=6, N=3, E=40, seed=3):
    from dcrecommend.dcue.dcue import DCUENet
    from oracle import dcue_oracle as O
    torch.manual_seed(seed)
    net = DCUENet({"feature_dim": d, "conv_hidden": H, "user_embdim": E, "user_count": n_users,
                   "model_type": model_type}).to(DEV).train()
    torch.manual_seed(seed)
    p, b = O.init_params(d, H, E, n_users, model_type)
    gen = torch.Generator().manual_seed(seed + 10)
    u = torch.randint(0, n_users, (B,), generator=gen)
    pos = torch.randn(B, 128, 131, generator=gen) * scale
    neg = torch.randn(B, N, 128, 131, generator=gen) * scale
    scores, uf, pf, nf = net(u.to(DEV), pos.to(DEV), neg.to(DEV))
    loss = torch.max(torch.zeros_like(scores), 0.2 - scores).sum(dim=1).mean()
    loss.backward()
    torch.cuda.synchronize()
    p64 = {k: v.double() for k, v in p.items()}
    b64 = {k: (v.double() if v.is_floating_point() else v.clone()) for k, v in b.items()}
    ref_loss, grads, (rs, ruf, rpf, rnf) = O.loss_and_grads(p64, b64, u, pos.double(), neg.double())
    net.eval()
    with torch.no_grad():
        e_got = net(u.to(DEV), pos.to(DEV), neg.to(DEV))
        e_ref = O.forward(p64, b64, u, pos.double(), neg.double(), train=False)
    return net, (scores, uf, pf, nf, loss), (rs, ruf, rpf, rnf, ref_loss), grads, e_got, e_ref


def _close(got, ref, frac, what):
    got = torch.as_tensor(got).detach().double().cpu()
    ref = torch.as_tensor(ref).double()
    assert bool(torch.isfinite(got).all()), "%s: non-finite" % what
    scale = max(float(ref.abs().max()), 1e-300)
    err = float((got - ref).abs().max()) / scale
    assert err <= frac, "%s: %.3e of max" % (what, err)
    return err


@pytest.mark.parametrize("model_type,scale", [
    ("truedcuemel1d", 1e3), ("truedcuemel1d", 1e-3), ("truedcuemel1d", 1e5),
    ("truedcuemel1dres", 1e3), ("truedcuemel1dres", 1e-3),
    ("truedcuemel1dbn", 1e3), ("truedcuemel1dbn", 1e-3)])
def test_split_forward_range_against_fp64_oracle(model_type, scale):
    net, got, ref, grads, e_got, e_ref = _step(model_type, scale)
    for name, a, r in zip(("scores", "user feats", "pos feats", "neg feats", "loss"), got, ref):
        _close(a, r, 1e-4, name)
    for name, a, r in zip(("eval scores", "eval user feats", "eval pos feats", "eval neg feats"), e_got, e_ref):
        _close(a, r, 1e-4, name)
    named = dict(net.named_parameters())
    worst = 0.0
    for k, g_ref in grads.items():
        if k not in named or named[k].grad is None or float(g_ref.abs().max()) == 0.0:
            continue
        worst = max(worst, _close(named[k].grad, g_ref, 1e-3, "grad " + k))
    print("%s x%g: worst gradient error %.2e of max" % (model_type, scale, worst))
