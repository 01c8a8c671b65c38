"""NativeAdam (dcue_adam_step) against torch.optim.Adam's per-element arithmetic on IDENTICAL
gradients, isolating the optimizer from gradient rounding.

oracle/optim_oracle.py restates torch 2.10's CPU Adam kernels op by op; tests/test_adam_cpu.py pins
it bit for bit against torch.optim.Adam itself (nn/dcue.py:143-147). The GPU computes the same
operations with a correctly rounded sqrt, so the bar here is BIT-EXACT against the restatement with
the exact sqrt -- for the dense buffer and for every user-table row (touched or not), in the dense
sweep and in the deferred replay, with and without weight decay -- and, against torch.optim.Adam
on CPU, equality everywhere except where torch's sqrt is one ulp off.
"""
import numpy as np
import pytest
import torch

from oracle import optim_oracle as A

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _snapshot(net, opt):
    fl = net._flat
    st = opt._adam_state()
    net.sync_user_table()
    return dict(P=fl["P"].cpu().numpy().copy(), G=fl["G"].cpu().numpy().copy(),
                m=st["m"].cpu().numpy().copy(), v=st["v"].cpu().numpy().copy(),
                E=net.user_embd.embeddings.weight.detach().cpu().numpy().copy(),
                EG=net.embedding_grad_dense().cpu().numpy().copy(),
                em=st["em"].cpu().numpy().copy(), ev=st["ev"].cpu().numpy().copy())


@pytest.mark.parametrize("defer,wd,betas", [(False, 0.0, (0.9, 0.99)), (True, 0.0, (0.9, 0.99)),
                                            (False, 1e-3, (0.9, 0.999)), (True, 1e-3, (0.3, 0.99)),
                                            # beta1 <= 0.5: the lerp's base is g (0: weight 1, m = g);
                                            # the deferred replay's zero-gradient steps must follow it
                                            (True, 0.0, (0.3, 0.99)), (True, 0.0, (0.0, 0.99)),
                                            (False, 0.0, (0.0, 0.99)), (True, 0.0, (0.5, 0.99))])
def test_native_adam_bit_exact_with_restatement(defer, wd, betas):
    from dcrecommend import _native as nat
    from dcrecommend.dcue.dcue import DCUENet
    from dcrecommend.optim import NativeAdam
    n_users, B, N, n_tracks, E = 30, 8, 3, 40, 40
    torch.manual_seed(2)
    net = DCUENet({"feature_dim": 32, "conv_hidden": 32, "user_embdim": E, "user_count": n_users,
                   "model_type": "truedcuemel1dbn"}).cuda().train()
    opt = NativeAdam(net.parameters(), 1e-3, betas, 1e-8, wd, defer_embedding=defer, flush_every=4)
    gen = torch.Generator(device=DEV).manual_seed(9)
    tracks = torch.randn((n_tracks, 131, 128), generator=gen, device=DEV).half()
    lrs = [1e-3, 7e-4, 2e-3, 1e-4, 5e-4, 1e-3]
    torch_p = None
    for t, lr in enumerate(lrs, 1):
        users = torch.randint(0, n_users, (B,), generator=gen, device=DEV)
        items = torch.randint(0, n_tracks, (B * (1 + N),), generator=gen, device=DEV,
                              dtype=torch.int64).to(torch.int32)
        net.native_forward(users, tracks, items, N, nat.LAYOUT_CATALOGUE, None, train=True, margin=0.2)
        net.native_backward(None)
        s0 = _snapshot(net, opt)
        opt.param_groups[0]["lr"] = lr
        opt.step()
        torch.cuda.synchronize()
        s1 = _snapshot(net, opt)
        # the dense flat buffer: every element's update, bit for bit
        p, m, v = A.adam_elementwise(s0["P"], s0["G"], s0["m"], s0["v"], lr, betas[0], betas[1], 1e-8, wd, t)
        for name, got, want in (("params", s1["P"], p), ("exp_avg", s1["m"], m), ("exp_avg_sq", s1["v"], v)):
            bad = int((got.view(np.int32) != want.view(np.int32)).sum())
            assert bad == 0, "step %d dense %s: %d elements differ" % (t, name, bad)
        # the user table: the batch's rows with their gradient, every other row with g = 0
        p, m, v = A.adam_elementwise(s0["E"], s0["EG"], s0["em"], s0["ev"], lr, betas[0], betas[1], 1e-8, wd, t)
        for name, got, want in (("table", s1["E"], p), ("exp_avg", s1["em"], m), ("exp_avg_sq", s1["ev"], v)):
            bad = int((got.view(np.int32) != want.view(np.int32)).sum())
            assert bad == 0, "step %d user %s: %d elements differ" % (t, name, bad)
        # torch.optim.Adam itself, on the same gradients (CPU): equal but for its sqrt's ulps
        if torch_p is None:
            torch_p = torch.tensor(s0["P"]).requires_grad_(True)
            topt = torch.optim.Adam([torch_p], lr=lr, betas=betas, eps=1e-8, weight_decay=wd, foreach=False)
        topt.param_groups[0]["lr"] = lr
        torch_p.grad = torch.from_numpy(s0["G"])
        topt.step()
        close = np.abs(torch_p.detach().numpy() - s1["P"]) <= 1e-6 * np.abs(s1["P"]) + 1e-12
        assert close.mean() > 0.999 and np.allclose(torch_p.detach().numpy(), s1["P"], rtol=1e-4, atol=1e-7)
