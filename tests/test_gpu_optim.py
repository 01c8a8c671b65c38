"""NativeSGD / NativeRanger (dcue_optimizer_step): the trainer's optimize='sgd' | 'ranger'
(nn/dcue.py:148-157) on the GPU.

Bars:
* on the reference's own fixture (tests/golden/optim.npz: its Ranger and torch.optim.SGD stepped 13
  times on fixed gradients with a changing lr), fed through the model's flat dense buffer: SGD
  bit-exact; Ranger bit-exact with the restatement using a correctly rounded sqrt and within 4 ulp
  of max of the reference (torch's CPU sqrt is not correctly rounded);
* on the user table (dense embedding gradient: rows outside the batch step with g = 0): bit-exact
  against the restatement over the whole table;
* DCUE(optimize=...) trains end to end with each optimizer through the plan.
"""
import numpy as np
import pytest
import torch

from oracle import optim_oracle as A

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _net(n_users=12, E=40):
    from dcrecommend.dcue.dcue import DCUENet
    torch.manual_seed(3)
    return DCUENet({"feature_dim": 32, "conv_hidden": 32, "user_embdim": E, "user_count": n_users,
                    "model_type": "truedcuemel1dbn"}).to(DEV).train()


def _make(kind, net, cfg, lr):
    from dcrecommend.optim import NativeRanger, NativeSGD
    b1, b2, wd = cfg
    if kind == "ranger":
        return NativeRanger(net.parameters(), lr=lr, alpha=0.5, k=6, N_sma_threshhold=5, betas=(b1, b2), eps=1e-5,
                            weight_decay=wd)
    return NativeSGD(net.parameters(), lr, b1, weight_decay=wd, nesterov=True)


@pytest.mark.parametrize("tag", ["ranger_a", "ranger_b", "sgd_a", "sgd_b"])
def test_reference_fixture_through_flat_buffer(golden, tag):
    """The fixture's three tensors are laid into the flat dense buffer (the rest of it and the table
    have zero gradient and start at the model's values); every step's result is compared."""
    g = golden("optim.npz")
    kind = tag.split("_")[0]
    cfg = [float(x) for x in g[tag + ".cfg"]]
    net = _net()
    fl = net._flat
    net._workspace(1, 0, 1)  # compact embedding gradient buffers, no row touched
    sizes = [np.array(g["init.%d" % i]).size for i in range(3)]
    offs = np.cumsum([0] + sizes)
    with torch.no_grad():
        for i in range(3):
            fl["P"][offs[i]:offs[i + 1]] = torch.from_numpy(np.array(g["init.%d" % i]).reshape(-1)).to(DEV)
    opt = _make(kind, net, cfg, float(g["lr"][0]))
    P0 = fl["P"].cpu().numpy().copy()
    slow = P0.copy()
    m = np.zeros_like(P0)
    v = np.zeros_like(P0)
    p_ref = P0.copy()
    for t in range(len(g["lr"])):
        lr = float(g["lr"][t])
        G = np.zeros_like(P0)
        for i in range(3):
            G[offs[i]:offs[i + 1]] = np.array(g["grad.%d.%d" % (t, i)]).reshape(-1)
        fl["G"].copy_(torch.from_numpy(G).to(DEV))
        opt.param_groups[0]["lr"] = lr
        opt.step()
        torch.cuda.synchronize()
        got = fl["P"].cpu().numpy()
        if kind == "ranger":
            p_ref, m, v, slow = A.ranger_elementwise(p_ref, G, m, v, slow, lr, cfg[0], cfg[1], 1e-5, cfg[2], t + 1)
        else:
            p_ref, m = A.sgd_elementwise(p_ref, G, m, lr, cfg[0], cfg[2], t + 1)
        assert np.array_equal(got.view(np.int32), p_ref.view(np.int32)), "step %d: %d elements differ" % (
            t + 1, int((got != p_ref).sum()))
        for i in range(3):
            want = np.array(g["%s.p.%d.%d" % (tag, t, i)]).reshape(-1)
            seg = got[offs[i]:offs[i + 1]]
            if kind == "sgd":
                assert np.array_equal(seg.view(np.int32), want.view(np.int32)), "step %d tensor %d" % (t + 1, i)
            else:
                assert np.abs(seg - want).max() <= 4 * np.spacing(np.abs(want).max()), "step %d tensor %d" % (t + 1, i)


@pytest.mark.parametrize("kind", ["ranger", "sgd"])
def test_user_table_dense_sweep(kind):
    """Batch rows step with their gradient, every other row with g = 0, over 8 steps (two lookahead
    syncs' worth for k = 6 is not needed: one sync at step 6)."""
    from dcrecommend import _native as nat
    net = _net(n_users=30)
    cfg = (0.9, 0.99, 1e-2)
    opt = _make(kind, net, cfg, 1e-3)
    gen = torch.Generator(device=DEV).manual_seed(5)
    tracks = torch.randn((40, 131, 128), generator=gen, device=DEV).half()
    emb = net.user_embd.embeddings.weight
    E0 = emb.detach().cpu().numpy().copy()
    m, v, slow = np.zeros_like(E0), np.zeros_like(E0), E0.copy()
    ref = E0.copy()
    for t in range(1, 9):
        users = torch.randint(0, 30, (8,), generator=gen, device=DEV)
        items = torch.randint(0, 40, (32,), generator=gen, device=DEV).to(torch.int32)
        net.native_forward(users, tracks, items, 3, nat.LAYOUT_CATALOGUE, None, train=True)
        net.native_backward(None)
        EG = net.embedding_grad_dense().cpu().numpy()
        opt.step()
        torch.cuda.synchronize()
        if kind == "ranger":
            ref, m, v, slow = A.ranger_elementwise(ref, EG, m, v, slow, 1e-3, cfg[0], cfg[1], 1e-5, cfg[2], t)
        else:
            ref, m = A.sgd_elementwise(ref, EG, m, 1e-3, cfg[0], cfg[2], t)
        got = emb.detach().cpu().numpy()
        assert np.array_equal(got.view(np.int32), ref.view(np.int32)), "step %d: %d elements differ" % (
            t, int((got != ref).sum()))


@pytest.mark.parametrize("optimize", ["ranger", "sgd"])
def test_trainer_fit_with_optimizer(tmp_path, optimize):
    import train_dcue
    dcue = train_dcue.main(["--synthetic", "--synthetic-users", "24", "--synthetic-tracks", "80",
                            "--synthetic-pairs", "300", "--feature-dim", "32", "--conv-hidden", "32",
                            "--batch-size", "8", "--neg-batch-size", "3", "--num-epochs", "1",
                            "--eval-pct", "1.0", "--lr", "1e-3", "--optimize", optimize,
                            "--save-dir", str(tmp_path)])
    assert dcue.nn_epoch >= 9 and 0.0 <= dcue.best_val_auc <= 1.0
    assert np.isfinite(dcue.best_val_loss)
