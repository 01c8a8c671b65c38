"""Pins oracle/optim_oracle.py -- the per-element restatement NativeAdam implements -- against the
reference's optimizer itself: torch.optim.Adam (nn/dcue.py:143-147, foreach=False, CPU float32).

Bar: BIT-EXACT over several steps, with and without weight decay, for both lerp branches, when the
restatement uses torch's own CPU sqrt. With a correctly rounded sqrt (what the GPU computes) the
only differences left are the elements where torch's vectorised sqrt is off by one ulp.
"""
import numpy as np
import pytest
import torch

from oracle import optim_oracle as A


def _inputs(n, steps, seed):
    rng = np.random.default_rng(seed)
    p0 = (rng.standard_normal(n) * 0.1).astype(np.float32)
    # gradients over 8 decades, signed zeros and exact zeros included
    gs = [(rng.standard_normal(n) * 10.0 ** rng.uniform(-8, 0, n)).astype(np.float32) for _ in range(steps)]
    for g in gs:
        g[::97] = 0.0
        g[1::193] = -0.0
    return p0, gs


@pytest.mark.parametrize("lr,betas,wd", [(1e-5, (0.9, 0.99), 0.0), (1e-3, (0.9, 0.999), 1e-4),
                                         (3e-4, (0.3, 0.99), 1e-2), (3e-4, (0.3, 0.99), 0.0),
                                         (1e-3, (0.0, 0.99), 0.0), (1e-3, (0.5, 0.99), 0.0)])
def test_restatement_matches_torch_adam_bit_exact(lr, betas, wd):
    n, steps = 40_003, 4
    p0, gs = _inputs(n, steps, 1)
    tp = torch.tensor(p0.copy()).requires_grad_(True)
    opt = torch.optim.Adam([tp], lr=lr, betas=betas, eps=1e-8, weight_decay=wd, foreach=False)
    p, m, v = p0.copy(), np.zeros(n, np.float32), np.zeros(n, np.float32)
    ulp_off = 0
    pe, me, ve = p.copy(), m.copy(), v.copy()
    for t, g in enumerate(gs, 1):
        tp.grad = torch.from_numpy(g.copy())
        opt.step()
        p, m, v = A.adam_elementwise(p, g, m, v, lr, betas[0], betas[1], 1e-8, wd, t, sqrt=A.torch_cpu_sqrt)
        want = tp.detach().numpy()
        st = opt.state[tp]
        assert np.array_equal(p.view(np.int32), want.view(np.int32)), "step %d: param differs" % t
        assert np.array_equal(m.view(np.int32), st["exp_avg"].numpy().view(np.int32)), "step %d: exp_avg" % t
        assert np.array_equal(v.view(np.int32), st["exp_avg_sq"].numpy().view(np.int32)), "step %d: exp_avg_sq" % t
        pe, me, ve = A.adam_elementwise(pe, g, me, ve, lr, betas[0], betas[1], 1e-8, wd, t)
        ulp_off = int((pe != want).sum())
    # the exact-sqrt form drifts only where torch's sqrt rounds the other way
    assert ulp_off < 0.05 * n


def test_torch_cpu_sqrt_is_not_correctly_rounded():
    """Why the GPU cannot be bit-exact with the CPU reference: its sqrt is not IEEE on this host."""
    x = np.abs(np.random.default_rng(2).standard_normal(100_000)).astype(np.float32)
    diff = A.torch_cpu_sqrt(x) != A.exact_sqrt(x)
    ulps = np.abs(A.torch_cpu_sqrt(x).view(np.int32)[diff] - A.exact_sqrt(x).view(np.int32)[diff])
    assert ulps.size == 0 or ulps.max() == 1


def _optim_case(g, tag, kind):
    steps, n_par = len(g["lr"]), 3
    beta_a, beta_b, wd = (float(x) for x in g[tag + ".cfg"])
    ps = [np.array(g["init.%d" % i]).reshape(-1) for i in range(n_par)]
    state = [dict(m=np.zeros_like(p), v=np.zeros_like(p), slow=p.copy(), buf=np.zeros_like(p)) for p in ps]
    for t in range(steps):
        lr = float(g["lr"][t])
        for i in range(n_par):
            grad = np.array(g["grad.%d.%d" % (t, i)]).reshape(-1)
            st = state[i]
            if kind == "ranger":
                ps[i], st["m"], st["v"], st["slow"] = A.ranger_elementwise(
                    ps[i], grad, st["m"], st["v"], st["slow"], lr, beta_a, beta_b, 1e-5, wd, t + 1, sqrt=A.torch_cpu_sqrt)
            else:
                ps[i], st["buf"] = A.sgd_elementwise(ps[i], grad, st["buf"], lr, beta_a, wd, t + 1)
            want = np.array(g["%s.p.%d.%d" % (tag, t, i)]).reshape(-1)
            assert np.array_equal(ps[i].view(np.int32), want.view(np.int32)), "%s step %d param %d" % (tag, t + 1, i)


@pytest.mark.parametrize("tag", ["ranger_a", "ranger_b"])
def test_ranger_restatement_matches_reference(golden, tag):
    """oracle ranger_elementwise == the reference's Ranger (optim/ranger.py), bit for bit, over 13
    steps: the un-rectified first steps, the RAdam steps, two lookahead syncs (k = 6)."""
    _optim_case(golden("optim.npz"), tag, "ranger")


@pytest.mark.parametrize("tag", ["sgd_a", "sgd_b"])
def test_sgd_restatement_matches_torch(golden, tag):
    """oracle sgd_elementwise == torch.optim.SGD(momentum, nesterov=True) as the trainer builds it."""
    _optim_case(golden("optim.npz"), tag, "sgd")
