"""DCBR oracle checks on the CPU (BASELINE config 5; parity unpinned against the reference, which
never published DCBR -- oracle/wrmf_oracle.py). The fp64 WRMF half-step must be the exact
minimiser of the objective over the solved side (so ALS never increases it), and the host-side
device CSR builder must agree with the oracle's."""
import numpy as np
import torch

from oracle import wrmf_oracle as W


def _problem(seed=0, n_users=30, n_items=45, nnz=200, d=8):
    rs = np.random.RandomState(seed)
    rows = rs.randint(0, n_users, nnz)
    cols = rs.randint(0, n_items, nnz)
    keys = np.unique(rows * n_items + cols)
    rows, cols = keys // n_items, keys % n_items
    vals = rs.randint(1, 20, len(rows)).astype(np.float64)
    X = rs.randn(n_users, d) * 0.1
    Y = rs.randn(n_items, d) * 0.1
    return rows, cols, vals, X, Y


def test_half_step_minimises_objective():
    rows, cols, vals, X, Y = _problem()
    alpha, lam = 2.0, 0.1
    ip, ix, iv = W.csr(rows, cols, vals, X.shape[0])
    X1 = W.half_step(Y, ip, ix, iv, alpha, lam)
    f0 = W.objective(X, Y, rows, cols, vals, alpha, lam)
    f1 = W.objective(X1, Y, rows, cols, vals, alpha, lam)
    assert f1 <= f0
    # exact minimiser: any perturbation of the solved side increases the objective
    rs = np.random.RandomState(1)
    for _ in range(5):
        assert W.objective(X1 + 1e-3 * rs.randn(*X1.shape), Y, rows, cols, vals, alpha, lam) > f1
    # and ALS alternation is monotone
    ipi, ixi, ivi = W.csr(cols, rows, vals, Y.shape[0])
    Y1 = W.half_step(X1, ipi, ixi, ivi, alpha, lam)
    assert W.objective(X1, Y1, rows, cols, vals, alpha, lam) <= f1


def test_device_csr_matches_oracle():
    from dcrecommend.dcbr.wrmf import device_csr
    rows, cols, vals, X, _ = _problem(seed=3)
    ip, ix, iv = W.csr(rows, cols, vals, X.shape[0])
    dp, dx, dv = device_csr(torch.as_tensor(rows), torch.as_tensor(cols), torch.as_tensor(vals), X.shape[0])
    assert np.array_equal(dp.numpy(), ip)
    assert np.array_equal(dx.numpy().astype(np.int64), ix)
    assert np.allclose(dv.numpy(), iv)


def test_dcbr_mse_oracle_matches_torch_definition():
    from oracle import dcue_oracle as O
    torch.manual_seed(0)
    p, b = O.init_params(8, 16, 4, 2)
    X = torch.randn(5, 128, 131)
    target = torch.randn(5, 8)
    loss, grads, f = W.dcbr_loss_and_grads(p, b, X, target)
    assert torch.allclose(loss, ((f - target) ** 2).mean())
    assert "conv.fc.weight" in grads and "user_embd.linear1.weight" not in grads
