"""ORACLE -- numpy fp64 restatement of the DCBR path.  TEST INFRASTRUCTURE ONLY.

Only tests/ may import this module, as the checker of dcue_wrmf_half_step / dcue_dcbr_step. The
product path (amplifai-deepcontentrecommenders_amd/) never imports it.

The reference never published DCBR (`dcrecommend/dcbr` is git-ignored: reference `.gitignore:13`;
`nn/dcue_orig.py:35` imports it and fails), so there is nothing of the reference to pin against:
PARITY UNPINNED against the reference. This restates the published algorithms:

* WRMF / implicit ALS, Hu, Koren, Volinsky, "Collaborative Filtering for Implicit Feedback
  Datasets" (ICDM 2008), eqs. (3)-(4): c_ui = 1 + alpha r_ui, p_ui = [r_ui > 0],
  x_u = (Y^T C^u Y + lambda I)^{-1} Y^T C^u p(u), and the same for items with X fixed.
* DCBR's regression objective, van den Oord, Dieleman, Schrauwen, "Deep content-based music
  recommendation" (NIPS 2013), sec. 4: the mean squared error between the ConvNet's output and the
  item's latent factors (torch.nn.MSELoss 'mean' over all entries).
"""
import numpy as np
import torch


def half_step(fixed, indptr, indices, values, alpha, lam):
    """fp64 WRMF half-step: X[r] for every row r of the CSR (indptr, indices, values or None)."""
    F = np.asarray(fixed, dtype=np.float64)
    n_rows = len(indptr) - 1
    d = F.shape[1]
    G = F.T @ F
    X = np.zeros((n_rows, d))
    for r in range(n_rows):
        p0, p1 = int(indptr[r]), int(indptr[r + 1])
        if p1 <= p0:
            continue
        cols = np.asarray(indices[p0:p1], dtype=np.int64)
        v = np.ones(p1 - p0) if values is None else np.asarray(values[p0:p1], dtype=np.float64)
        c = 1.0 + alpha * v
        Fr = F[cols]
        A = G + (Fr * (c - 1.0)[:, None]).T @ Fr + lam * np.eye(d)
        b = (Fr * c[:, None]).sum(0)
        X[r] = np.linalg.solve(A, b)
    return X


def objective(X, Y, rows, cols, values, alpha, lam):
    """sum_{u,i} c_ui (p_ui - x_u . y_i)^2 + lam (|X|^2 + |Y|^2), fp64, dense."""
    X = np.asarray(X, dtype=np.float64)
    Y = np.asarray(Y, dtype=np.float64)
    S = X @ Y.T
    C = np.ones_like(S)
    P = np.zeros_like(S)
    v = np.ones(len(rows)) if values is None else np.asarray(values, dtype=np.float64)
    C[rows, cols] = 1.0 + alpha * v
    P[rows, cols] = 1.0
    return float((C * (P - S) ** 2).sum() + lam * ((X ** 2).sum() + (Y ** 2).sum()))


def csr(rows, cols, values, n_rows):
    order = np.argsort(rows, kind="stable")
    indptr = np.zeros(n_rows + 1, dtype=np.int64)
    np.add.at(indptr, np.asarray(rows) + 1, 1)
    indptr = np.cumsum(indptr)
    return indptr, np.asarray(cols)[order], None if values is None else np.asarray(values)[order]


def dcbr_loss_and_grads(p, b, X, target):
    """MSE(item_tower(X), target) and its gradients w.r.t. every item-tower parameter (torch autograd
    over oracle/dcue_oracle.py's item tower, in the dtype of p)."""
    from oracle import dcue_oracle as O
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in p.items()}
    f = O.item_tower(leaves, b, X, train=True)
    loss = torch.nn.functional.mse_loss(f, target)
    loss.backward()
    grads = {k: v.grad.detach().clone() for k, v in leaves.items() if v.grad is not None}
    return loss.detach(), grads, f.detach()
