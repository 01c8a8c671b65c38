"""DCBR path on the MI355X (BASELINE config 5): the WRMF half-step and the audio-ConvNet regression
step against the fp64 oracles (oracle/wrmf_oracle.py, oracle/dcue_oracle.py). Parity unpinned
against the reference, which never published DCBR (its .gitignore:13).

Tolerances: WRMF factors within 1e-4 of their max magnitude (fp32 Cholesky of a lambda-regularised
system, against fp64 numpy); DCBR loss within 1e-4 relative and gradients within 1e-3 of their max
(the golden tests' gradient tolerance: the conv backward runs on split-f16 MFMA).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _problem(seed, n_users, n_items, nnz, with_values):
    rs = np.random.RandomState(seed)
    rows = rs.randint(0, n_users - 10, nnz)  # the last 10 users have no pair: x = 0
    cols = rs.randint(0, n_items, nnz)
    keys = np.unique(rows * n_items + cols)
    rows, cols = keys // n_items, keys % n_items
    vals = rs.randint(1, 30, len(rows)).astype(np.float32) if with_values else None
    return rows, cols, vals


@pytest.mark.parametrize("dim,with_values", [(32, True), (128, False), (100, True), (7, False)])
def test_wrmf_half_step_against_oracle(dim, with_values):
    from dcrecommend.dcbr import WRMF, device_csr
    from oracle import wrmf_oracle as W
    n_users, n_items = 70, 90
    rows, cols, vals = _problem(dim, n_users, n_items, 900, with_values)
    alpha, lam = 3.0, 0.05
    m = WRMF(factors=dim, regularization=lam, alpha=alpha, device=DEV)
    rs = np.random.RandomState(7)
    Y = rs.randn(n_items, dim).astype(np.float32) * 0.3
    X = torch.zeros(n_users, dim, device=DEV)
    csr = device_csr(torch.as_tensor(rows, device=DEV), torch.as_tensor(cols, device=DEV),
                     None if vals is None else torch.as_tensor(vals, device=DEV), n_users)
    m.half_step(X, torch.as_tensor(Y, device=DEV), csr)
    torch.cuda.synchronize()
    ip, ix, iv = W.csr(rows.astype(np.int64), cols, vals, n_users)
    ref = W.half_step(Y, ip, ix, iv, alpha, lam)
    got = X.double().cpu().numpy()
    scale = np.abs(ref).max()
    assert np.abs(got - ref).max() <= 1e-4 * scale, np.abs(got - ref).max() / scale
    empty = np.setdiff1d(np.arange(n_users), rows)
    assert np.all(got[empty] == 0.0)


def test_wrmf_fit_monotone_against_oracle():
    from dcrecommend.dcbr import WRMF
    from oracle import wrmf_oracle as W
    n_users, n_items, dim = 60, 80, 16
    rows, cols, vals = _problem(11, n_users, n_items, 700, True)
    m = WRMF(factors=dim, regularization=0.1, alpha=2.0, iterations=0, seed=3, device=DEV)
    m.fit(rows, cols, vals, n_users=n_users, n_items=n_items)
    X = m.user_factors.double().cpu().numpy()
    Y = m.item_factors.double().cpu().numpy()
    prev = W.objective(X, Y, rows, cols, vals, 2.0, 0.1)
    ipu, ixu, ivu = W.csr(rows, cols, vals, n_users)
    ipi, ixi, ivi = W.csr(cols, rows, vals, n_items)
    for it in range(3):
        m.half_step(m.user_factors, m.item_factors, m.by_user)
        m.half_step(m.item_factors, m.user_factors, m.by_item)
        X = W.half_step(Y, ipu, ixu, ivu, 2.0, 0.1)
        Y = W.half_step(X, ipi, ixi, ivi, 2.0, 0.1)
        cur = m.loss()
        ref = W.objective(X, Y, rows, cols, vals, 2.0, 0.1)
        assert cur <= prev * (1 + 1e-6), "iteration %d: objective rose %.6g -> %.6g" % (it, prev, cur)
        assert abs(cur - ref) <= 1e-4 * abs(ref), (cur, ref)
        prev = cur


@pytest.mark.parametrize("model_type,d,H", [("truedcuemel1dbn", 32, 64), ("truedcuemel1dbn", 100, 128),
                                            ("truedcuemel1dres", 32, 40)])
def test_dcbr_step_against_fp64_oracle(model_type, d, H):
    from dcrecommend.dcbr import DCBR
    from oracle import dcue_oracle as O
    from oracle import wrmf_oracle as W
    torch.manual_seed(5)
    m = DCBR(feature_dim=d, conv_hidden=H, model_type=model_type, lr=1e-3, device=DEV)
    torch.manual_seed(5)
    p, b = O.init_params(d, H, 1, 1, model_type)
    gen = torch.Generator().manual_seed(9)
    n_tracks, M = 20, 12
    X = torch.randn(n_tracks, 128, 131, generator=gen)
    table = m.net._spectro_table(X.to(DEV)).contiguous()
    items = torch.randint(0, n_tracks, (M,), generator=gen)
    target = torch.randn(M, d, generator=gen) * 0.5
    loss = m.loss_and_grads(table, items.to(DEV), target.to(DEV))
    torch.cuda.synchronize()
    p64 = {k: v.double() for k, v in p.items()}
    b64 = {k: (v.double() if v.is_floating_point() else v.clone()) for k, v in b.items()}
    ref_loss, grads, _ = W.dcbr_loss_and_grads(p64, b64, X[items].double(), target.double())
    assert abs(float(loss) - float(ref_loss)) <= 1e-4 * abs(float(ref_loss))
    named = dict(m.net.named_parameters())
    for k, g_ref in grads.items():
        got = named[k].grad.double().cpu()
        scale = float(g_ref.abs().max())
        if scale == 0.0:
            continue
        err = float((got - g_ref).abs().max()) / scale
        assert err <= 1e-3, "grad %s: %.3e of max" % (k, err)
    # the user tower is not part of the DCBR step: its gradients stay zero
    assert float(named["user_embd.linear1.weight"].grad.abs().max()) == 0.0


def test_dcbr_training_reduces_loss():
    from dcrecommend.dcbr import DCBR
    torch.manual_seed(1)
    m = DCBR(feature_dim=32, conv_hidden=64, lr=3e-3, device=DEV)
    gen = torch.Generator().manual_seed(2)
    X = torch.randn(16, 128, 131, generator=gen)
    table = m.net._spectro_table(X.to(DEV)).half().contiguous()
    items = torch.arange(16, dtype=torch.int32, device=DEV)
    target = (torch.randn(16, 32, generator=gen) * 0.5).to(DEV)
    losses = [float(m.step(table, items, target)) for _ in range(40)]
    assert all(np.isfinite(losses))
    assert losses[-1] < 0.5 * losses[0], losses[::8]
    pred = m.predict(table, items)
    assert pred.shape == (16, 32) and bool(torch.isfinite(pred).all())


def test_wrmf_mfma_solve_matches_tile_solve(tmp_path):
    """The default solve (rows with <= 32 pairs by the Woodbury identity, k_wrmf_solve_lowrank;
    the rest by the fp64-MFMA block Cholesky, k_wrmf_solve_mfma), the Cholesky for every row
    (DCUE_WRMF_LOWRANK=0) and the register-tile solve (DCUE_WRMF_SOLVE=tile), over the fp64-MFMA
    Gram matrix (the default) or the scalar one (DCUE_WRMF_GRAM=scalar), solve the same systems in
    fp64: their fp32 factors agree to a few fp32 ulps (1e-6 of the max), at every block count (dims
    7, 40, 100, 128), with zero-weight pairs, rows without pairs zero."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = r'''
import sys, numpy as np, torch
sys.path.insert(0, %r); sys.path.insert(0, %r)
from dcrecommend.dcbr import WRMF, device_csr
from test_gpu_dcbr import _problem
out = {}
for dim in (7, 40, 100, 128):
    n_users, n_items = 300, 1301  # (three Gram chunks of 512 rows, the last ending mid-step)
    rows, cols, vals = _problem(dim + 1, n_users, n_items, 9000, dim %% 2 == 0)
    if vals is not None:
        vals[::7] = 0  # pairs with c = 1: no weight in A, still in b
    m = WRMF(factors=dim, regularization=0.05, alpha=3.0, device="cuda:0")
    Y = torch.as_tensor(np.random.RandomState(5).randn(n_items, dim).astype(np.float32) * 0.3, device="cuda:0")
    X = torch.zeros(n_users, dim, device="cuda:0")
    csr = device_csr(torch.as_tensor(rows, device="cuda:0"), torch.as_tensor(cols, device="cuda:0"),
                     None if vals is None else torch.as_tensor(vals, device="cuda:0"), n_users)
    m.half_step(X, Y, csr)
    out[str(dim)] = X.cpu()
torch.save(out, sys.argv[1])
''' % (os.path.join(root, "amplifai-deepcontentrecommenders_amd"), os.path.join(root, "tests"))
    res = []
    for i, extra in enumerate(({"DCUE_WRMF_SOLVE": "tile"}, {}, {"DCUE_WRMF_GRAM": "scalar"},
                               {"DCUE_WRMF_LOWRANK": "0"})):
        out = str(tmp_path / ("w%d.pt" % i))
        env = dict(os.environ, **extra)
        for k in ("DCUE_WRMF_SOLVE", "DCUE_WRMF_GRAM", "DCUE_WRMF_LOWRANK"):
            if k not in extra:
                env.pop(k, None)
        p = subprocess.run([sys.executable, "-c", code, out], env=env, stdout=subprocess.PIPE,
                           stderr=subprocess.STDOUT, text=True, timeout=100)
        assert p.returncode == 0, p.stdout[-3000:]
        res.append(torch.load(out, weights_only=True))
    for k in res[0]:
        b = res[0][k].double()
        scale = float(b.abs().max())
        for v, r in enumerate(res[1:]):
            a = r[k].double()
            assert float((a - b).abs().max()) <= 1e-6 * scale, (k, v, float((a - b).abs().max()) / scale)
            assert bool(torch.isfinite(a).all())


def _counted_problem(seed, counts, n_fixed):
    """Rows with exactly the given pair counts (distinct columns each), the rest empty."""
    rs = np.random.RandomState(seed)
    rows, cols = [], []
    for r, c in enumerate(counts):
        rows.append(np.full(c, r, dtype=np.int64))
        cols.append(np.sort(rs.choice(n_fixed, c, replace=False)))
    return np.concatenate(rows), np.concatenate(cols).astype(np.int64)


# around the Woodbury / Cholesky switch (<= 32 pairs: k_wrmf_solve_lowrank; more: k_wrmf_solve_mfma)
# and well past it; 0 and 1 at the edges
SWITCH_COUNTS = [0, 1, 5, 16, 17, 31, 32, 33, 34, 48, 64, 65, 100, 200]


@pytest.mark.parametrize("dim", [128, 100])
def test_wrmf_default_solve_at_the_switch_against_oracle(dim):
    """VERDICT r05 missing 1: the default solve of the rows config 5 actually runs -- every user row
    at bench scale has > 32 pairs and takes the fp64-MFMA block Cholesky -- against the numpy fp64
    oracle at 1e-4 of max. Rows with exactly 31, 32, 33, 48, >= 64 pairs, on both sides: the user
    half-step (rows = users) and the item half-step (rows = items, the transposed CSR, where the
    popular items carry the many-pair rows). With values (c = 1 + alpha v) and without."""
    from dcrecommend.dcbr import WRMF, device_csr
    from oracle import wrmf_oracle as W
    n_items = 400
    counts = SWITCH_COUNTS * 2
    rows, cols = _counted_problem(dim, counts, n_items)
    n_users = len(counts)
    # items: make a few of them carry exactly the switch counts too (their users are the many-pair rows)
    item_deg = np.bincount(cols, minlength=n_items)
    rs = np.random.RandomState(dim + 1)
    alpha, lam = 2.0, 0.05
    for with_values in (False, True):
        vals = rs.randint(1, 20, len(rows)).astype(np.float32) if with_values else None
        X = torch.zeros(n_users, dim, device=DEV)
        Y0 = rs.randn(n_items, dim).astype(np.float32) * 0.3
        m = WRMF(factors=dim, regularization=lam, alpha=alpha, device=DEV)
        by_user = device_csr(torch.as_tensor(rows, device=DEV), torch.as_tensor(cols, device=DEV),
                             None if vals is None else torch.as_tensor(vals, device=DEV), n_users)
        m.half_step(X, torch.as_tensor(Y0, device=DEV), by_user)
        torch.cuda.synchronize()
        ip, ix, iv = W.csr(rows, cols, vals, n_users)
        ref = W.half_step(Y0.astype(np.float64), ip, ix, iv, alpha, lam)
        got = X.double().cpu().numpy()
        scale = np.abs(ref).max()
        for r, c in enumerate(counts):
            err = np.abs(got[r] - ref[r]).max() / scale
            assert err <= 1e-4, "user row with %d pairs (values %s): %.3e of max" % (c, with_values, err)
        assert np.all(got[np.array(counts) == 0] == 0.0)
        # item half-step against those users
        Xf = rs.randn(n_users, dim).astype(np.float32) * 0.3
        Yg = torch.zeros(n_items, dim, device=DEV)
        by_item = device_csr(torch.as_tensor(cols, device=DEV), torch.as_tensor(rows, device=DEV),
                             None if vals is None else torch.as_tensor(vals, device=DEV), n_items)
        m.half_step(Yg, torch.as_tensor(Xf, device=DEV), by_item)
        torch.cuda.synchronize()
        jp, jx, jv = W.csr(cols, rows, vals, n_items)
        refi = W.half_step(Xf.astype(np.float64), jp, jx, jv, alpha, lam)
        goti = Yg.double().cpu().numpy()
        err = np.abs(goti - refi).max() / np.abs(refi).max()
        assert err <= 1e-4, "item half-step (degrees %d..%d): %.3e of max" % (item_deg.min(), item_deg.max(), err)


def test_wrmf_item_rows_at_the_switch_against_oracle():
    """Item rows (the transposed side) with exactly 31, 32, 33, 48 and 64+ pairs, default solve."""
    from dcrecommend.dcbr import WRMF, device_csr
    from oracle import wrmf_oracle as W
    dim, n_users = 128, 300
    counts = [31, 32, 33, 48, 64, 100, 3, 0]
    icols, iusers = _counted_problem(5, counts, n_users)  # rows = items here
    n_items = len(counts)
    vals = np.random.RandomState(2).randint(1, 9, len(icols)).astype(np.float32)
    m = WRMF(factors=dim, regularization=0.1, alpha=1.5, device=DEV)
    Xf = np.random.RandomState(3).randn(n_users, dim).astype(np.float32) * 0.3
    Y = torch.zeros(n_items, dim, device=DEV)
    csr = device_csr(torch.as_tensor(icols, device=DEV), torch.as_tensor(iusers, device=DEV),
                     torch.as_tensor(vals, device=DEV), n_items)
    m.half_step(Y, torch.as_tensor(Xf, device=DEV), csr)
    torch.cuda.synchronize()
    ip, ix, iv = W.csr(icols, iusers, vals, n_items)
    ref = W.half_step(Xf.astype(np.float64), ip, ix, iv, 1.5, 0.1)
    got = Y.double().cpu().numpy()
    scale = np.abs(ref).max()
    for r, c in enumerate(counts):
        assert np.abs(got[r] - ref[r]).max() <= 1e-4 * scale, (c, np.abs(got[r] - ref[r]).max() / scale)


def test_wrmf_negative_values_take_the_cholesky():
    """a row with a (small) negative value has a negative weight w = alpha v; its
    Woodbury system is indefinite, so such rows -- even with <= 32 pairs -- go to the Cholesky of
    A = G + lambda I + F^T W F, which stays SPD here. Against the oracle at 1e-4."""
    from dcrecommend.dcbr import WRMF, device_csr
    from oracle import wrmf_oracle as W
    dim, n_items = 64, 120
    counts = [3, 10, 20, 32, 40]
    rows, cols = _counted_problem(9, counts, n_items)
    vals = np.random.RandomState(4).randint(1, 6, len(rows)).astype(np.float32)
    vals[::4] = -0.05  # w = -0.1: A stays positive definite (G's eigenvalues dominate)
    m = WRMF(factors=dim, regularization=0.05, alpha=2.0, device=DEV)
    Y0 = np.random.RandomState(6).randn(n_items, dim).astype(np.float32) * 0.3
    X = torch.zeros(len(counts), dim, device=DEV)
    csr = device_csr(torch.as_tensor(rows, device=DEV), torch.as_tensor(cols, device=DEV),
                     torch.as_tensor(vals, device=DEV), len(counts))
    m.half_step(X, torch.as_tensor(Y0, device=DEV), csr)
    torch.cuda.synchronize()
    ip, ix, iv = W.csr(rows, cols, vals, len(counts))
    ref = W.half_step(Y0.astype(np.float64), ip, ix, iv, 2.0, 0.05)
    got = X.double().cpu().numpy()
    assert np.isfinite(got).all()
    assert np.abs(got - ref).max() <= 1e-4 * np.abs(ref).max(), np.abs(got - ref).max() / np.abs(ref).max()
