"""WRMF target factors on the MI355X (BASELINE config 5, the DCBR path).

The reference never published its DCBR package (`dcrecommend/dcbr` is git-ignored, reference
`.gitignore:13`; `nn/dcue_orig.py:35` imports it and fails), so this follows the paper it names:
weighted regularized matrix factorisation for implicit feedback (Hu, Koren, Volinsky, ICDM 2008).
Parity is unpinned against the reference; `oracle/wrmf_oracle.py` (numpy fp64) pins the GPU solver.

Every ALS half-step is one call of `dcue_wrmf_half_step` (csrc/wrmf.hip): the Gram matrix of the
fixed side once, then one workgroup per row builds G + sum (c - 1) f f^T + lambda I in LDS and
solves it by Cholesky. Interactions stay on the device as two CSRs (by user, by item).
"""
import ctypes

import torch

from dcrecommend import _native as nat


def device_csr(rows, cols, vals, n_rows):
    """(indptr int64 [n_rows + 1], indices int32, values fp32 or None), rows sorted, on rows' device."""
    rows = rows.to(torch.int64)
    order = torch.argsort(rows, stable=True)
    counts = torch.bincount(rows, minlength=n_rows)
    indptr = torch.zeros(n_rows + 1, dtype=torch.int64, device=rows.device)
    indptr[1:] = torch.cumsum(counts, 0)
    indices = cols[order].to(torch.int32).contiguous()
    values = None if vals is None else vals[order].to(torch.float32).contiguous()
    return indptr, indices, values


class WRMF:
    """Implicit-feedback ALS: confidence c = 1 + alpha * v on the observed pairs (v = play counts,
    or 1), preference 1 there and 0 elsewhere, L2 weight `regularization` on both factor sets.

    `fit(user_idx, item_idx, values=None)` runs `iterations` sweeps (users, then items) and leaves
    `user_factors` [n_users, factors] and `item_factors` [n_items, factors] on the device.

    Data parallelism (comm: a distributed.NativeComm / HostComm): every rank holds the whole
    interaction set and both factor matrices; a half-step solves this rank's contiguous 1/world of
    the rows (rows are independent, so each is solved exactly as on one GPU) and an in-place
    all-gather (dcue_comm_allgather) hands every rank all of them before the next half-step. The
    factor matrices are kept padded to a multiple of world rows (the pad rows have no pairs: 0)."""

    def __init__(self, factors=128, regularization=0.01, alpha=40.0, iterations=15, seed=0, device="cuda",
                 comm=None):
        if not 1 <= int(factors) <= 128:
            raise ValueError("factors must be in [1, 128] (the per-row solve holds a factors^2 matrix in LDS)")
        if not regularization > 0:
            raise ValueError("regularization must be > 0")
        self.factors, self.regularization, self.alpha = int(factors), float(regularization), float(alpha)
        self.iterations, self.seed, self.device = int(iterations), int(seed), torch.device(device)
        self.user_factors = self.item_factors = None
        self._ws = None
        self.comm = comm
        self.world = comm.world if comm is not None else 1
        self.rank = comm.rank if comm is not None else 0
        self._uf = self._if = None  # the padded storage behind user_factors / item_factors

    def _workspace(self, n_fixed):
        nbytes = ctypes.c_size_t()
        nat.check(nat.lib().dcue_wrmf_workspace_bytes(self.factors, int(n_fixed), ctypes.byref(nbytes)),
                  "dcue_wrmf_workspace_bytes")
        if self._ws is None or self._ws.numel() < nbytes.value:
            self._ws = torch.empty(nbytes.value, dtype=torch.uint8, device=self.device)
        return self._ws

    def half_step(self, solve, fixed, csr):
        """solve[r] <- the WRMF least-squares solution of row r with `fixed` held (in place). Under a
        communicator, `solve` is a view of padded storage (user_factors / item_factors): this rank
        solves its part of the rows, then every rank gathers the others'."""
        indptr, indices, values = csr
        if indptr.numel() != solve.shape[0] + 1:
            raise ValueError("the CSR has %d rows, the solved factors %d" % (indptr.numel() - 1, solve.shape[0]))
        if solve.shape[1] != self.factors or fixed.shape[1] != self.factors:
            raise ValueError("factor matrices must be [n, %d]" % self.factors)
        ws = self._workspace(fixed.shape[0])
        n = solve.shape[0]
        per = (n + self.world - 1) // self.world
        r0, r1 = min(n, self.rank * per), min(n, (self.rank + 1) * per)
        if r1 > r0:
            nat.check(nat.lib().dcue_wrmf_half_step(
                nat.ptr(solve[r0:r1]), r1 - r0, nat.ptr(fixed), fixed.shape[0], self.factors,
                nat.ptr(indptr[r0:]), nat.ptr(indices), nat.ptr(values), self.alpha, self.regularization,
                nat.ptr(ws), ws.numel(), nat.stream_handle()), "dcue_wrmf_half_step")
        if self.world > 1:
            full = self._storage(solve)
            self.comm.allgather_(full[:per * self.world].view(-1))
        return solve

    def _storage(self, view):
        for buf in (self._uf, self._if):
            if buf is not None and view.data_ptr() == buf.data_ptr():
                return buf
        raise ValueError("under a communicator, half_step solves user_factors or item_factors in place")

    def init_factors(self, n_users, n_items):
        g = torch.Generator(device="cpu").manual_seed(self.seed)
        uf = (torch.randn(n_users, self.factors, generator=g) * 0.01).to(self.device)
        itf = (torch.randn(n_items, self.factors, generator=g) * 0.01).to(self.device)
        w = self.world
        self._uf = torch.zeros(((n_users + w - 1) // w) * w, self.factors, device=self.device)
        self._if = torch.zeros(((n_items + w - 1) // w) * w, self.factors, device=self.device)
        self._uf[:n_users].copy_(uf)
        self._if[:n_items].copy_(itf)
        self.user_factors, self.item_factors = self._uf[:n_users], self._if[:n_items]

    def fit(self, user_idx, item_idx, values=None, n_users=None, n_items=None):
        u = torch.as_tensor(user_idx, device=self.device)
        i = torch.as_tensor(item_idx, device=self.device)
        v = None if values is None else torch.as_tensor(values, device=self.device)
        n_users = int(u.max()) + 1 if n_users is None else int(n_users)
        n_items = int(i.max()) + 1 if n_items is None else int(n_items)
        # every index is a row of the other side's factors: the solver gathers them unchecked
        if int(u.min()) < 0 or int(u.max()) >= n_users or int(i.min()) < 0 or int(i.max()) >= n_items:
            raise ValueError("user / item indices must lie in [0, n_users) / [0, n_items)")
        self.by_user = device_csr(u, i, v, n_users)
        self.by_item = device_csr(i, u, v, n_items)
        # (re)initialise unless both factor sets already have this problem's shapes (a refit with a
        # different item count must not keep item factors the CSRs index past)
        if (self.user_factors is None or self.user_factors.shape[0] != n_users
                or self.item_factors.shape[0] != n_items):
            self.init_factors(n_users, n_items)
        for _ in range(self.iterations):
            self.half_step(self.user_factors, self.item_factors, self.by_user)
            self.half_step(self.item_factors, self.user_factors, self.by_item)
        return self

    def loss(self):
        """The WRMF objective sum_{u,i} c_ui (p_ui - x_u.y_i)^2 + lambda (|X|^2 + |Y|^2), evaluated
        in fp64 from the dense score matrix (small problems: diagnostics and tests)."""
        X, Y = self.user_factors.double(), self.item_factors.double()
        S = X @ Y.T
        indptr, indices, values = self.by_user
        rows = torch.repeat_interleave(torch.arange(X.shape[0], device=X.device), indptr[1:] - indptr[:-1])
        C = torch.ones_like(S)
        P = torch.zeros_like(S)
        vv = torch.ones(indices.shape[0], dtype=torch.float64, device=X.device) if values is None else values.double()
        C[rows, indices.long()] = 1.0 + self.alpha * vv
        P[rows, indices.long()] = 1.0
        return float((C * (P - S) ** 2).sum() + self.regularization * ((X ** 2).sum() + (Y ** 2).sum()))
