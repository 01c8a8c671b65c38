"""GPU ranking evaluation of DCUE (nn/dcue.py:380-476) over include/dcue.h dcue_rank_metrics.

The reference scores one user at a time: it builds a pandas frame of every split song
(DCUEPredset.create_user_data), batches it through a DataLoader, gathers factors row by row,
calls model.sim and sklearn's roc_auc_score / average_precision_score. Here the candidate lists
are two bitmasks over the catalogue plus the all-split interaction CSR, built once per dataset on
the host, and every sampled query is ranked on the GPU in one call.
"""
import numpy as np
import torch

from dcrecommend import _native as nat

LIST_PRED, LIST_TRUTH = 1, 2


def _csr_users_to_items(ds):
    csc = ds.item_user.tocsc()  # columns = users
    csc.sort_indices()
    return csc.indptr.astype(np.int64), csc.indices.astype(np.int32)


def _csr_items_to_users(ds):
    csr = ds.item_user.tocsr()  # rows = items
    csr.sort_indices()
    return csr.indptr.astype(np.int64), csr.indices.astype(np.int32)


def user_split_inputs(pred_ds, truth_ds, index_ds=None):
    """DCUE.score's candidate lists (nn/dcue.py:399-416 over dcuepredset.py:39-93): pred list =
    the pred split's songs, truth list = the truth split's songs, a user's positives = every song
    the user interacted with in any split (the lists' negatives exclude all of them)."""
    index_ds = index_ds if index_ds is not None else pred_ds
    ptr, idx = _csr_users_to_items(index_ds)
    cls = np.zeros(index_ds.n_items, dtype=np.uint8)
    cls[pred_ds.split_items()] |= LIST_PRED
    cls[truth_ds.split_items()] |= LIST_TRUTH
    return {"pos_ptr": ptr, "pos_idx": idx, "cand_class": cls}


def song_inputs(pred_ds):
    """DCUE.score_song's lists (nn/dcue.py:463-474 over dcuepredset.py:53-62, 95-124): positives =
    the song's users (bit 1 = the split's users); label-0 list (bit 0) = every split user except
    user index 0, the song's own users included -- the reference's `getrow(i).nonzero()[0]` yields
    row indices (all 0), so only user 0 is ever excluded."""
    ptr, idx = _csr_items_to_users(pred_ds)
    cls = np.zeros(pred_ds.n_users, dtype=np.uint8)
    users = pred_ds.split_users()
    cls[users] = LIST_PRED | LIST_TRUTH
    if len(pred_ds.split_items()):
        cls[0] &= ~np.uint8(LIST_PRED)
    return {"pos_ptr": ptr, "pos_idx": idx, "cand_class": cls}


def mean_until_missing(values, has_pos):
    """DCUE.score's mean: the user loop `break`s at the first user without pred-split songs
    (nn/dcue.py:393-394), so only the users before it count."""
    has_pos = np.asarray(has_pos, bool)
    stop = int(np.argmin(has_pos)) if not has_pos.all() else len(has_pos)
    return float(np.mean(np.asarray(values, np.float64)[:stop]))


class RankEvaluator:
    """Device-resident candidate lists for one (query kind, pred split, truth split) and the
    workspace of dcue_rank_metrics."""

    def __init__(self, inputs, device, max_score_bytes=1 << 30):
        self.device = torch.device(device)
        self.pos_ptr = torch.from_numpy(inputs["pos_ptr"]).to(self.device)
        self.pos_idx = torch.from_numpy(inputs["pos_idx"]).to(self.device)
        if self.pos_idx.numel() == 0:
            self.pos_idx = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.cand_class = torch.from_numpy(inputs["cand_class"]).to(self.device)
        self.n_cand = int(self.cand_class.numel())
        self.max_score_bytes = max_score_bytes
        self._ws = None

    def _workspace(self, d, qb):
        import ctypes
        nbytes = ctypes.c_size_t()
        nat.check(nat.lib().dcue_rank_workspace_bytes(self.n_cand, d, qb, ctypes.byref(nbytes)),
                  "dcue_rank_workspace_bytes")
        if self._ws is None or self._ws.numel() < nbytes.value:
            self._ws = torch.empty(nbytes.value, dtype=torch.uint8, device=self.device)
        return self._ws

    def metrics(self, query_feat, cand_feat, queries, mode):
        """(auc, ap, has_pos) numpy arrays, one entry per query (fp64).

        Raises ValueError where the reference's sklearn calls would (roc_auc_score /
        average_precision_score on NaN or infinite scores, nn/dcue.py:440,447,473-474): DCUE.score
        for a query before the first one without pred positives (its loop breaks there, :396-397),
        DCUE.score_song for any query with both labels."""
        nat.require_gpu(query_feat, "query_feat")
        nat.require_gpu(cand_feat, "cand_feat")
        query_feat = query_feat.contiguous().float()
        cand_feat = cand_feat.contiguous().float()
        if cand_feat.shape[0] != self.n_cand or cand_feat.shape[1] != query_feat.shape[1]:
            raise ValueError("candidate factors %s do not match %d candidates / d=%d"
                             % (tuple(cand_feat.shape), self.n_cand, query_feat.shape[1]))
        if query_feat.shape[0] + 1 != self.pos_ptr.numel():
            raise ValueError("query factors have %d rows, the CSR %d" % (query_feat.shape[0],
                                                                          self.pos_ptr.numel() - 1))
        q = torch.as_tensor(np.asarray(queries, dtype=np.int32)).to(self.device)
        nq = int(q.numel())
        auc = torch.zeros(max(nq, 1), dtype=torch.float64, device=self.device)
        ap = torch.zeros_like(auc)
        flag = torch.zeros(max(nq, 1), dtype=torch.int32, device=self.device)
        if nq:
            if int(q.min()) < 0 or int(q.max()) >= query_feat.shape[0]:
                raise IndexError("query index out of range")
            d = int(query_feat.shape[1])
            qb = int(max(16, min(nq, self.max_score_bytes // (4 * max(self.n_cand, 1)))))
            ws = self._workspace(d, qb)
            nat.check(nat.lib().dcue_rank_metrics(
                nat.ptr(query_feat), query_feat.shape[0], nat.ptr(cand_feat), self.n_cand, d, nat.ptr(q), nq,
                nat.ptr(self.pos_ptr), nat.ptr(self.pos_idx), nat.ptr(self.cand_class), int(mode), qb,
                nat.ptr(ws), ws.numel(), nat.ptr(auc), nat.ptr(ap), nat.ptr(flag), nat.stream_handle(self.device)),
                "dcue_rank_metrics")
        auc, ap, flag = auc[:nq].cpu().numpy(), ap[:nq].cpu().numpy(), flag[:nq].cpu().numpy()
        ok = (flag & 1).astype(bool)
        nonfinite = (flag & 2).astype(bool)
        checked = nonfinite[:int(np.argmin(ok))] if (mode == nat.RANK_SPLIT and not ok.all()) else nonfinite
        if checked.any():
            # (a cosine of finite factors is finite: non-finite factors make NaN scores)
            raise ValueError("Input contains NaN. (DCUE scores of query %d: the model's factors are not "
                             "finite)" % int(np.asarray(queries)[int(np.argmax(checked))]))
        sane = ~nonfinite
        if not (np.all((auc[sane] >= 0.0) & (auc[sane] <= 1.0)) and np.all((ap[sane] >= 0.0) & (ap[sane] <= 1.0))):
            raise RuntimeError("dcue_rank_metrics: AUC / AP outside [0, 1]")
        return auc, ap, ok
