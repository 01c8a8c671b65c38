"""ORACLE -- CPU restatement of the DCUE evaluation metrics.  TEST INFRASTRUCTURE ONLY.

Only tests/ (and __graft_entry__.smoke()) may import this module, as the checker of the GPU
evaluator (csrc/rank.hip, include/dcue.h dcue_rank_*). The product path never imports it.

What it restates (reference = estebandito22/Amplifai-DeepContentRecommenders @ /root/reference):

* DCUE.score: per user, a split-weighted AUC over                      nn/dcue.py:380-449
    pos set = pred-split positives (1) + truth-split negatives (0)
    neg set = pred-split negatives (0) + truth-split positives (1)
  each set scored 1 if all its targets are 1 (empty included), 0 if none are, else
  sklearn roc_auc_score; weights = set sizes / total; mAP = sklearn average_precision_score over
  both sets concatenated.  The user loop stops at the first user without pred-split songs (:393-394).
* DCUE.score_song: per song, plain AUC / AP over the pred split, 1/1 when every target is 1,
  0/0 when none is, songs without users skipped                         nn/dcue.py:451-476
  Its negative list is every split user except user index 0 -- the song's own users included --
  because DCUEPredset._song_nonuser_userids reads `getrow(i).nonzero()[0]`, the ROW indices of a
  1-row matrix (all 0), as the song's users (datasets/dcuepredset.py:53-62).
* the candidate lists of DCUEPredset.create_user_data / create_song_data
  (positives = the split's triplets of the user/song, negatives = the split's songs/users the
  user/song never interacted with in ANY split)                        datasets/dcuepredset.py:39-131
* DCUE._item_factors: eval conv over the item set, summed n_iter times, / n_iter  nn/dcue.py:640-668
* DCUE._user_factors: eval user tower for every user index                        nn/dcue.py:629-638
* scores: the model's nn.CosineSimilarity(dim=1) on (user factor, item factor) rows (:517).

sklearn (1.7.2 here; not vendored in the reference) is restated from its published definitions:
roc_auc_score = area under the tie-aware ROC = Mann-Whitney U / (n_pos n_neg) with ties counted
1/2; average_precision_score = sum over distinct thresholds of (R_k - R_{k-1}) P_k, 0 without
positives.  Pinned by tests/golden/metrics.npz (sklearn on tied vectors) and tests/golden/eval.npz
(the reference's DCUE.score / score_song / factor builders run end to end).
"""
import numpy as np
import torch


def _assert_all_finite(s):
    """sklearn's input validation (utils.validation._assert_all_finite, run by roc_auc_score and
    average_precision_score on y_score): NaN or infinity raises ValueError."""
    if not np.isfinite(s).all():
        raise ValueError("Input contains NaN." if np.isnan(s).any() else
                         "Input contains infinity or a value too large for dtype('float64').")


def roc_auc(targets, scores):
    """sklearn roc_auc_score for binary targets with both classes present (tie-aware)."""
    y = np.asarray(targets).astype(bool)
    s = np.asarray(scores, dtype=np.float64)
    _assert_all_finite(s)
    sp, sn = s[y], s[~y]
    if len(sp) == 0 or len(sn) == 0:
        raise ValueError("roc_auc needs both classes")
    sn = np.sort(sn)
    lt = np.searchsorted(sn, sp, side="left")
    le = np.searchsorted(sn, sp, side="right")
    return float((lt + 0.5 * (le - lt)).sum() / (len(sp) * len(sn)))


def average_precision(targets, scores):
    """sklearn average_precision_score: mean over positives of precision at the positive's score
    (every item with a score >= it counted), 0 when there is no positive."""
    y = np.asarray(targets).astype(bool)
    s = np.asarray(scores, dtype=np.float64)
    _assert_all_finite(s)
    if not y.any():
        return 0.0
    srt = np.sort(s)
    ps = np.sort(s[y])
    all_ge = len(s) - np.searchsorted(srt, s[y], side="left")
    pos_ge = len(ps) - np.searchsorted(ps, s[y], side="left")
    return float((pos_ge / all_ge).sum() / len(ps))


def _auc_or_const(targets, scores):
    t = np.asarray(targets)
    if t.sum() == len(t):
        return 1.0
    if t.sum() == 0:
        return 0.0
    return roc_auc(t, scores)


def user_metrics(s_pred, y_pred, s_truth, y_truth):
    """One user of DCUE.score (nn/dcue.py:399-447): (split-weighted AUC, AP)."""
    s_pred, y_pred = np.asarray(s_pred, np.float64), np.asarray(y_pred)
    s_truth, y_truth = np.asarray(s_truth, np.float64), np.asarray(y_truth)
    pp, pn = y_pred == 1, y_pred == 0
    tp, tn = y_truth == 1, y_truth == 0
    pos_s = np.concatenate([s_pred[pp], s_truth[tn]])
    pos_t = np.concatenate([y_pred[pp], y_truth[tn]])
    neg_s = np.concatenate([s_pred[pn], s_truth[tp]])
    neg_t = np.concatenate([y_pred[pn], y_truth[tp]])
    total = len(pos_s) + len(neg_s)
    auc = (len(pos_s) / total) * _auc_or_const(pos_t, pos_s) + (len(neg_s) / total) * _auc_or_const(neg_t, neg_s)
    ap = average_precision(np.concatenate([pos_t, neg_t]), np.concatenate([pos_s, neg_s]))
    return auc, ap


def song_metrics(scores, targets):
    """One song of DCUE.score_song (nn/dcue.py:463-474): (AUC, AP)."""
    t = np.asarray(targets)
    if t.sum() == len(t):
        return 1.0, 1.0
    if t.sum() == 0:
        return 0.0, 0.0
    return roc_auc(t, scores), average_precision(t, scores)


def cosine_rows(a, b):
    """nn.CosineSimilarity(dim=1) on CPU fp32, as DCUE.predict calls it (nn/dcue.py:517)."""
    return torch.nn.functional.cosine_similarity(torch.as_tensor(a), torch.as_tensor(b), dim=1).numpy()


def rank_metrics(query_feat, cand_feat, queries, pos_ptr, pos_idx, cand_class, mode):
    """The GPU evaluator's contract (dcue_rank_metrics) restated per query with the functions
    above. mode 0 (DCUE.score): candidates with class bit 0 form the pred list, bit 1 the truth
    list; a candidate is a positive of query row q iff it is in q's CSR row. mode 1
    (DCUE.score_song): positives = CSR row & bit 1, label-0 list = every bit-0 candidate.
    Returns (auc, ap, has_pos) arrays. Raises ValueError where the reference's sklearn calls would
    on non-finite scores: mode 0 for a query before the first one without pred positives (the
    reference's user loop breaks there, nn/dcue.py:396-397), mode 1 for any query."""
    cand_class = np.asarray(cand_class)
    inP = (cand_class & 1) != 0
    inT = (cand_class & 2) != 0
    auc = np.zeros(len(queries))
    ap = np.zeros(len(queries))
    flag = np.zeros(len(queries), dtype=np.int32)
    stopped = False
    for k, q in enumerate(queries):
        pos = np.zeros(len(cand_class), dtype=bool)
        pos[pos_idx[pos_ptr[q]:pos_ptr[q + 1]]] = True
        qv = np.repeat(np.asarray(query_feat[q:q + 1], np.float32), len(cand_class), axis=0)
        s = cosine_rows(qv, np.asarray(cand_feat, np.float32)).astype(np.float64)
        if mode == 0:
            flag[k] = int((pos & inP).any())
            stopped |= not flag[k]
            try:
                auc[k], ap[k] = user_metrics(s[inP], pos[inP].astype(int), s[inT], pos[inT].astype(int))
            except ValueError:
                if not stopped:
                    raise
                auc[k] = ap[k] = np.nan
        else:
            # score_song's list: the song's users (1) + every list-0 user (0), its own users included
            # (dcuepredset.py:53-62 keeps them: getrow(i).nonzero()[0] are row indices, all 0)
            sp = s[pos & inT]
            flag[k] = int(len(sp) > 0)
            auc[k], ap[k] = song_metrics(np.concatenate([sp, s[inP]]),
                                         np.concatenate([np.ones(len(sp), int), np.zeros(int(inP.sum()), int)]))
    return auc, ap, flag


def item_factors_avg(f, n_iter=10):
    """DCUE._item_factors' accumulation: n_iter fp32 sums of the same eval pass, then / n_iter
    (the pass is deterministic for 131-frame tracks, which need no crop)."""
    f = torch.as_tensor(f, dtype=torch.float32)
    acc = torch.zeros_like(f)
    for _ in range(n_iter):
        acc += f
    return acc / n_iter
