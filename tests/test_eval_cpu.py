"""Evaluation path on the host: the metric oracle against sklearn / the reference's DCUE.score and
score_song outputs, and the dataset mirror's indices and splits against the reference's."""
import numpy as np
import pandas as pd
import pytest

from oracle import rank_oracle as R


def test_metric_arithmetic_matches_sklearn(golden):
    g = golden("metrics.npz")
    for c in range(3):
        sp, tp = g["c%d_sp" % c], g["c%d_tp" % c]
        if 0 < tp.sum() < len(tp):
            assert abs(R.roc_auc(tp, sp) - float(g["c%d_auc" % c])) < 1e-12
        assert abs(R.average_precision(tp, sp) - float(g["c%d_ap" % c])) < 1e-12


def eval_datasets(g):
    """Our dataset mirror over the fixture's raw triplets (same frames the reference saw)."""
    from dcrecommend.datasets.dcuepredset import DCUEPredset
    from dcrecommend.datasets.dcueitemset import DCUEItemset
    trip = pd.DataFrame({"user_id": g["raw_users"], "song_id": g["raw_songs"], "score": g["raw_score"]})
    meta = pd.DataFrame({"idx": np.arange(len(g["meta_songs"])), "song_id": g["meta_songs"],
                         "data_mel": [""] * len(g["meta_songs"])})
    train = DCUEPredset(trip.copy(), meta, split="train")
    val = DCUEPredset(trip.copy(), meta, split="val")
    items = DCUEItemset(trip.copy(), meta)
    return train, val, items


def eval_structures(g, train, val, items):
    """Device-side inputs of the evaluator, built by the product's host code (dcrecommend.nn.rank)."""
    from dcrecommend.nn import rank
    uf = g["user_factors"].astype(np.float32)
    itf = g["item_factors"].astype(np.float32)
    cand = itf[items.item_rows()]  # item-index order
    return rank.user_split_inputs(train, val, train), rank.song_inputs(val), uf, cand


@pytest.fixture(scope="module")
def ev(golden):
    g = golden("eval.npz")
    train, val, items = eval_datasets(g)
    return g, train, val, items


def test_dataset_indices_and_split(ev):
    g, train, val, items = ev
    assert list(train.user_index) == list(g["user_categories"])
    assert list(train.item_index) == list(g["song_categories"])
    assert np.array_equal(train.split_items(), g["train_split_items"])
    assert np.array_equal(val.split_items(), g["val_split_items"])


def _users(ds, names):
    return np.array([ds.user_index[u] for u in names], dtype=np.int64)


def test_oracle_matches_reference_scores(ev):
    g, train, val, items = ev
    (u_in, s_in, uf, cand) = eval_structures(g, train, val, items)
    for split, names, want_auc, want_ap in (("val", g["val_users"], g["val_auc"], g["val_ap"]),):
        q = _users(train, names)
        auc, ap, flag = R.rank_metrics(uf, cand, q, u_in["pos_ptr"], u_in["pos_idx"], u_in["cand_class"], 0)
        assert flag.all()
        np.testing.assert_allclose(auc, want_auc, rtol=0, atol=1e-12)
        np.testing.assert_allclose(ap, want_ap, rtol=0, atol=1e-12)
    from dcrecommend.nn import rank
    t_in = rank.user_split_inputs(train, train, train)
    q = _users(train, g["train_users"])
    auc, ap, _ = R.rank_metrics(uf, cand, q, t_in["pos_ptr"], t_in["pos_idx"], t_in["cand_class"], 0)
    np.testing.assert_allclose(auc, g["train_auc"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(ap, g["train_ap"], rtol=0, atol=1e-12)
    # score_song: queries are songs (item factors), candidates users
    songs = np.array([val.item_index[s] for s in g["val_songs"]], dtype=np.int64)
    auc, ap, flag = R.rank_metrics(cand, uf, songs, s_in["pos_ptr"], s_in["pos_idx"], s_in["cand_class"], 1)
    assert flag.all()
    np.testing.assert_allclose(auc, g["song_auc"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(ap, g["song_ap"], rtol=0, atol=1e-12)


def test_score_mean_and_break(ev):
    g, train, val, items = ev
    from dcrecommend.nn import rank
    assert rank.mean_until_missing(g["val_auc"][:9], np.ones(9, bool)) == pytest.approx(float(g["mean9_auc"]), abs=1e-12)
    assert rank.mean_until_missing(g["val_ap"][:9], np.ones(9, bool)) == pytest.approx(float(g["mean9_ap"]), abs=1e-12)
    # the reference's user loop breaks at the first user without pred songs (nn/dcue.py:393-394)
    assert rank.mean_until_missing(np.array([0.2, 0.4, 0.9]), np.array([1, 1, 0], bool)) == pytest.approx(0.3)


def test_item_factor_average(ev):
    g = ev[0]
    f = np.random.RandomState(0).randn(48, 16).astype(np.float32)
    out = R.item_factors_avg(f).numpy()
    assert np.abs(out - f).max() < 1e-6


def test_nonfinite_factors_raise_like_sklearn(ev):
    """The reference's sklearn calls raise ValueError on NaN / inf scores (nn/dcue.py:440,447,473-474):
    the restatement raises where they would -- a user before the score() loop's break, any song with
    both labels -- and not for a user after the break."""
    from sklearn.metrics import average_precision_score, roc_auc_score
    for f in (roc_auc_score, average_precision_score, R.roc_auc, R.average_precision):
        with pytest.raises(ValueError, match="Input contains NaN"):
            f([0, 1, 1], [0.1, np.nan, 0.3])
    g, train, val, items = ev
    (u_in, s_in, uf, cand) = eval_structures(g, train, val, items)
    q = _users(train, g["val_users"])
    bad = np.array(uf, dtype=np.float32, copy=True)
    bad[q[0]] = np.nan
    with pytest.raises(ValueError, match="Input contains NaN"):
        R.rank_metrics(bad, cand, q, u_in["pos_ptr"], u_in["pos_idx"], u_in["cand_class"], 0)
    # a user with no pred-split songs stops the loop: a NaN factor after it is never scored
    ptr = np.asarray(u_in["pos_ptr"])
    cls = np.asarray(u_in["cand_class"])
    no_pred = [u for u in range(len(ptr) - 1)
               if not (cls[np.asarray(u_in["pos_idx"])[ptr[u]:ptr[u + 1]]] & 1).any()]
    if no_pred:
        after = np.array([q[0], no_pred[0], q[1]], dtype=np.int64)
        bad2 = np.array(uf, dtype=np.float32, copy=True)
        bad2[q[1]] = np.nan
        _, _, flag = R.rank_metrics(bad2, cand, after, u_in["pos_ptr"], u_in["pos_idx"], u_in["cand_class"], 0)
        assert list(flag[:2]) == [1, 0]
    songs = np.array([val.item_index[s] for s in g["val_songs"]], dtype=np.int64)
    badc = np.array(cand, dtype=np.float32, copy=True)
    badc[songs[0]] = np.inf
    with pytest.raises(ValueError):
        R.rank_metrics(badc, uf, songs, s_in["pos_ptr"], s_in["pos_idx"], s_in["cand_class"], 1)
