"""Row f2 at scale: DCUEDataset's host index builders are vectorised (category codes), so the
config-3 shape -- 1M users x 1M tracks, 50M interactions (BASELINE.json configs[2]) -- builds in
seconds per million rows instead of per-row dict lookups.

Parity: the vectorised split_rows / uniq_*_idxs / split_items / split_users equal the reference's
per-row lookups (datasets/dcuedataset.py:74-97: user_index / item_index of each triplet's ids)
on the same frame; user_split_ranks (the GPU catalogue sampler's CSR) equals a direct per-user
restatement of datasets/dcuedataset.py:214-218 on sampled users.
"""
import time

import numpy as np
import pandas as pd

from dcrecommend.datasets.csr import user_split_ranks
from dcrecommend.datasets.dcuedataset import DCUEDataset


def _frame(n_rows, n_users, n_songs, seed):
    rs = np.random.RandomState(seed)
    u = rs.randint(0, n_users, n_rows)
    s = rs.zipf(1.3, n_rows) % n_songs  # skewed popularity, like play counts
    trip = pd.DataFrame({"user_id": pd.Series(u).map("u{:07d}".format),
                         "song_id": pd.Series(s).map("S{:07d}".format),
                         "score": rs.randint(1, 5, n_rows)})
    songs = np.unique(trip["song_id"].to_numpy())
    meta = pd.DataFrame({"x": np.arange(len(songs)), "song_id": songs, "data_mel": ["-"] * len(songs)})
    return trip, meta


def test_vectorised_indices_match_per_row_lookups():
    trip, meta = _frame(60_000, 3_000, 20_000, 0)
    for split in ("train", "val", "test"):
        ds = DCUEDataset(trip.copy(), meta, split=split)
        u, s = ds.split_rows()
        want_u = np.array([ds.user_index[x] for x in ds.triplets["user_id"]], dtype=np.int64)
        want_s = np.array([ds.item_index[x] for x in ds.triplets["song_id"]], dtype=np.int64)
        assert np.array_equal(u, want_u) and np.array_equal(s, want_s)
        assert ds.uniq_song_idxs == [ds.item_index[x] for x in ds.uniq_songs]
        assert ds.uniq_user_idxs == [ds.user_index[x] for x in ds.uniq_users]
        assert np.array_equal(ds.split_items(), np.array(sorted(ds.item_index[x] for x in ds.uniq_songs)))
        assert np.array_equal(ds.split_users(), np.array(sorted(ds.user_index[x] for x in ds.uniq_users)))


def test_catalogue_csr_matches_reference_candidates():
    """user_split_ranks holds, per user, the split positions of the user's interacted split items;
    the reference's candidate list is the split items minus those (dcuedataset.py:214-218)."""
    trip, meta = _frame(40_000, 2_000, 8_000, 1)
    ds = DCUEDataset(trip.copy(), meta, split="train")
    split = ds.split_items()
    coo = ds.item_user.tocoo()
    indptr, ranks = user_split_ranks(coo.col, coo.row, ds.n_users, split)
    rs = np.random.RandomState(2)
    for ui in rs.choice(ds.n_users, 200, replace=False):
        items = ds.item_user.getcol(ui).nonzero()[0]
        nonitems = ds.all_items[(~np.in1d(ds.all_items, items)) & np.in1d(ds.all_items, ds.uniq_song_idxs)]
        mine = np.setdiff1d(np.arange(len(split)), ranks[indptr[ui]:indptr[ui + 1]])
        assert np.array_equal(split[mine], nonitems)


def test_build_time_at_scale():
    """2M interactions over 200k users x 500k songs: every index builder of the trainer in well
    under a minute (the per-row form took ~1 s per 0.5M rows for split_rows alone)."""
    trip, meta = _frame(2_000_000, 200_000, 500_000, 3)
    t0 = time.perf_counter()
    ds = DCUEDataset(trip, meta, split="train")
    u, s = ds.split_rows()
    split = ds.split_items()
    coo = ds.item_user.tocoo()
    indptr, ranks = user_split_ranks(coo.col, coo.row, ds.n_users, split)
    dt = time.perf_counter() - t0
    assert len(u) == len(ds) and indptr[-1] == len(ranks)
    assert dt < 60, "index build took %.1f s" % dt
