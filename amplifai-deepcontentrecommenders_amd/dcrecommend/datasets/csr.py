"""Host-side index structures the GPU catalogue sampler reads (built once per dataset)."""
import numpy as np


def user_split_ranks(user_idx, item_idx, n_users, split_items):
    """CSR over users of the sorted, distinct ranks (positions in `split_items`) of each user's
    interacted items that belong to the split.

    This is the information datasets/dcuedataset.py:214-218 recomputes per sample with np.in1d over
    every item (`items = item_user.getcol(i).nonzero()[0]`; non-items = split songs minus items):
    the GPU sampler turns a draw r into the r-th non-item by skipping these ranks.
    """
    split_items = np.asarray(split_items, dtype=np.int64)
    user_idx = np.asarray(user_idx, dtype=np.int64)
    item_idx = np.asarray(item_idx, dtype=np.int64)
    n = len(split_items)
    pos = np.searchsorted(split_items, item_idx)
    inside = pos < n
    inside[inside] = split_items[pos[inside]] == item_idx[inside]
    key = np.unique(user_idx[inside] * (n + 1) + pos[inside])
    u, r = key // (n + 1), key % (n + 1)
    indptr = np.zeros(n_users + 1, dtype=np.int64)
    np.add.at(indptr, u + 1, 1)
    return np.cumsum(indptr), r.astype(np.int32)
