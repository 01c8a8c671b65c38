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
    indptr[1:] = np.cumsum(np.bincount(u, minlength=n_users)[:n_users])
    return indptr, r.astype(np.int32)


def saturated_users(indptr, n_split):
    """Users who interacted with every song of the split: the reference's
    np.random.choice(nonitems, N) raises ValueError for them (datasets/dcuedataset.py:219, an empty
    `nonitems`). The GPU sampler writes -1 for such a row; callers check batches against this set
    on the host first and raise as the reference does."""
    return np.nonzero(np.diff(np.asarray(indptr, dtype=np.int64)) >= int(n_split))[0]


def check_catalogue_users(users, saturated):
    """Raise numpy's ValueError if a batch row's user has no candidate negative."""
    if len(saturated) and np.isin(np.asarray(users), saturated).any():
        raise ValueError("a cannot be empty unless no samples are taken")
