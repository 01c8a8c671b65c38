"""DCUEDataset: the reference's interaction dataset (datasets/dcuedataset.py:14-256), host side.

Same constructor, attributes (item_user, user_index, item_index, songid2metaindex,
itemindex2songid, userindex2userid, uniq_songs/uniq_song_idxs, uniq_users/uniq_user_idxs,
all_items/all_users, n_items/n_users), song split, get_batches, subset and per-sample
__getitem__, so reference code that builds datasets keeps working.

What the MI355X trainer reads instead of per-sample __getitem__ (which torch.loads 21 tensors and
runs np.in1d over every item per row, dcuedataset.py:207-256) are the device structures of
`gpu_index()`: the user -> item CSR over ALL interactions and the split's item list, consumed by
the GPU catalogue sampler (include/dcue.h dcue_sample_catalogue) and the evaluator (dcue_rank_*).
"""
import numpy as np
import pandas as pd
import torch
import torch.nn.functional as F
from scipy.sparse import csr_matrix
from torch.utils.data import Dataset

N_FRAMES = 131


class DCUEDataset(Dataset):

    def __init__(self, triplets, metadata, neg_samples=20, split='train', n_users=20000, n_items=10000,
                 song_artist_map=None, artist_bios=None, random_seed=None):
        """triplets: DataFrame (user_id, song_id, score) by column position; metadata: DataFrame with
        song_id in column 1 and a `data_mel` path column (dcuedataset.py:17-31)."""
        self.triplets = triplets
        self.metadata = metadata
        self.neg_samples = neg_samples
        self.split = split
        self.song_artist_map = song_artist_map
        self.artist_bios = artist_bios
        self.random_seed = random_seed
        # interaction matrix and category indices over ALL triplets, before the split (:74-97):
        # item / user index = lexicographic rank of the id (pandas category codes)
        self.triplets['user_id'] = self.triplets['user_id'].astype("category")
        self.triplets['song_id'] = self.triplets['song_id'].astype("category")
        items = self.triplets['song_id'].cat
        users = self.triplets['user_id'].cat
        self.item_user = csr_matrix((self.triplets['score'], (items.codes.copy(), users.codes.copy())),
                                    shape=(len(items.categories), len(users.categories))).tocsc()
        self.user_index = {u: i for i, u in enumerate(users.categories)}
        self.item_index = {s: i for i, s in enumerate(items.categories)}
        self.songid2metaindex = {s: i for i, s in self.metadata['song_id'].to_dict().items()}
        self.itemindex2songid = {i: s for s, i in self.item_index.items()}
        self.userindex2userid = {i: u for u, i in self.user_index.items()}
        self._split_triplets()
        self.n_items, self.n_users = self.item_user.shape
        self.all_items = np.arange(0, self.n_items)
        self.all_users = np.arange(0, self.n_users)
        # the split's songs/users in order of appearance and their indices; the category codes ARE
        # the indices (item_index / user_index enumerate the same categories), so no per-row lookups
        self.uniq_songs = self.triplets['song_id'].unique()
        self.uniq_song_idxs = pd.unique(self.triplets['song_id'].cat.codes.to_numpy()).astype(np.int64).tolist()
        self.uniq_users = self.triplets['user_id'].unique()
        self.uniq_user_idxs = pd.unique(self.triplets['user_id'].cat.codes.to_numpy()).astype(np.int64).tolist()
        self._gpu = None

    def _split_triplets(self):
        """Song split 80/10/10 (dcuedataset.py:146-164): both masks are drawn right after
        np.random.seed(10), so the global numpy stream is left where the reference leaves it."""
        if self.song_artist_map is not None:
            # the reference's artist split calls Series.get_values() (dcuedataset.py:112), removed in
            # pandas 1.0: it cannot run with the pinned pandas either
            raise NotImplementedError("artist splitting (song_artist_map) is not supported: the "
                                      "reference path needs pandas < 1.0")
        songs = self.triplets['song_id'].unique()
        np.random.seed(10)
        in_train = np.random.rand(len(songs)) < 0.80
        train_songs = songs[in_train]
        np.random.seed(10)
        in_val = np.random.rand(int(in_train.sum())) < 0.1 / 0.8
        val_songs = train_songs[in_val]
        sid = self.triplets['song_id']
        if self.split == 'train':
            keep = sid.isin(train_songs) & ~sid.isin(val_songs)
        elif self.split == 'val':
            keep = sid.isin(val_songs)
        elif self.split == 'test':
            keep = ~sid.isin(train_songs)
        else:
            return
        self.triplets = self.triplets[keep]

    # ------------------------------------------------------------------ reference API
    def _sample(self, X, length, dim=1):
        """Crop/pad to `length` frames (dcuedataset.py:166-187): zero-pad shorter tracks; a longer
        track gets a random crop from an OS-entropy reseed, as the reference does."""
        if self.random_seed is not None:
            np.random.seed(self.random_seed)
        if dim not in (0, 1):
            raise ValueError("dim must be 0 or 1.")
        n = X.size()[dim]
        if n <= length:
            pad = (0, 0, 0, length - n) if dim == 0 else (0, length - n, 0, 0)
            return F.pad(X, pad)
        np.random.seed()
        start = np.random.randint(0, n - length)
        return X[start:start + length] if dim == 0 else X[:, start:start + length]

    def get_batches(self, k=5):
        """Shuffled row indices in chunks of ceil(len/k); the last chunk is dropped when
        len % k != 0 (dcuedataset.py:189-201)."""
        order = list(range(len(self)))
        np.random.shuffle(order)
        size = int(np.ceil(len(order) / k))
        chunks = [order[s:s + size] for s in range(0, len(order), size)]
        if len(order) % k != 0:
            chunks = chunks[:-1]
        return chunks

    def subset(self, p):
        self.triplets = self.triplets.sample(frac=p, random_state=10)

    def _user_nonitem_songids(self, user_id):
        """N catalogue negatives for one user, drawn on the host from the global numpy stream
        (dcuedataset.py:207-220); the trainer draws the same values on the GPU."""
        items = self.item_user.getcol(self.user_index[user_id]).nonzero()[0]
        nonitems = self.all_items[(~np.in1d(self.all_items, items)) &
                                  np.in1d(self.all_items, self.uniq_song_idxs)]
        nonitems = np.random.choice(nonitems, self.neg_samples)
        return [self.itemindex2songid[i] for i in nonitems]

    def _load(self, song_id):
        path = self.metadata.at[self.songid2metaindex[song_id], 'data_mel']
        return self._sample(torch.load(path, weights_only=True), N_FRAMES, 1)

    def __len__(self):
        return self.triplets.shape[0]

    def __getitem__(self, i):
        song_id = self.triplets.iat[i, 1]
        user_id = self.triplets.iat[i, 0]
        X = self._load(song_id)
        Ns = torch.stack([self._load(s) for s in self._user_nonitem_songids(user_id)])
        y = torch.full([self.neg_samples], -1.0, dtype=torch.float32)
        return {'u': torch.tensor(self.user_index[user_id]), 'X': X, 'y': y, 'Ns': Ns}

    # ------------------------------------------------------------- device-side structures
    def user_item_csr(self):
        """(indptr [n_users+1] int64, items int32): each user's interacted item indices over all
        splits, sorted -- the rows of the item_user matrix's columns (dcuedataset.py:87-89)."""
        csc = self.item_user.tocsc()
        csc.sort_indices()
        return csc.indptr.astype(np.int64), csc.indices.astype(np.int32)

    def split_items(self):
        """Sorted item indices of this split's songs (the `uniq_song_idxs` filter of :217)."""
        return np.sort(np.asarray(self.uniq_song_idxs, dtype=np.int64))

    def split_users(self):
        return np.sort(np.asarray(self.uniq_user_idxs, dtype=np.int64))

    def split_rows(self):
        """(user index, item index) of every triplet of the split, in DataFrame order: the category
        codes (user_index / item_index of each row), vectorised for config-3 scale (50M rows)."""
        u = self.triplets['user_id'].cat.codes.to_numpy().astype(np.int64)
        s = self.triplets['song_id'].cat.codes.to_numpy().astype(np.int64)
        return u, s
