"""DCUEItemset: every catalogue track once, for item factors (datasets/dcueitemset.py:8-53).

`track_table()` is what the MI355X trainer uses: all of the set's spectrograms loaded ONCE into an
HBM-resident [n_meta][131][128] table (fp16 when every value is fp16-representable, else fp32), so
the item factors (DCUE._item_factors) and training batches index rows instead of torch.loading
tensors per sample (dcueitemset.py:44-53, dcuedataset.py:233-252).
"""
import numpy as np
import torch

from dcrecommend.datasets.dcuedataset import DCUEDataset, N_FRAMES


class DCUEItemset(DCUEDataset):

    def __init__(self, triplets, metadata, n_users=20000, n_items=10000, song_artist_map=None,
                 artist_bios=None, random_seed=None):
        DCUEDataset.__init__(self, triplets, metadata, n_users=n_users, n_items=n_items,
                             song_artist_map=song_artist_map, artist_bios=artist_bios,
                             random_seed=random_seed)
        self.metadata = self.metadata[self.metadata['song_id'].isin(list(self.item_index.keys()))]
        del self.item_user
        del self.triplets

    def __len__(self):
        return self.metadata.shape[0]

    def __getitem__(self, i):
        song_idx = self.songid2metaindex[self.metadata.iat[i, 1]]
        X = torch.load(self.metadata.at[song_idx, 'data_mel'], weights_only=True)
        return {'X': self._sample(X, N_FRAMES, 1), 'metadata_index': song_idx}

    def metadata_indexes(self):
        """Metadata index of every row of the set, in set order (the item loader's order)."""
        return np.array([self.songid2metaindex[s] for s in self.metadata['song_id']], dtype=np.int64)

    def track_table(self, device, n_meta=None, dtype=None):
        """[n_meta][131][128] spectrogram rows indexed by metadata index, on `device`. Rows of
        metadata indices outside the set stay zero. dtype None: fp16 if lossless, else fp32."""
        idx = self.metadata_indexes()
        n_meta = int(n_meta if n_meta is not None else (idx.max() + 1 if len(idx) else 0))
        host = torch.zeros((n_meta, N_FRAMES, 128), dtype=torch.float32)
        for i, m in enumerate(idx):
            X = self.__getitem__(i)['X'].float()
            host[m] = X.t()
        if dtype is None:
            dtype = torch.float16 if torch.equal(host.half().float(), host) else torch.float32
        return host.to(dtype).to(device)

    def item_rows(self):
        """metadata index of every item index (songid2metaindex over item_index), -1 if absent."""
        rows = np.full(len(self.item_index), -1, dtype=np.int64)
        for s, i in self.item_index.items():
            rows[i] = self.songid2metaindex.get(s, -1)
        return rows
