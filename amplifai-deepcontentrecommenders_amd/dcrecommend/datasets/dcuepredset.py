"""DCUEPredset: per-user / per-song candidate lists for evaluation (datasets/dcuepredset.py:10-148).

The host-side API is kept (create_user_data / create_song_data / __getitem__) for reference code
that iterates it; the MI355X evaluator (dcrecommend.nn.rank) never builds these per-query frames:
it reads the split's item list and the all-split interaction CSR once and ranks every query on
the GPU (include/dcue.h dcue_rank_metrics).
"""
import numpy as np
import pandas as pd
import torch

from dcrecommend.datasets.dcuedataset import DCUEDataset


class DCUEPredset(DCUEDataset):

    def __init__(self, triplets, metadata, split='train', n_users=20000, n_items=10000,
                 song_artist_map=None, artist_bios=None, random_seed=None):
        DCUEDataset.__init__(self, triplets, metadata, split=split, n_users=n_users, n_items=n_items,
                             song_artist_map=song_artist_map, artist_bios=artist_bios,
                             random_seed=random_seed)
        self.triplets_user = self.triplets
        self.user_has_songs = False
        self.song_has_users = False

    def _user_nonitem_songids(self, user_id):
        """Every split song the user never interacted with (no sampling, dcuepredset.py:39-51)."""
        items = self.item_user.getcol(self.user_index[user_id]).nonzero()[0]
        keep = (~np.in1d(self.all_items, items)) & np.in1d(self.all_items, self.uniq_song_idxs)
        return [self.itemindex2songid[i] for i in self.all_items[keep]]

    def _song_nonuser_userids(self, song_id):
        users = self.item_user.getrow(self.item_index[song_id]).nonzero()[1]
        keep = (~np.in1d(self.all_users, users)) & np.in1d(self.all_users, self.uniq_user_idxs)
        return [self.userindex2userid[i] for i in self.all_users[keep]]

    def _candidate_frame(self, others, fixed_col, fixed_val, other_col):
        frame = self.triplets[self.triplets[fixed_col] == fixed_val].copy()
        has = not frame.empty
        if has:
            frame['score'] = 1
        comp = pd.DataFrame({fixed_col: [fixed_val] * len(others), other_col: others,
                             'score': [0] * len(others)})
        frame = pd.concat([frame, comp]) if has else comp
        return frame[['user_id', 'song_id', 'score']], has

    def create_user_data(self, user_id):
        """The user's split songs (score 1) + every other split song (score 0), :64-93."""
        self.triplets_user, self.user_has_songs = self._candidate_frame(
            self._user_nonitem_songids(user_id), 'user_id', user_id, 'song_id')

    def create_song_data(self, song_id):
        """The song's split users (score 1) + every other split user (score 0), :95-124."""
        self.triplets_user, self.song_has_users = self._candidate_frame(
            self._song_nonuser_userids(song_id), 'song_id', song_id, 'user_id')

    def __len__(self):
        return self.triplets_user.shape[0]

    def __getitem__(self, i):
        song_id = self.triplets_user.iat[i, 1]
        user_idx = self.user_index[self.triplets_user.iat[i, 0]]
        y = torch.from_numpy(np.array(self.triplets_user.iat[i, 2])).float()
        return {'u': torch.tensor(user_idx), 'y': y, 'song_idx': self.songid2metaindex[song_id]}
