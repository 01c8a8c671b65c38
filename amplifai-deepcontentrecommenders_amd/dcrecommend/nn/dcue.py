"""DCUE trainer on MI355X: the reference's dcrecommend.nn.dcue.DCUE (nn/dcue.py:43-785).

Same constructor arguments and attributes, the same fit / score / score_song / predict /
predict_song / save / load / insert_best_factors / get_item_factors methods and the same
sub-epoch loop (10 shuffled chunks per epoch, a val pass, factors and AUC/mAP after each chunk,
best-by-val-mAP checkpoints), so a train script written against the reference runs unchanged.

What runs where:
* spectrograms are loaded ONCE into an HBM table (DCUEItemset.track_table) instead of 21
  torch.loads per row in DataLoader workers;
* per batch: catalogue negatives on the GPU (MT19937 continuing numpy's global stream, the
  reference's num_workers=0 draw order), then one TrainPlan step (forward, hinge, backward,
  NativeAdam, include/dcue.h dcue_plan_step) and the cyclic LR schedule;
* item / user factors through the eval towers (dcue_item_tower_eval, dcue_user_tower);
* AUC / mAP through dcue_rank_metrics (dcrecommend.nn.rank) instead of per-user pandas frames
  and sklearn calls.
The only host work per batch is the index permutation (torch RandomSampler, as the reference's
DataLoader(shuffle=True)) and the kernel launches. numpy's and torch's global random streams are
consumed as the reference consumes them with num_workers=0 loaders (negative draws continue numpy's
stream on the GPU; every DataLoader iteration's torch draws are mirrored), so a seeded fit follows
the reference's trajectory: tests/golden/fit.npz.
"""
import ctypes
import os

import numpy as np
import torch
from torch.utils.data import RandomSampler

from dcrecommend import _native as nat
from dcrecommend.datasets.csr import check_catalogue_users, saturated_users, user_split_ranks
from dcrecommend.dcue.dcue import DCUENet
from dcrecommend.dcue.plan import TrainPlan
from dcrecommend.nn import rank
from dcrecommend.nn.trainer import Trainer
from dcrecommend.optim import NativeAdam, NativeRanger, NativeSGD
from dcrecommend.optim.cyclic_scheduler import CyclicLRWithRestarts


def _dataset(x):
    """The reference passes DataLoaders around; accept a loader or its dataset."""
    return getattr(x, "dataset", x)


def _loader_draws(n):
    """The draws n DataLoader iterations take from torch's global RNG: each iterator draws a base
    seed (torch/utils/data/dataloader.py _BaseDataLoaderIter), so torch's stream -- and with it every
    later RandomSampler permutation -- stays where the reference's trainer leaves it."""
    for _ in range(n):
        torch.empty((), dtype=torch.int64).random_()


class _IndexBatches:
    """One sub-epoch loader (nn/dcue.py:711-721): the rows of a get_batches chunk in
    RandomSampler order (DataLoader(shuffle=True)), cut into batches, drop_last. Iterating takes the
    same two draws from torch's global RNG as the DataLoader: its base seed, then the sampler's."""

    def __init__(self, rows, batch_size):
        self.rows = np.asarray(rows, dtype=np.int64)
        self.batch_size = batch_size

    def __len__(self):
        return len(self.rows) // self.batch_size

    def __iter__(self):
        _loader_draws(1)
        order = np.fromiter(iter(RandomSampler(range(len(self.rows)))), dtype=np.int64, count=len(self.rows))
        rows = self.rows[order]
        B = self.batch_size
        for b in range(len(self)):
            yield rows[b * B:(b + 1) * B]


class _Negatives:
    """GPU catalogue sampler over one split (datasets/dcuedataset.py:207-220): the user -> split-rank
    CSR, the split's item list and the MT19937 stream on the device."""

    def __init__(self, ds, device):
        self.ds = ds
        self.device = device
        split = ds.split_items()
        coo = ds.item_user.tocoo()
        indptr, ranks = user_split_ranks(coo.col, coo.row, ds.n_users, split)
        self.split = torch.from_numpy(split).to(device)
        self.indptr = torch.from_numpy(indptr).to(device)
        self.ranks = torch.from_numpy(ranks if len(ranks) else np.zeros(1, np.int32)).to(device)
        self.reseed = ds.random_seed is not None
        self.seed = int(ds.random_seed) if self.reseed else 0
        self.saturated = saturated_users(indptr, len(split))  # usually empty

    def check(self, users):
        """ValueError (numpy's) before a batch whose user has no candidate negative is sampled."""
        if len(self.saturated):
            check_catalogue_users(users.cpu().numpy() if torch.is_tensor(users) else users, self.saturated)

    def draw(self, mt, users, N, out, stream=None):
        nat.check(nat.lib().dcue_sample_catalogue(
            None if self.reseed else nat.ptr(mt), int(self.reseed), self.seed, nat.ptr(self.split),
            self.split.numel(), nat.ptr(self.indptr), nat.ptr(self.ranks), nat.ptr(users), users.numel(), N,
            nat.ptr(out), nat.stream_handle(self.device) if stream is None else stream), "dcue_sample_catalogue")


def _mt_from_numpy(device):
    """numpy's global MT19937 state as a device dcue_mt_state (624 words + position)."""
    name, key, pos = np.random.get_state()[:3]
    buf = np.zeros(nat.MT_STATE_BYTES // 4, dtype=np.uint32)
    buf[:624] = key
    buf[624] = np.uint32(pos)
    return torch.from_numpy(buf.view(np.uint8).copy()).to(device)


def _mt_to_numpy(mt):
    """Continue numpy's global stream where the device stream stopped."""
    buf = mt.cpu().numpy().view(np.uint32)
    np.random.set_state(("MT19937", buf[:624].copy(), int(buf[624]), 0, 0.0))


class DCUE(Trainer):

    def __init__(self, feature_dim=100, conv_hidden=128, batch_size=64, neg_batch_size=20, u_embdim=300,
                 margin=0.2, optimize='adam', lr=0.00001, beta_one=0.9, beta_two=0.99, eps=1e-8,
                 weight_decay=0, restart_period=30, t_mult=2, num_epochs=90, model_type='truedcuemel1dbn',
                 eval_pct=0.025, val_pct=1.0, device=None, defer_embedding=True):
        """Arguments as nn/dcue.py:47-50; device (default cuda:current) and defer_embedding (the
        bit-identical deferred user-table Adam, dcrecommend.optim.NativeAdam) are MI355X additions."""
        Trainer.__init__(self)
        self.feature_dim = feature_dim
        self.conv_hidden = conv_hidden
        self.batch_size = batch_size
        self.neg_batch_size = neg_batch_size
        self.u_embdim = u_embdim
        self.margin = margin
        self.optimize = optimize
        self.lr = lr
        self.beta_one = beta_one
        self.beta_two = beta_two
        self.eps = eps
        self.weight_decay = weight_decay
        self.restart_period = restart_period
        self.t_mult = t_mult
        self.num_epochs = num_epochs
        self.model_type = model_type
        self.eval_pct = eval_pct
        self.val_pct = val_pct
        self.n_users = None
        self.n_items = None
        self.epoch_size = None
        self.model_dir = None
        self.train_data = self.val_data = self.test_data = None
        self.pred_data = self.truth_data = self.item_data = None
        self.model = None
        self.optimizer = None
        self.scheduler = None
        self.loss_func = None
        self.dict_args = None
        self.nn_epoch = 0
        self.item_factors = None
        self.user_factors = None
        self.best_item_factors = None
        self.best_user_factors = None
        self.best_val_map = 0
        self.best_val_auc = 0
        self.best_val_loss = float('inf')
        self.metadata_path = None
        self.triplets_path = None
        self.USE_CUDA = True
        self.device = torch.device(device if device is not None else "cuda")
        self.defer_embedding = defer_embedding
        self._tracks = None       # [n_items][131][128] HBM table, item-index order
        self._item_meta = None    # metadata index of every item index
        self._plan = None
        self._plan_n = None
        self._evals = {}

    # ------------------------------------------------------------------ model / optimizer
    def _init_nn(self, audio_model=None):
        self.dict_args = {'feature_dim': self.feature_dim, 'conv_hidden': self.conv_hidden,
                          'user_embdim': self.u_embdim, 'user_count': self.n_users,
                          'model_type': self.model_type}
        self.model = DCUENet(self.dict_args)
        if audio_model is not None:
            sd = self.model.state_dict()
            sd.update(audio_model)
            self.model.load_state_dict(sd)
        self.model = self.model.to(self.device)
        if self.optimize == 'adam':
            self.optimizer = NativeAdam(self.model.parameters(), self.lr, (self.beta_one, self.beta_two), self.eps,
                                        self.weight_decay, defer_embedding=self.defer_embedding)
        elif self.optimize == 'sgd':
            # nn/dcue.py:148-152; its StepLR(optimizer, 1, 1 - 1e-6) is replaced by the cyclic schedule
            # right after (:159) and never stepped, so it changes nothing
            self.optimizer = NativeSGD(self.model.parameters(), self.lr, self.beta_one,
                                       weight_decay=self.weight_decay, nesterov=True)
        elif self.optimize == 'ranger':
            self.optimizer = NativeRanger(self.model.parameters(), lr=self.lr, alpha=0.5, k=6, N_sma_threshhold=5,
                                          betas=(self.beta_one, self.beta_two), eps=1e-5,
                                          weight_decay=self.weight_decay)
        else:
            # the reference leaves self.optimizer None and its scheduler raises TypeError
            # (nn/dcue.py:159-162, optim/cyclic_scheduler.py)
            self.optimizer = None
        self.scheduler = CyclicLRWithRestarts(self.optimizer, self.batch_size, epoch_size=self.epoch_size,
                                              restart_period=self.restart_period, t_mult=self.t_mult,
                                              policy='cosine')
        self._plan = None

    def _loss_func(self, preds):
        """nn/dcue.py:167-170."""
        return torch.max(torch.zeros_like(preds), self.margin - preds).sum(dim=1).mean()

    # ------------------------------------------------------------------ device data
    def _bind_items(self, item_dataset):
        """Load the catalogue once: track table in item-index order, item -> metadata row map."""
        if self._tracks is not None and self._tracks_src is item_dataset:
            return
        meta = item_dataset.item_rows()
        table_meta = item_dataset.track_table(self.device, n_meta=max(len(item_dataset.songid2metaindex), 1))
        rows = torch.from_numpy(np.where(meta >= 0, meta, 0)).to(self.device)
        self._tracks = table_meta.index_select(0, rows).contiguous()
        self._item_meta = meta
        self._tracks_src = item_dataset

    def _n_neg(self, ds):
        """Negatives per row: the dataset's neg_samples, as in the reference, where the trainer's
        neg_batch_size is never read (datasets/dcuedataset.py:18,219)."""
        return int(getattr(ds, "neg_samples", self.neg_batch_size))

    def _train_plan(self, N):
        if self._plan is None or self._plan_n != N:
            self._plan = TrainPlan(self.model, self._tracks, self.batch_size, N,
                                   margin=self.margin, optimizer=self.optimizer)
            self._plan_n = N
        return self._plan

    # ------------------------------------------------------------------ epochs
    def _train_epoch(self, loader):
        """nn/dcue.py:172-218: per batch sample negatives, forward, hinge, backward, Adam, LR step.

        The reference draws each row's catalogue negatives in its DataLoader workers, ahead of the
        step that consumes them (datasets/dcuedataset.py:207-256). Here the batches' negatives are
        drawn two steps ahead on a sampling stream -- in batch order on the one numpy-compatible
        MT19937 stream, so the very same negatives -- and each batch's item list is built there too,
        so the plan also prepares the next batch's bn0 statistics beside the current step."""
        self.model.train()
        ds = loader.dataset if hasattr(loader, "dataset") else self.train_data
        neg = self._negatives(ds)
        B, N = self.batch_size, self._n_neg(ds)
        plan = self._train_plan(N)
        users_all, items_all = self._rows(ds)
        batches = list(loader)  # the loader's RNG draws happen when its iteration starts, as before
        dev = self.device
        main = torch.cuda.current_stream(dev)
        samp = torch.cuda.Stream(device=dev)
        mt = _mt_from_numpy(dev)
        users = [torch.empty(B, dtype=torch.int64, device=dev) for _ in range(3)]
        pos = [torch.empty(B, dtype=torch.int64, device=dev) for _ in range(3)]
        negs = [torch.empty((B, N), dtype=torch.int64, device=dev) for _ in range(3)]
        items = [torch.empty(B * (1 + N), dtype=torch.int32, device=dev) for _ in range(3)]
        ready = [torch.cuda.Event() for _ in range(3)]
        done = [torch.cuda.Event() for _ in range(3)]
        loss_sum = torch.zeros((), dtype=torch.float64, device=dev)
        samp.wait_stream(main)  # the sampler state and the row tables are written on the main stream

        def prepare(s):
            k = s % 3
            with torch.cuda.stream(samp):
                r = torch.from_numpy(batches[s]).to(dev)
                torch.index_select(users_all, 0, r, out=users[k])
                torch.index_select(items_all, 0, r, out=pos[k])
                neg.check(users[k])
                neg.draw(mt, users[k], N, negs[k], stream=samp.cuda_stream)
                nat.check(nat.lib().dcue_build_catalogue_batch(nat.ptr(pos[k]), nat.ptr(negs[k]), B, N,
                                                               nat.ptr(items[k]), samp.cuda_stream),
                          "dcue_build_catalogue_batch")
                ready[k].record(samp)

        n = len(batches)
        for s in range(min(2, n)):
            prepare(s)
        for s in range(n):
            main.wait_event(ready[min(s + 1, n - 1) % 3])  # this batch and the next one are built
            if s + 1 < n:
                plan.set_next(items[(s + 1) % 3])
            plan.step(users[s % 3], items[s % 3])
            self.scheduler.batch_step()
            loss_sum += plan.loss.double() * B
            done[s % 3].record(main)
            if s + 2 < n:  # buffers (s+2) % 3 were batch s-1's
                if s >= 1:
                    samp.wait_event(done[(s - 1) % 3])
                prepare(s + 2)
        main.wait_stream(samp)
        _mt_to_numpy(mt)
        return n * B, float(loss_sum) / max(n * B, 1)

    def _eval_epoch(self, loader):
        """nn/dcue.py:220-262: eval-mode loss over the val set in order (last batch partial)."""
        _loader_draws(1)  # DataLoader(shuffle=False): its iterator's base seed
        self.model.eval()
        ds = _dataset(loader)
        neg = self._negatives(ds)
        users_all, items_all = self._rows(ds)
        B, N = self.batch_size, self._n_neg(ds)
        mt = _mt_from_numpy(self.device)
        loss_sum = torch.zeros((), dtype=torch.float64, device=self.device)
        n = users_all.numel()
        for s in range(0, n, B):
            users = users_all[s:s + B].contiguous()
            b = users.numel()
            negs = torch.empty((b, N), dtype=torch.int64, device=self.device)
            neg.check(users)
            neg.draw(mt, users, N, negs)
            track = torch.empty(b * (1 + N), dtype=torch.int32, device=self.device)
            nat.check(nat.lib().dcue_build_catalogue_batch(nat.ptr(items_all[s:s + B].contiguous()), nat.ptr(negs),
                                                           b, N, nat.ptr(track), nat.stream_handle()),
                      "dcue_build_catalogue_batch")
            _, _, _, loss = self.model.native_forward(users, self._tracks, track, N, nat.LAYOUT_CATALOGUE,
                                                      train=False, margin=self.margin, copy_outputs=False)
            loss_sum += loss.double() * b
        _mt_to_numpy(mt)
        return n, float(loss_sum) / max(n, 1)

    def _negatives(self, ds):
        key = ("neg", id(ds))
        if key not in self._evals:
            self._evals[key] = _Negatives(ds, self.device)
        return self._evals[key]

    def _rows(self, ds):
        key = ("rows", id(ds), len(ds))
        if key not in self._evals:
            u, s = ds.split_rows()
            self._evals[key] = (torch.from_numpy(u).to(self.device), torch.from_numpy(s).to(self.device))
        return self._evals[key]

    def _batch_loaders(self, dataset, k=None):
        """nn/dcue.py:711-721: get_batches chunks, each a shuffled drop_last loader."""
        loaders = []
        for chunk in dataset.get_batches(k):
            it = _IndexBatches(chunk, self.batch_size)
            it.dataset = dataset
            loaders.append(it)
        return loaders

    # ------------------------------------------------------------------ fit
    def fit(self, train_dataset, val_dataset, test_dataset, pred_dataset, truth_dataset, item_dataset,
            n_users, n_items, triplets_path, metadata_path, save_dir, warm_start=False, audio_model=None):
        """nn/dcue.py:264-378 (same loop, same prints, same checkpoint policy)."""
        print("Settings:\n Feature Dim: {}\n Conv Dim: {}\n User Embedding Dim: {}\n Batch Size: {}\n "
              "Negative Batch Size: {}\n Margin: {}\n Optimizer: {}\n Learning Rate: {}\n Weight Decay: {}\n "
              "Restart Period: {}\n T Multiplier: {}\n Num Epochs: {}\n Model Type: {}\n Num Users: {}\n "
              "Num Items: {}\n Triplets TXT: {}\n Metadata CSV: {}\n Save Dir: {}".format(
                  self.feature_dim, self.conv_hidden, self.u_embdim, self.batch_size, self.neg_batch_size,
                  self.margin, self.optimize, self.lr, self.weight_decay, self.restart_period, self.t_mult,
                  self.num_epochs, self.model_type, n_users, n_items, triplets_path, metadata_path, save_dir),
              flush=True)
        self.epoch_size = int(int(np.ceil(len(train_dataset) / 10)) // self.batch_size) * self.batch_size
        self.n_users, self.n_items = n_users, n_items
        self.triplets_path, self.metadata_path = triplets_path, metadata_path
        self.model_dir = save_dir
        self.train_data, self.val_data, self.test_data = train_dataset, val_dataset, test_dataset
        self.pred_data, self.truth_data, self.item_data = pred_dataset, truth_dataset, item_dataset
        val_dataset.subset(p=self.val_pct)
        if not warm_start:
            self._init_nn(audio_model)
        self._bind_items(item_dataset)
        train_loss, samples_processed = 0, 0
        while self.nn_epoch < self.num_epochs + 1:
            for train_loader in self._batch_loaders(train_dataset, k=10):
                if self.nn_epoch > 0:
                    self.scheduler.step()
                    print("\nInitializing train epoch...", flush=True)
                    sp, train_loss = self._train_epoch(train_loader)
                    samples_processed += sp
                print("\nInitializing val epoch...", flush=True)
                _, val_loss = self._eval_epoch(val_dataset)
                print("\nInitializing AUC computation...", flush=True)
                self._user_factors(item_dataset)
                self._item_factors(item_dataset)
                val_auc, val_map = self._compute_scores('val', pred_dataset, truth_dataset, train_dataset,
                                                        val_dataset, test_dataset, pct=self.eval_pct)
                val_user_auc, val_user_map = self._compute_scores_song(pred_dataset, pct=self.eval_pct)
                train_auc, train_map = self._compute_scores('train', truth_dataset, truth_dataset, train_dataset,
                                                            val_dataset, test_dataset, pct=self.eval_pct)
                print("\nEpoch: [{}/{}]\tSamples: [{}/{}]\tTrain Loss: {}\tVal Loss: {}\tTrain AUC: {}\t"
                      "Val AUC: {}\tTrain mAP: {}\tVal mAP: {}\tVal UAUC: {}\tVal UmAP: {}".format(
                          self.nn_epoch, self.num_epochs, samples_processed, len(train_dataset) * self.num_epochs,
                          train_loss, val_loss, train_auc, val_auc, train_map, val_map, val_user_auc,
                          val_user_map), flush=True)
                self._update_best(val_map, val_auc, val_loss)
                self.nn_epoch += 1

    # ------------------------------------------------------------------ factors
    def _user_factors(self, item_data):
        """nn/dcue.py:629-638: eval user tower for every user index (one batched call)."""
        self.model.eval()
        self.model._require_device()
        self.user_factors = torch.zeros([self.n_users, self.feature_dim], device=self.device)
        idx = torch.as_tensor(np.fromiter(item_data.user_index.values(), dtype=np.int64)).to(self.device)
        step = 65536
        # the towers write rows at the storage width d_s (zero past d; include/dcue.h)
        ds = nat.storage_dims(self.model._flat["dims"]).feature_dim
        feat = torch.empty((min(step, max(idx.numel(), 1)), ds), device=self.device)
        model = self.model._model_struct()
        for s in range(0, idx.numel(), step):
            part = idx[s:s + step].contiguous()
            n = part.numel()
            ws = self._factor_ws(n, 1)
            nat.check(nat.lib().dcue_user_tower(ctypes.byref(model), nat.ptr(part), n, nat.ptr(ws), ws.numel(),
                                                nat.ptr(feat), nat.stream_handle()), "dcue_user_tower")
            self.user_factors.index_copy_(0, part, feat[:n, :self.feature_dim])

    def _factor_ws(self, rows, items):
        """Workspace of the factor passes, apart from the model's (a TrainPlan binds that one)."""
        nbytes = nat.workspace_bytes(self.model._flat["dims"], rows, 0, items)
        if getattr(self, "_fws", None) is None or self._fws.numel() < nbytes:
            self._fws = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        return self._fws

    def _item_factors(self, item_data, n_iter=10):
        """nn/dcue.py:640-668: [len(songid2metaindex), d], rows of the set's tracks = eval conv
        summed n_iter times / n_iter (identical passes for 131-frame tracks)."""
        self.item_factors = self._factors_over(item_data, n_iter)

    def get_item_factors(self, loader, n_iter=1):
        """nn/dcue.py:670-694."""
        return self._factors_over(_dataset(loader), n_iter)

    def _factors_over(self, item_data, n_iter):
        _loader_draws(n_iter)  # the reference iterates its item loader n_iter times
        self._bind_items(item_data)
        self.model.eval()
        self.model._require_device()
        n_meta = len(item_data.songid2metaindex)
        out = torch.zeros([n_meta, self.feature_dim], device=self.device)
        items = np.nonzero(self._item_meta >= 0)[0].astype(np.int32)
        if len(items):
            step = 8192
            ds = nat.storage_dims(self.model._flat["dims"]).feature_dim
            feat = torch.empty((min(step, len(items)), ds), device=self.device)
            tr = nat.Tracks(self._tracks.data_ptr(), self._tracks.shape[0],
                            0 if self._tracks.dtype == torch.float16 else 1, 0)
            model = self.model._model_struct()
            for s in range(0, len(items), step):
                it = torch.from_numpy(items[s:s + step]).to(self.device)
                n = it.numel()
                ws = self._factor_ws(1, n)
                nat.check(nat.lib().dcue_item_tower_eval(ctypes.byref(model), ctypes.byref(tr), nat.ptr(it), n,
                                                         nat.ptr(ws), ws.numel(), nat.ptr(feat), nat.stream_handle()),
                          "dcue_item_tower_eval")
                rows = torch.from_numpy(self._item_meta[items[s:s + step]]).to(self.device)
                out.index_copy_(0, rows, feat[:n, :self.feature_dim])
            nat.check(nat.lib().dcue_factor_repeat_mean(nat.ptr(out), out.numel(), int(n_iter), nat.stream_handle()),
                      "dcue_factor_repeat_mean")
        return out

    def _item_feat_by_index(self):
        """item factors in item-index order (the evaluator's candidate rows)."""
        rows = torch.from_numpy(np.where(self._item_meta >= 0, self._item_meta, 0)).to(self.device)
        f = self.item_factors.index_select(0, rows)
        f[torch.from_numpy(self._item_meta < 0).to(self.device)] = 0
        return f

    # ------------------------------------------------------------------ scoring
    def _evaluator(self, kind, pred_ds, truth_ds=None):
        key = (kind, id(pred_ds), id(truth_ds))
        if key not in self._evals:
            inputs = (rank.user_split_inputs(pred_ds, truth_ds) if kind == "user" else rank.song_inputs(pred_ds))
            self._evals[key] = rank.RankEvaluator(inputs, self.device)
        return self._evals[key]

    def score_users(self, user_idx, pred_dataset, truth_dataset):
        """Per-user (auc, ap, has_pred_songs) arrays for user indices (the GPU core of score())."""
        ev = self._evaluator("user", pred_dataset, truth_dataset)
        return ev.metrics(self.user_factors, self._item_feat_by_index(), user_idx, nat.RANK_SPLIT)

    def score(self, users, pred_loader, truth_loader, k=10000):
        """nn/dcue.py:380-449: mean split-weighted AUC and mAP over `users` (user ids)."""
        self.model.eval()
        pred, truth = _dataset(pred_loader), _dataset(truth_loader)
        idx = np.array([pred.user_index[u] for u in users], dtype=np.int64)
        auc, ap, ok = self.score_users(idx, pred, truth)
        # torch-RNG parity: the reference iterates a shuffling loader per predict() call that finds
        # songs (base seed + sampler seed), for every user up to and including the one it stops at
        in_pred, in_truth = set(pred.triplets['user_id']), set(truth.triplets['user_id'])
        stop = int(np.argmin(ok)) + 1 if not ok.all() else len(users)
        _loader_draws(sum(2 * ((u in in_pred) + (u in in_truth)) for u in list(users)[:stop]))
        return rank.mean_until_missing(auc, ok), rank.mean_until_missing(ap, ok)

    def score_song(self, songs, pred_loader, k=10000):
        """nn/dcue.py:451-476: mean AUC and AP over `songs` (song ids); songs without users are
        skipped."""
        self.model.eval()
        pred = _dataset(pred_loader)
        idx = np.array([pred.item_index[s] for s in songs], dtype=np.int64)
        ev = self._evaluator("song", pred)
        auc, ap, ok = ev.metrics(self._item_feat_by_index(), self.user_factors, idx, nat.RANK_SINGLE)
        _loader_draws(2 * int(ok.sum()))  # one shuffling loader pass per song with users
        return float(np.mean(auc[ok])), float(np.mean(ap[ok]))

    def predict(self, user, loader):
        """nn/dcue.py:478-519: (scores, targets) over the user's pred-split candidate list, in the
        reference's order (the user's split triplets, then the other split songs by item index)."""
        ds = _dataset(loader)
        u = ds.user_index[user]
        pos = [ds.item_index[s] for s in ds.triplets.loc[ds.triplets['user_id'] == user, 'song_id']]
        if not pos:
            return None, None
        inter = set(ds.item_user.getcol(u).nonzero()[0].tolist())
        rest = [i for i in ds.split_items().tolist() if i not in inter]
        return self._sim_list(self.user_factors[u], pos + rest, [1] * len(pos) + [0] * len(rest), items=True)

    def predict_song(self, song, loader):
        """nn/dcue.py:521-562 (with the reference's non-user list: every split user but user 0)."""
        ds = _dataset(loader)
        i = ds.item_index[song]
        pos = [ds.user_index[x] for x in ds.triplets.loc[ds.triplets['song_id'] == song, 'user_id']]
        if not pos:
            return None, None
        rest = [u for u in ds.split_users().tolist() if u != 0]
        feat = self._item_feat_by_index()[i]
        return self._sim_list(feat, pos + rest, [1] * len(pos) + [0] * len(rest), items=False)

    def _sim_list(self, q, cands, targets, items):
        idx = torch.as_tensor(cands, dtype=torch.int64, device=self.device)
        rows = (self._item_feat_by_index() if items else self.user_factors).index_select(0, idx)
        with torch.no_grad():
            s = self.model.sim(q.unsqueeze(0).expand_as(rows), rows)
        return s.cpu().numpy().tolist(), [float(t) for t in targets]

    def _compute_scores(self, split, pred_loader, truth_loader, train_data, val_data, test_data, pct=0.025):
        """nn/dcue.py:580-603."""
        if split == 'train':
            users = list(train_data.uniq_users)
        elif split == 'val':
            users = list(set(train_data.uniq_users).intersection(set(val_data.uniq_users)))
        elif split == 'test':
            users = list(set(train_data.uniq_users).intersection(set(test_data.uniq_users)))
        else:
            raise ValueError(split)
        sample = np.random.choice(users, int(len(users) * pct)) if pct < 1 else users
        return self.score(sample, pred_loader, truth_loader)

    def _compute_scores_song(self, pred_loader, pct=0.025):
        """nn/dcue.py:605-613."""
        songs = list(_dataset(pred_loader).uniq_songs)
        sample = np.random.choice(songs, int(len(songs) * pct)) if pct < 1 else songs
        return self.score_song(sample, pred_loader)

    # ------------------------------------------------------------------ bookkeeping
    def insert_best_factors(self):
        self.item_factors = self.best_item_factors
        self.user_factors = self.best_user_factors

    def _update_best(self, val_map, val_auc, val_loss):
        """nn/dcue.py:564-578: keep the best-by-val-mAP factors; checkpoint then, or every 5th."""
        if val_map > self.best_val_map:
            self.best_val_map, self.best_val_auc, self.best_val_loss = val_map, val_auc, val_loss
            if self.best_item_factors is None or self.best_user_factors is None:
                self.best_item_factors = torch.zeros_like(self.item_factors)
                self.best_user_factors = torch.zeros_like(self.user_factors)
            self.best_item_factors.copy_(self.item_factors)
            self.best_user_factors.copy_(self.user_factors)
            self.save(models_dir=self.model_dir)
        elif self.nn_epoch % 5 == 0:
            self.save(models_dir=self.model_dir)

    def _format_model_subdir(self):
        return ("DCUE_fd_{}_ch_{}_uh_{}_op_{}_lr_{}_wd_{}_rp_{}_tm_{}_nu_{}_ni_{}_mt_{}".format(
            self.feature_dim, self.conv_hidden, self.u_embdim, self.optimize, self.lr, self.weight_decay,
            self.restart_period, self.t_mult, self.n_users, self.n_items, self.model_type))

    _SCALARS = ("feature_dim", "conv_hidden", "batch_size", "neg_batch_size", "u_embdim", "margin", "optimize",
                "lr", "beta_one", "beta_two", "eps", "weight_decay", "restart_period", "t_mult", "num_epochs",
                "model_type", "eval_pct", "val_pct", "n_users", "n_items", "epoch_size", "nn_epoch",
                "best_val_map", "best_val_auc", "best_val_loss", "metadata_path", "triplets_path", "model_dir",
                "defer_embedding")
    _TENSORS = ("item_factors", "user_factors", "best_item_factors", "best_user_factors")

    def _checkpoint(self):
        out = {k: getattr(self, k) for k in self._SCALARS}
        out.update({k: (None if getattr(self, k) is None else getattr(self, k).cpu()) for k in self._TENSORS})
        out["model"] = {k: v.cpu() for k, v in self.model.state_dict().items()}
        opt = self.optimizer.state_dict()
        mom = opt["native"]["moments"]
        out["optimizer"] = {"step": opt["native"]["step"],
                            "moments": None if mom is None else {k: v.cpu() for k, v in mom.items()}}
        out["scheduler"] = {k: v for k, v in self.scheduler.__dict__.items()
                            if isinstance(v, (int, float, bool, str)) or v is None}
        return out

    def save(self, models_dir=None):
        """nn/dcue.py:723-741: models_dir/<subdir>/epoch_{n}.pth. The file holds tensors and plain
        values only (torch.load(weights_only=True) reads it); the reference pickles the trainer."""
        if self.model is None or models_dir is None:
            return
        d = os.path.join(models_dir, self._format_model_subdir())
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "epoch_{}.pth".format(self.nn_epoch)), 'wb') as f:
            torch.save(self._checkpoint(), f)

    def load(self, model_dir, epoch):
        """nn/dcue.py:743-785: restore attributes, model, optimizer and scheduler; nn_epoch + 1."""
        with open(os.path.join(model_dir, "epoch_{}.pth".format(epoch)), 'rb') as f:
            ck = torch.load(f, map_location="cpu", weights_only=True)
        for k in self._SCALARS:
            if k in ck:
                setattr(self, k, ck[k])
        self._init_nn()
        self.model.load_state_dict(ck["model"])
        for k in self._TENSORS:
            setattr(self, k, None if ck.get(k) is None else ck[k].to(self.device))
        opt = ck["optimizer"]
        moments = None if opt["moments"] is None else {k: v.to(self.device) for k, v in opt["moments"].items()}
        base = self.optimizer.state_dict()
        base["native"] = dict(step=opt["step"], moments=moments)
        self.optimizer.load_state_dict(base)
        self.scheduler.__dict__.update(ck["scheduler"])
        self.nn_epoch += 1
