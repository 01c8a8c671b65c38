"""Generate the golden parity fixtures by running the REFERENCE (dcrecommend) on CPU.

Run in the build container only (the reference never travels to the GPU box):

    PYTHONPATH=/root/reference PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Every fixture is data (inputs + the reference's outputs); no reference source is stored.
Which reference code produced what:

* model_*.npz   -- dcrecommend/dcue/dcue.py:21-108 (DCUENet fwd), nn/dcue.py:167-170 (hinge loss),
                   torch autograd backward, torch.optim.Adam as built at nn/dcue.py:143-147;
                   model_{plain,res,resbn}.npz the same for the other wired towers
                   (audiomodels/truedcuemel1d.py, truedcuemel1dres.py, truedcuemel1dresbn.py);
                   model_d100.npz at the trainer's default widths (feature_dim=100, conv_hidden=128,
                   nn/dcue.py:44-45), model_w_*.npz at odd H / d in the other towers.
* inbatch_*.npz -- the in-batch sampler spec of nn/dcue.py:698-709 (commented out in the reference;
                   the draws below follow that text literally), plus a forward/backward of the
                   reference model on the duplicated [pos; neg] batch it builds.
* catalogue.npz -- DCUEDataset._user_nonitem_songids (datasets/dcuedataset.py:207-220) under both
                   RNG protocols (random_seed set -> reseed per sample :167-168; global stream).
* batches.npz   -- DCUEDataset.get_batches (datasets/dcuedataset.py:189-201).
* scheduler.npz -- CyclicLRWithRestarts (optim/cyclic_scheduler.py:49-215) driven the way
                   DCUE.fit/_train_epoch drive it (nn/dcue.py:338-341, 209-210).
* train5.npz    -- five DCUE train steps (nn/dcue.py:202-210) with Adam + scheduler.
* fit.npz       -- DCUE.fit for one epoch (10 sub-epochs) with num_workers=0 loaders: per sub-epoch
                   train / val loss and AUC / mAP, final parameters.
* eval.npz      -- the evaluation path end to end: DCUE._user_factors / _item_factors over
                   DCUEItemset, DCUE.score (val and train splits, DCUEPredset) and score_song.
* metrics.npz   -- DCUE.score's split-weighted AUC / mAP arithmetic (nn/dcue.py:399-449) and
                   score_song's (nn/dcue.py:463-476), on fixed score vectors.
* optim.npz     -- the trainer's other optimizers as DCUE._init_nn builds them (nn/dcue.py:148-157):
                   the reference's Ranger (optim/ranger.py:26-165, RAdam + Lookahead, k=6, alpha=0.5,
                   N_sma_threshhold=5, eps=1e-5) and torch.optim.SGD(momentum=beta_one, nesterov=True),
                   13 steps on fixed gradients with a changing lr, every step's parameters and state.
"""
import os
import sys

import numpy as np
import pandas as pd
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("DCUE_REFERENCE", "/root/reference")
if REF not in sys.path:
    sys.path.insert(0, REF)

from dcrecommend.dcue.dcue import DCUENet  # noqa: E402  (reference)
from dcrecommend.nn.dcue import DCUE  # noqa: E402  (reference)
from dcrecommend.datasets.dcuedataset import DCUEDataset  # noqa: E402  (reference)
from dcrecommend.optim.cyclic_scheduler import CyclicLRWithRestarts  # noqa: E402  (reference)

torch.set_num_threads(8)


def _spectros(gen, *shape):
    """Synthetic spectrograms, rounded to fp16-representable values."""
    return torch.randn(*shape, generator=gen).half().float()


def _state(model):
    return {k: v.detach().clone() for k, v in model.state_dict().items()}


def _save(name, **arrays):
    path = os.path.join(HERE, name)
    out = {}
    for k, v in arrays.items():
        if isinstance(v, torch.Tensor):
            v = v.detach().cpu().numpy()
        out[k] = np.asarray(v)
    np.savez_compressed(path, **out)
    print("wrote", path, sum(a.nbytes for a in out.values()) // 1024, "KiB raw")


def model_fixture(name, H, d, n_users, B, N, lr=1e-3, store_init=True, store_steps=True, seed=0,
                  model_type="truedcuemel1dbn"):
    """fwd (train) -> hinge -> bwd -> Adam(lr) step -> Adam(lr, wd=1e-4) step -> eval fwd."""
    torch.manual_seed(seed)
    net = DCUENet({"feature_dim": d, "conv_hidden": H, "user_embdim": 300,
                   "user_count": n_users, "model_type": model_type})
    init = _state(net)
    gen = torch.Generator().manual_seed(seed + 1)
    u = torch.randint(0, n_users, (B,), generator=gen)
    pos = _spectros(gen, B, 128, 131)
    neg = _spectros(gen, B, N, 128, 131)
    trainer = DCUE(feature_dim=d, conv_hidden=H, batch_size=B, margin=0.2)

    net.train()
    net.zero_grad()
    scores, uf, pf, nf = net(u, pos, neg)
    loss = trainer._loss_func(scores)
    loss.backward()
    grads = {"grad." + n: p.grad.detach().clone() for n, p in net.named_parameters()}
    after_fwd = _state(net)  # running stats updated by the train-mode forward

    opt = torch.optim.Adam(net.parameters(), lr, (0.9, 0.99), 1e-8, 0)
    opt.step()
    step1 = {"step1." + k: v for k, v in _state(net).items()}
    # second step, same grads, weight decay on (exercises Adam's grad += wd * p)
    for g in opt.param_groups:
        g["weight_decay"] = 1e-4
    opt.step()
    step2 = {"step2." + k: v for k, v in _state(net).items()}

    net.eval()
    with torch.no_grad():
        e_scores, e_uf, e_pf, e_nf = net(u, pos, neg)

    payload = dict(H=H, d=d, n_users=n_users, B=B, N=N, lr=lr, seed=seed, model_type=model_type,
                   u=u, pos=pos.half(), neg=neg.half(),
                   scores=scores, uf=uf, pf=pf, nf=nf, loss=loss,
                   eval_scores=e_scores, eval_uf=e_uf, eval_pf=e_pf, eval_nf=e_nf)
    payload.update(grads)
    payload.update({"fwd." + k: v for k, v in after_fwd.items() if "running" in k or "num_batches" in k})
    if store_steps:
        payload.update(step1)
        payload.update(step2)
    if store_init:
        payload.update({"init." + k: v for k, v in init.items()})
    else:
        payload.update({"initsum." + k: v.double().sum() for k, v in init.items()})
        payload.update({"initsq." + k: (v.double() ** 2).sum() for k, v in init.items()})
    _save(name, **payload)


def inbatch_draws(B, N, seed):
    """nn/dcue.py:698-709 text: for i<B, j<N: rand_idx = np.random.choice([0..i-1, i+1..B-1])."""
    np.random.seed(seed)
    r = np.zeros((B, N), dtype=np.int64)
    for i in range(B):
        indexes = [x for x in range(0, i)] + [x for x in range(i + 1, B)]
        for j in range(N):
            r[i, j] = np.random.choice(indexes)
    return r


def inbatch_fixtures():
    seeds = [0, 5, 99]
    draws = {"seed%d" % s: inbatch_draws(64, 20, s) for s in seeds}
    draws.update({"small_seed3": inbatch_draws(8, 5, 3)})
    _save("inbatch_draws.npz", **draws)

    # model-level: negatives are copies of in-batch positives (the reference conv runs on the
    # duplicated [pos; neg] stack, so BN statistics count each copy).
    H, d, n_users, B, N = 32, 32, 10, 8, 5
    torch.manual_seed(0)
    net = DCUENet({"feature_dim": d, "conv_hidden": H, "user_embdim": 300,
                   "user_count": n_users, "model_type": "truedcuemel1dbn"})
    gen = torch.Generator().manual_seed(11)
    u = torch.randint(0, n_users, (B,), generator=gen)
    pos = _spectros(gen, B, 128, 131)
    r = torch.from_numpy(draws["small_seed3"])
    neg = pos[r.reshape(-1)].reshape(B, N, 128, 131).clone()
    trainer = DCUE(feature_dim=d, conv_hidden=H, batch_size=B, margin=0.2)
    net.train()
    net.zero_grad()
    scores, uf, pf, nf = net(u, pos, neg)
    loss = trainer._loss_func(scores)
    loss.backward()
    payload = dict(H=H, d=d, n_users=n_users, B=B, N=N, u=u, pos=pos.half(), r=r,
                   scores=scores, uf=uf, pf=pf, nf=nf, loss=loss)
    payload.update({"grad." + n: p.grad for n, p in net.named_parameters()})
    payload.update({"fwd." + k: v for k, v in _state(net).items() if "running" in k})
    _save("inbatch_model.npz", **payload)


def _synthetic_triplets(n_users, n_tracks, n_pairs, seed):
    rs = np.random.RandomState(seed)
    pairs = set()
    while len(pairs) < n_pairs:
        pairs.add((int(rs.randint(n_users)), int(rs.randint(n_tracks))))
    pairs = sorted(pairs)
    users = ["u%05d" % p[0] for p in pairs]
    songs = ["S%07d" % p[1] for p in pairs]
    score = rs.randint(1, 10, size=len(pairs))
    order = rs.permutation(len(pairs))
    return pd.DataFrame({"user_id": np.array(users)[order], "song_id": np.array(songs)[order],
                         "score": score[order]})


def catalogue_fixture():
    n_users, n_tracks, n_pairs, N = 40, 60, 600, 7
    trip = _synthetic_triplets(n_users, n_tracks, n_pairs, 0)
    raw_users = trip["user_id"].to_numpy().astype(str)
    raw_songs = trip["song_id"].to_numpy().astype(str)
    raw_score = trip["score"].to_numpy()
    meta = pd.DataFrame({"song_id": sorted(set(raw_songs)), "data_mel": ""})
    ds = DCUEDataset(trip.copy(), meta, neg_samples=N, split="train")
    split_items = np.array(sorted(ds.uniq_song_idxs), dtype=np.int64)
    # the CSR over all interactions, as item indices per user index
    users_seq = np.random.RandomState(42).randint(0, len(ds.user_index), size=50)
    userids = [ds.userindex2userid[int(i)] for i in users_seq]

    def codes(songs):
        return np.array([ds.item_index[s] for s in songs], dtype=np.int64)

    # (1) random_seed=S protocol: the RNG is reseeded before every sample (dcuedataset.py:167-168)
    seeded = []
    for uid in userids:
        np.random.seed(1234)
        seeded.append(codes(ds._user_nonitem_songids(uid)))
    # (2) global-stream protocol: one np.random.seed then draws in sampler order
    np.random.seed(77)
    stream = [codes(ds._user_nonitem_songids(uid)) for uid in userids]
    _save("catalogue.npz", raw_users=raw_users, raw_songs=raw_songs, raw_score=raw_score,
          n_items=ds.n_items, n_users=ds.n_users, N=N,
          user_categories=np.array(list(ds.user_index.keys())).astype(str),
          song_categories=np.array(list(ds.item_index.keys())).astype(str),
          split_items=split_items, users_seq=users_seq,
          seeded=np.stack(seeded), stream=np.stack(stream), train_len=len(ds),
          train_users=np.array([ds.user_index[x] for x in ds.triplets["user_id"]], dtype=np.int64),
          train_songs=np.array([ds.item_index[x] for x in ds.triplets["song_id"]], dtype=np.int64))


class _Len:
    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n


def batches_fixture():
    out = {}
    for n, seed in [(95, 0), (100, 1), (1003, 2), (7, 3)]:
        np.random.seed(seed)
        chunks = DCUEDataset.get_batches(_Len(n), k=10)
        out["n%d_lens" % n] = np.array([len(c) for c in chunks], dtype=np.int64)
        out["n%d_flat" % n] = np.array([x for c in chunks for x in c], dtype=np.int64)
    _save("batches.npz", **out)


def scheduler_fixture():
    out = {}
    for tag, (B, n_train, period, t_mult, base_wd) in {
            "a": (64, 6400, 2, 2, 0.0), "b": (32, 1000, 3, 1.5, 1e-3)}.items():
        p = torch.nn.Parameter(torch.zeros(1))
        opt = torch.optim.Adam([p], 1e-3, (0.9, 0.99), 1e-8, base_wd)
        epoch_size = int(int(np.ceil(n_train / 10)) // B) * B  # nn/dcue.py:302-303
        sch = CyclicLRWithRestarts(opt, B, epoch_size=epoch_size, restart_period=period,
                                   t_mult=t_mult, policy="cosine")
        chunk = int(np.ceil(n_train / 10))
        nb = chunk // B  # DataLoader(drop_last=True) over one get_batches chunk
        lrs, wds = [], []
        for sub in range(20):
            sch.step()
            for _ in range(nb):
                lrs.append(opt.param_groups[0]["lr"])
                wds.append(opt.param_groups[0]["weight_decay"])
                sch.batch_step()
        # overrun: the reference raises StopIteration once the increments run out
        sch.step()
        raised = 0
        try:
            for _ in range(nb + 5):
                sch.batch_step()
        except StopIteration:
            raised = 1
        out[tag + "_cfg"] = np.array([B, n_train, period, t_mult, base_wd, epoch_size, nb], dtype=np.float64)
        out[tag + "_lr"] = np.array(lrs)
        out[tag + "_wd"] = np.array(wds)
        out[tag + "_raised"] = np.array(raised)
    _save("scheduler.npz", **out)


def train5_fixture():
    H, d, n_users, B, N = 32, 32, 12, 4, 3
    torch.manual_seed(0)
    trainer = DCUE(feature_dim=d, conv_hidden=H, batch_size=B, margin=0.2, lr=1e-3,
                   restart_period=2, t_mult=2)
    trainer.n_users = n_users
    trainer.epoch_size = 5 * B
    trainer.USE_CUDA = False
    trainer._init_nn()
    gen = torch.Generator().manual_seed(5)
    us, poss, negs, losses, lrs = [], [], [], [], []
    trainer.model.train()
    trainer.scheduler.step()
    for _ in range(5):
        u = torch.randint(0, n_users, (B,), generator=gen)
        pos = _spectros(gen, B, 128, 131)
        neg = _spectros(gen, B, N, 128, 131)
        lrs.append(trainer.optimizer.param_groups[0]["lr"])
        trainer.model.zero_grad()
        preds, _, _, _ = trainer.model(u, pos, neg)
        loss = trainer._loss_func(preds)
        loss.backward()
        trainer.optimizer.step()
        trainer.scheduler.batch_step()
        us.append(u)
        poss.append(pos.half())
        negs.append(neg.half())
        losses.append(loss.item())
    payload = dict(H=H, d=d, n_users=n_users, B=B, N=N, u=torch.stack(us), pos=torch.stack(poss),
                   neg=torch.stack(negs), loss=np.array(losses), lr=np.array(lrs))
    payload.update({"final." + k: v for k, v in _state(trainer.model).items()})
    _save("train5.npz", **payload)


def metrics_fixture():
    """The AUC/mAP arithmetic of DCUE.score / score_song on fixed vectors (sklearn underneath)."""
    from sklearn.metrics import roc_auc_score, average_precision_score
    rs = np.random.RandomState(3)
    cases = []
    for n in [5, 17, 40]:
        sp = np.round(rs.rand(n), 2)  # rounding creates ties (sklearn tie semantics)
        tp = (rs.rand(n) < 0.3).astype(np.int64)
        st = np.round(rs.rand(n + 3), 2)
        tt = (rs.rand(n + 3) < 0.5).astype(np.int64)
        cases.append((sp, tp, st, tt))
    out = {}
    for c, (sp, tp, st, tt) in enumerate(cases):
        out["c%d_sp" % c], out["c%d_tp" % c], out["c%d_st" % c], out["c%d_tt" % c] = sp, tp, st, tt
        out["c%d_auc" % c] = roc_auc_score(tp, sp) if 0 < tp.sum() < len(tp) else np.nan
        out["c%d_ap" % c] = average_precision_score(tp, sp)
    _save("metrics.npz", **out)


def eval_fixture():
    """DCUE's evaluation path end to end (nn/dcue.py:380-476, 629-668; datasets/dcuepredset.py,
    dcueitemset.py): factors from a small eval-mode model over torch.save'd spectrograms, then
    per-user split-weighted AUC / mAP (val and train) and per-song AUC / AP."""
    import tempfile
    from torch.utils.data import DataLoader
    from dcrecommend.datasets.dcuepredset import DCUEPredset  # reference
    from dcrecommend.datasets.dcueitemset import DCUEItemset  # reference
    n_users, n_tracks, n_pairs, H, d = 30, 48, 420, 32, 32
    trip = _synthetic_triplets(n_users, n_tracks, n_pairs, 11)
    songs = sorted(set(trip["song_id"]))
    # metadata rows in a shuffled order: metadata index != item (category) index
    meta_order = np.random.RandomState(5).permutation(len(songs))
    meta_songs = [songs[i] for i in meta_order]
    gen = torch.Generator().manual_seed(21)
    spec = _spectros(gen, len(songs), 128, 131)
    # two tracks share one spectrogram: identical factors -> exact score ties across items
    spec[7] = spec[3]
    tmp = tempfile.mkdtemp()
    paths = []
    for k in range(len(songs)):
        p = os.path.join(tmp, "t%03d.pt" % k)
        torch.save(spec[k].clone(), p)
        paths.append(p)
    meta = pd.DataFrame({"idx": np.arange(len(songs)), "song_id": meta_songs, "data_mel": paths})
    train = DCUEPredset(trip.copy(), meta, split="train")
    val = DCUEPredset(trip.copy(), meta, split="val")
    items = DCUEItemset(trip.copy(), meta)
    torch.manual_seed(4)
    tr = DCUE(feature_dim=d, conv_hidden=H, batch_size=8)
    tr.n_users, tr.n_items = len(train.user_index), len(train.item_index)
    tr.epoch_size = 64
    tr._init_nn()
    sd = tr.model.state_dict()
    g2 = torch.Generator().manual_seed(9)
    for k in list(sd):
        if k.endswith("running_mean"):
            sd[k] = 0.3 * torch.randn(sd[k].shape, generator=g2)
        elif k.endswith("running_var"):
            sd[k] = 0.5 + torch.rand(sd[k].shape, generator=g2)
        elif k.endswith("num_batches_tracked"):
            sd[k] = torch.tensor(7)
    tr.model.load_state_dict(sd)
    tr._user_factors(items)
    tr._item_factors(items)

    def loader(ds):
        return DataLoader(ds, batch_size=1024, shuffle=False, num_workers=0)
    val_users = sorted(set(train.uniq_users).intersection(set(val.uniq_users)))
    train_users = sorted(train.uniq_users)
    val_auc, val_ap, tr_auc, tr_ap = [], [], [], []
    for u in val_users:
        a, m = tr.score([u], loader(val), loader(train))
        val_auc.append(a)
        val_ap.append(m)
    for u in train_users:
        a, m = tr.score([u], loader(train), loader(train))
        tr_auc.append(a)
        tr_ap.append(m)
    val_songs = sorted(val.uniq_songs)
    song_auc, song_ap = [], []
    for s in val_songs:
        a, m = tr.score_song([s], loader(val))
        song_auc.append(a)
        song_ap.append(m)
    mean_val = tr.score(val_users[:9], loader(val), loader(train))
    _save("eval.npz", raw_users=trip["user_id"].to_numpy().astype(str),
          raw_songs=trip["song_id"].to_numpy().astype(str), raw_score=trip["score"].to_numpy(),
          meta_songs=np.array(meta_songs).astype(str), spec=spec.half(), H=H, d=d,
          **{"sd." + k: v for k, v in tr.model.state_dict().items()},
          user_factors=tr.user_factors, item_factors=tr.item_factors,
          val_users=np.array(val_users).astype(str), val_auc=np.array(val_auc), val_ap=np.array(val_ap),
          train_users=np.array(train_users).astype(str), train_auc=np.array(tr_auc),
          train_ap=np.array(tr_ap), val_songs=np.array(val_songs).astype(str),
          song_auc=np.array(song_auc), song_ap=np.array(song_ap),
          mean9_auc=mean_val[0], mean9_ap=mean_val[1],
          user_categories=np.array(list(train.user_index.keys())).astype(str),
          song_categories=np.array(list(train.item_index.keys())).astype(str),
          train_split_items=np.array(sorted(train.uniq_song_idxs), dtype=np.int64),
          val_split_items=np.array(sorted(val.uniq_song_idxs), dtype=np.int64))


class _RecDCUE(DCUE):
    """The reference trainer, recording what fit() computes (methods on the class: fit's checkpoint
    pickles the instance __dict__)."""
    rec = {"train": [], "update": [], "scores": [], "song": []}

    def _train_epoch(self, loader):
        out = DCUE._train_epoch(self, loader)
        self.rec["train"].append(out)
        return out

    def _update_best(self, val_map, val_auc, val_loss):
        self.rec["update"].append((val_map, val_auc, val_loss))
        return DCUE._update_best(self, val_map, val_auc, val_loss)

    def _compute_scores(self, split, *a, **k):
        out = DCUE._compute_scores(self, split, *a, **k)
        self.rec["scores"].append((0 if split == "val" else 1,) + tuple(out))
        return out

    def _compute_scores_song(self, *a, **k):
        out = DCUE._compute_scores_song(self, *a, **k)
        self.rec["song"].append(out)
        return out


def fit_fixture():
    """DCUE.fit end to end (nn/dcue.py:264-378) for one epoch (10 sub-epochs) on the eval fixture's
    data, with every DataLoader forced to num_workers=0: the protocol under which negative draws and
    shuffles follow the global numpy / torch streams (multi-worker loaders reseed per worker).
    Records each sub-epoch's train loss, val loss, AUC / mAP numbers and the final parameters."""
    import tempfile
    import torch.utils.data as tud
    import dcrecommend.nn.dcue as refnn  # reference
    from dcrecommend.datasets.dcuepredset import DCUEPredset  # reference
    from dcrecommend.datasets.dcueitemset import DCUEItemset  # reference
    g = np.load(os.path.join(HERE, "eval.npz"), allow_pickle=False)
    trip = pd.DataFrame({"user_id": g["raw_users"], "song_id": g["raw_songs"], "score": g["raw_score"]})
    tmp = tempfile.mkdtemp()
    paths = []
    for k in range(len(g["meta_songs"])):
        pth = os.path.join(tmp, "m%03d.pt" % k)
        torch.save(torch.from_numpy(g["spec"][k].astype(np.float32)), pth)
        paths.append(pth)
    meta = pd.DataFrame({"idx": np.arange(len(g["meta_songs"])), "song_id": g["meta_songs"], "data_mel": paths})
    N, B = 4, 8
    train = DCUEDataset(trip.copy(), meta, neg_samples=N, split="train")
    val = DCUEDataset(trip.copy(), meta, neg_samples=N, split="val")
    test = DCUEDataset(trip.copy(), meta, neg_samples=N, split="test")
    pred = DCUEPredset(trip.copy(), meta, split="val")
    truth = DCUEPredset(trip.copy(), meta, split="train")
    items = DCUEItemset(trip.copy(), meta)
    orig = tud.DataLoader

    def loader0(*a, **k):
        k["num_workers"] = 0
        return orig(*a, **k)
    refnn.DataLoader = loader0
    rec = _RecDCUE.rec
    tr = _RecDCUE(feature_dim=32, conv_hidden=32, batch_size=B, neg_batch_size=N, lr=1e-3, num_epochs=1,
                  eval_pct=1.0)
    np.random.seed(31)
    torch.manual_seed(32)
    tr.fit(train, val, test, pred, truth, items, len(train.user_index), len(train.item_index), "t", "m",
           tempfile.mkdtemp())
    refnn.DataLoader = orig
    _save("fit.npz", N=N, B=B, np_seed=31, torch_seed=32,
          train=np.array(rec["train"], dtype=np.float64), update=np.array(rec["update"], dtype=np.float64),
          scores=np.array(rec["scores"], dtype=np.float64), song=np.array(rec["song"], dtype=np.float64),
          **{"final." + k: v for k, v in tr.model.state_dict().items()})


def optim_fixture():
    from dcrecommend.optim.ranger import Ranger  # reference
    shapes = [(37, 5), (64,), (3, 4, 2)]
    gen = torch.Generator().manual_seed(77)
    init = [torch.randn(*s, generator=gen) * 0.1 for s in shapes]
    steps = 13
    grads = []
    for t in range(steps):
        gs = []
        for s in shapes:
            g = torch.randn(*s, generator=gen) * (10.0 ** torch.empty(s).uniform_(-6, 0, generator=gen))
            g.view(-1)[:: 7 + t] = 0.0  # rows without a gradient, as the dense embedding gradient has
            gs.append(g)
        grads.append(gs)
    lrs = [1e-3 * (1.0 - 0.05 * t) for t in range(steps)]
    out = {"init.%d" % i: v for i, v in enumerate(init)}
    out.update({"grad.%d.%d" % (t, i): g for t in range(steps) for i, g in enumerate(grads[t])})
    out["lr"] = np.array(lrs)
    cfgs = {"ranger_a": ("ranger", (0.9, 0.99), 0.0), "ranger_b": ("ranger", (0.95, 0.999), 1e-2),
            "sgd_a": ("sgd", 0.9, 0.0), "sgd_b": ("sgd", 0.5, 1e-2)}
    for tag, (kind, beta, wd) in cfgs.items():
        ps = [torch.nn.Parameter(v.clone()) for v in init]
        if kind == "ranger":
            opt = Ranger(ps, lr=lrs[0], alpha=0.5, k=6, N_sma_threshhold=5, betas=beta, eps=1e-5, weight_decay=wd)
        else:
            opt = torch.optim.SGD(ps, lrs[0], beta, weight_decay=wd, nesterov=True)
        for t in range(steps):
            for p_, g in zip(ps, grads[t]):
                p_.grad = g.clone()
            opt.param_groups[0]["lr"] = lrs[t]
            opt.step()
            for i, p_ in enumerate(ps):
                out["%s.p.%d.%d" % (tag, t, i)] = p_.detach().clone()
                st = opt.state[p_]
                for k in ("exp_avg", "exp_avg_sq", "slow_buffer", "momentum_buffer"):
                    if k in st:
                        out["%s.%s.%d.%d" % (tag, k, t, i)] = st[k].clone()
        out["%s.cfg" % tag] = np.array([beta[0] if kind == "ranger" else beta,
                                        beta[1] if kind == "ranger" else 0.0, wd])
    _save("optim.npz", **out)


if __name__ == "__main__":
    jobs = {
        "model": lambda: (model_fixture("model_tiny.npz", H=32, d=32, n_users=10, B=4, N=3),
                          model_fixture("model_h128.npz", H=128, d=128, n_users=10, B=2, N=2,
                                        store_init=False, store_steps=False)),
        "towers": lambda: [model_fixture("model_%s.npz" % tag, H=32, d=32, n_users=10, B=4, N=3,
                                         store_init=False, model_type=mt)
                           for tag, mt in (("plain", "truedcuemel1d"), ("res", "truedcuemel1dres"),
                                           ("resbn", "truedcuemel1dresbn"))],
        # widths outside 32/64/128/256: the trainer's default feature_dim = 100 (nn/dcue.py:44) and
        # odd H / d in the other towers (the library pads them to its storage widths)
        "widths": lambda: (model_fixture("model_d100.npz", H=128, d=100, n_users=10, B=2, N=2,
                                         store_init=False, store_steps=False),
                           [model_fixture("model_w_%s.npz" % tag, H=H, d=d, n_users=10, B=4, N=3,
                                          store_init=False, model_type=mt)
                            for tag, H, d, mt in (("plain", 36, 20, "truedcuemel1d"),
                                                  ("res", 48, 52, "truedcuemel1dres"),
                                                  ("resbn", 40, 24, "truedcuemel1dresbn"))]),
        "inbatch": inbatch_fixtures, "catalogue": catalogue_fixture, "batches": batches_fixture,
        "scheduler": scheduler_fixture, "train5": train5_fixture, "metrics": metrics_fixture,
        "eval": eval_fixture, "fit": fit_fixture, "optim": optim_fixture,
    }
    for name in (sys.argv[1:] or list(jobs)):  # e.g. `make_golden.py eval` regenerates one fixture
        jobs[name]()
