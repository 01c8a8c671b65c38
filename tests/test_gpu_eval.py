"""GPU parity of the evaluation path (dcue_rank_metrics, the eval towers, the DCUE trainer's
score / score_song) against the reference's outputs (tests/golden/eval.npz) and the metric oracle.

Tolerances: per-query AUC / AP computed from the reference's own factors within 1e-9 of the
reference (the GPU's fp32 cosine may differ from torch's in the last ulp, which can only matter
for scores closer than that; none are in the fixture). Factors from our towers within 1e-4 of the
output's largest magnitude (north-star bar); AUC / mAP means from our factors within 1e-6. On the
gaussian random cases the oracle scores with torch's CPU cosine, so near-ties (< 1e-7 apart) may
order differently, each flip moving a small query's AUC by 1/(n_pos n_neg): 5e-5 there; the
lattice cases have exactly representable scores and are held to 1e-12.
"""
import os

import numpy as np
import pandas as pd
import pytest
import torch

from oracle import rank_oracle as R

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _datasets(g, tmp_path=None):
    from dcrecommend.datasets.dcuepredset import DCUEPredset
    from dcrecommend.datasets.dcueitemset import DCUEItemset
    trip = pd.DataFrame({"user_id": g["raw_users"], "song_id": g["raw_songs"], "score": g["raw_score"]})
    paths = [""] * len(g["meta_songs"])
    if tmp_path is not None:
        # metadata row k (song meta_songs[k]) points at spectrogram spec[k], as make_golden wrote it
        for k in range(len(g["meta_songs"])):
            p = os.path.join(str(tmp_path), "m%03d.pt" % k)
            torch.save(torch.from_numpy(g["spec"][k].astype(np.float32)), p)
            paths[k] = p
    meta = pd.DataFrame({"idx": np.arange(len(g["meta_songs"])), "song_id": g["meta_songs"], "data_mel": paths})
    return (DCUEPredset(trip.copy(), meta, split="train"), DCUEPredset(trip.copy(), meta, split="val"),
            DCUEItemset(trip.copy(), meta))


def test_rank_metrics_reference_factors(golden):
    from dcrecommend import _native as nat
    from dcrecommend.nn import rank
    g = golden("eval.npz")
    train, val, items = _datasets(g)
    uf = torch.from_numpy(g["user_factors"].astype(np.float32)).to(DEV)
    cand = torch.from_numpy(g["item_factors"].astype(np.float32)[items.item_rows()]).to(DEV)
    ev = rank.RankEvaluator(rank.user_split_inputs(val, train), DEV)
    q = np.array([train.user_index[u] for u in g["val_users"]])
    auc, ap, ok = ev.metrics(uf, cand, q, nat.RANK_SPLIT)
    assert ok.all()
    np.testing.assert_allclose(auc, g["val_auc"], rtol=0, atol=1e-9)
    np.testing.assert_allclose(ap, g["val_ap"], rtol=0, atol=1e-9)
    ev = rank.RankEvaluator(rank.user_split_inputs(train, train), DEV)
    q = np.array([train.user_index[u] for u in g["train_users"]])
    auc, ap, ok = ev.metrics(uf, cand, q, nat.RANK_SPLIT)
    np.testing.assert_allclose(auc, g["train_auc"], rtol=0, atol=1e-9)
    np.testing.assert_allclose(ap, g["train_ap"], rtol=0, atol=1e-9)
    ev = rank.RankEvaluator(rank.song_inputs(val), DEV)
    q = np.array([val.item_index[s] for s in g["val_songs"]])
    auc, ap, ok = ev.metrics(cand, uf, q, nat.RANK_SINGLE)
    assert ok.all()
    np.testing.assert_allclose(auc, g["song_auc"], rtol=0, atol=1e-9)
    np.testing.assert_allclose(ap, g["song_ap"], rtol=0, atol=1e-9)


def _lattice(rs, n, d):
    """Rows with 16 entries of +-1 (norm exactly 4): normalised entries are +-1/4 and every cosine
    is a multiple of 1/16, exact in fp32 whatever the summation order -- many exact ties."""
    x = np.zeros((n, d), np.float32)
    for r in range(n):
        x[r, rs.choice(d, 16, replace=False)] = rs.choice(np.array([-1.0, 1.0], np.float32), 16)
    return x


def _random_case(seed, n_rows, n_cand, d, max_pos, lattice=False):
    rs = np.random.RandomState(seed)
    cand = _lattice(rs, n_cand, d) if lattice else rs.randn(n_cand, d).astype(np.float32)
    dup = rs.choice(n_cand, n_cand // 20, replace=False)
    cand[dup] = cand[rs.choice(n_cand, len(dup))]  # identical rows: exact score ties
    cand[rs.choice(n_cand, 3, replace=False)] = 0.0  # zero vectors: cosine 0 via the eps clamp
    qf = _lattice(rs, n_rows, d) if lattice else rs.randn(n_rows, d).astype(np.float32)
    cls = rs.choice(np.array([0, 1, 2, 3], np.uint8), n_cand, p=[0.1, 0.3, 0.5, 0.1])
    ptr = [0]
    idx = []
    for r in range(n_rows):
        k = rs.randint(0, max_pos + 1)
        idx.append(np.sort(rs.choice(n_cand, k, replace=False)))
        ptr.append(ptr[-1] + k)
    return qf, cand, {"pos_ptr": np.array(ptr, np.int64), "pos_idx": np.concatenate(idx).astype(np.int32),
                      "cand_class": cls}


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("d", [32, 100, 128])
def test_rank_metrics_lattice_exact(mode, d):
    """Exactly representable scores with heavy ties: the GPU counts equal the oracle's."""
    from dcrecommend.nn import rank
    qf, cand, inp = _random_case(3 + d + mode, 120, 2500, d, 150, lattice=True)
    queries = np.random.RandomState(2).randint(0, 120, 150)
    ev = rank.RankEvaluator(inp, DEV, max_score_bytes=64 * 2500 * 4)
    auc, ap, ok = ev.metrics(torch.from_numpy(qf).to(DEV), torch.from_numpy(cand).to(DEV), queries, mode)
    want_auc, want_ap, want_ok = R.rank_metrics(qf, cand, queries, inp["pos_ptr"], inp["pos_idx"],
                                                inp["cand_class"], mode)
    assert np.array_equal(ok, want_ok.astype(bool))
    np.testing.assert_allclose(auc, want_auc, rtol=0, atol=1e-12)
    np.testing.assert_allclose(ap, want_ap, rtol=0, atol=1e-12)


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("d", [32, 100, 128])
def test_rank_metrics_random_vs_oracle(mode, d):
    from dcrecommend.nn import rank
    qf, cand, inp = _random_case(7 + d + mode, 120, 2500, d, 150)
    queries = np.random.RandomState(1).randint(0, 120, 200)
    ev = rank.RankEvaluator(inp, DEV, max_score_bytes=64 * 2500 * 4)  # several query batches
    auc, ap, ok = ev.metrics(torch.from_numpy(qf).to(DEV), torch.from_numpy(cand).to(DEV), queries, mode)
    want_auc, want_ap, want_ok = R.rank_metrics(qf, cand, queries, inp["pos_ptr"], inp["pos_idx"],
                                                inp["cand_class"], mode)
    assert np.array_equal(ok, want_ok.astype(bool))
    np.testing.assert_allclose(auc, want_auc, rtol=0, atol=5e-5)
    np.testing.assert_allclose(ap, want_ap, rtol=0, atol=5e-5)


def test_rank_metrics_nonfinite_raise():
    """NaN factors raise ValueError where the reference's sklearn calls would (nn/dcue.py:440,447,
    473-474) -- the oracle (pinned to sklearn in test_eval_cpu.py) and the GPU evaluator agree -- and
    never yield an AUC outside [0, 1]: a NaN user factor before score()'s loop break, a NaN candidate
    in a list; not a NaN candidate outside both lists, nor a NaN user after the break."""
    from dcrecommend.nn import rank
    qf, cand, inp = _random_case(11, 60, 1500, 64, 80)
    ptr, cls = inp["pos_ptr"], inp["cand_class"]
    has_pred = np.array([(cls[inp["pos_idx"][ptr[r]:ptr[r + 1]]] & 1).any() for r in range(60)])
    good = np.flatnonzero(has_pred)
    queries = good[:20]
    ev = rank.RankEvaluator(inp, DEV)
    args = (inp["pos_ptr"], inp["pos_idx"], inp["cand_class"])

    def both(q, c, qs, mode):
        err = []
        for fn in (lambda: ev.metrics(torch.from_numpy(q).to(DEV), torch.from_numpy(c).to(DEV), qs, mode),
                   lambda: R.rank_metrics(q, c, qs, *args, mode)):
            try:
                fn()
                err.append(None)
            except ValueError as e:
                err.append(str(e))
        return err

    clean = ev.metrics(torch.from_numpy(qf).to(DEV), torch.from_numpy(cand).to(DEV), queries, 0)
    bad_q = qf.copy()
    bad_q[queries[3]] = np.nan
    e = both(bad_q, cand, queries, 0)
    assert e[0] and e[1] and "Input contains NaN" in e[0], e
    bad_c = cand.copy()
    bad_c[np.flatnonzero(cls == 2)[0]] = np.nan  # truth list only: in average_precision's input
    assert all(both(qf, bad_c, queries, 0)), "a NaN truth-list candidate must raise"
    outside = cand.copy()
    outside[np.flatnonzero(cls == 0)[:5]] = np.nan  # in no list: never scored by the reference
    assert both(qf, outside, queries, 0) == [None, None]
    auc, ap, ok = ev.metrics(torch.from_numpy(qf).to(DEV), torch.from_numpy(outside).to(DEV), queries, 0)
    assert np.array_equal(auc, clean[0]) and np.array_equal(ap, clean[1])
    no_pred = np.flatnonzero(~has_pred)
    if len(no_pred):
        qs = np.array([good[0], no_pred[0], good[1]])
        late = qf.copy()
        late[good[1]] = np.nan  # after the break
        assert both(late, cand, qs, 0) == [None, None]
    # score_song: a NaN candidate of the label-0 list raises for every song with both labels
    bad_s = cand.copy()
    bad_s[np.flatnonzero(cls & 1)[0]] = np.nan
    e = both(qf, bad_s, queries, 1)
    assert e[0] and e[1], e


def test_rank_metrics_cap():
    from dcrecommend.nn import rank
    rs = np.random.RandomState(0)
    n = 6000
    inp = {"pos_ptr": np.array([0, 5000], np.int64), "pos_idx": np.arange(5000, dtype=np.int32),
           "cand_class": np.ones(n, np.uint8)}
    ev = rank.RankEvaluator(inp, DEV)
    with pytest.raises(RuntimeError, match="UNSUPPORTED"):
        ev.metrics(torch.from_numpy(rs.randn(1, 32).astype(np.float32)).to(DEV),
                   torch.from_numpy(rs.randn(n, 32).astype(np.float32)).to(DEV), [0], 0)


@pytest.fixture(scope="module")
def trained(golden, tmp_path_factory):
    from dcrecommend.nn.dcue import DCUE
    g = golden("eval.npz")
    train, val, items = _datasets(g, tmp_path_factory.mktemp("mel"))
    tr = DCUE(feature_dim=int(g["d"]), conv_hidden=int(g["H"]), batch_size=8, device=DEV)
    tr.n_users, tr.n_items, tr.epoch_size = len(train.user_index), len(train.item_index), 64
    tr._init_nn()
    sd = {k[3:]: torch.from_numpy(np.array(g[k])) for k in g.files if k.startswith("sd.")}
    tr.model.load_state_dict(sd)
    tr._user_factors(items)
    tr._item_factors(items)
    return g, tr, train, val, items


def test_trainer_factors(trained):
    g, tr, train, val, items = trained
    for what, got, want in (("user", tr.user_factors, g["user_factors"]), ("item", tr.item_factors, g["item_factors"])):
        want = torch.from_numpy(want)
        err = float((got.cpu() - want).abs().max() / want.abs().max())
        assert err < 1e-4, (what, err)


def test_trainer_score(trained):
    g, tr, train, val, items = trained
    auc, ap = tr.score(list(g["val_users"][:9]), val, train)
    assert abs(auc - float(g["mean9_auc"])) < 1e-6 and abs(ap - float(g["mean9_ap"])) < 1e-6
    auc, ap = tr.score_song(list(g["val_songs"]), val)
    assert abs(auc - float(np.mean(g["song_auc"]))) < 1e-6
    assert abs(ap - float(np.mean(g["song_ap"]))) < 1e-6
    # predict(): the reference's per-user lists scored by model.sim, through the oracle's
    # arithmetic, agree with the GPU evaluator for the same user
    u = g["val_users"][0]
    sp, tp = tr.predict(u, val)
    st, tt = tr.predict(u, train)
    want = R.user_metrics(sp, tp, st, tt)
    got = tr.score_users(np.array([train.user_index[u]]), val, train)
    assert abs(got[0][0] - want[0]) < 1e-9 and abs(got[1][0] - want[1]) < 1e-9


def test_trainer_fit_and_checkpoint(golden, tmp_path):
    from dcrecommend.nn.dcue import DCUE
    g = golden("eval.npz")
    train, val, items = _datasets(g, tmp_path)
    test = val
    tr = DCUE(feature_dim=32, conv_hidden=32, batch_size=8, neg_batch_size=4, num_epochs=1, eval_pct=1.0,
              lr=1e-3, device=DEV)
    np.random.seed(3)
    torch.manual_seed(3)
    tr.fit(train, val, test, val, train, items, len(train.user_index), len(train.item_index), "trip", "meta",
           str(tmp_path / "ck"))
    # one pass over the 10 (9 when len % 10 != 0) chunks finishes before the while re-checks
    assert tr.nn_epoch == (10 if len(train) % 10 == 0 else 9)
    assert np.isfinite(tr.best_val_loss) and 0 <= tr.best_val_auc <= 1 and 0 < tr.best_val_map <= 1
    sub = tmp_path / "ck" / tr._format_model_subdir()
    files = sorted(os.listdir(sub))
    assert files, "no checkpoint written"
    ep = int(files[0].split("_")[1].split(".")[0])
    tr2 = DCUE(device=DEV)
    tr2.load(str(sub), ep)
    assert tr2.nn_epoch == ep + 1 and tr2.feature_dim == 32
    assert torch.equal(tr2.model.conv.fc.weight.cpu(),
                       torch.load(str(sub / files[0]), weights_only=True)["model"]["conv.fc.weight"])


def test_train_dcue_driver_synthetic(tmp_path):
    """train_dcue.py (the reference README's train_* driver) end to end on synthetic files."""
    import train_dcue
    dcue = train_dcue.main(["--synthetic", "--synthetic-users", "24", "--synthetic-tracks", "80",
                            "--synthetic-pairs", "300", "--feature-dim", "32", "--conv-hidden", "32",
                            "--batch-size", "8", "--neg-batch-size", "3", "--num-epochs", "1",
                            "--eval-pct", "1.0", "--lr", "1e-3", "--save-dir", str(tmp_path)])
    assert dcue._plan_n == 3 and dcue.nn_epoch >= 9
    assert 0.0 <= dcue.best_val_auc <= 1.0
    assert os.listdir(tmp_path)


def test_train_dcue_driver_config1(tmp_path):
    """BASELINE.json configs[0]'s shape -- d=64, H=128, 1k users x 5k tracks of 131-frame
    spectrograms -- through the reference trainer API end to end (train_dcue.py: datasets from
    triplets/metadata frames, spectrogram files loaded once into the HBM table, DCUE.fit's sub-epoch
    loop with validation AUC, checkpoints)."""
    import train_dcue
    dcue = train_dcue.main(["--synthetic", "--synthetic-users", "1000", "--synthetic-tracks", "5000",
                            "--synthetic-pairs", "20000", "--feature-dim", "64", "--conv-hidden", "128",
                            "--batch-size", "64", "--neg-batch-size", "20", "--num-epochs", "1",
                            "--lr", "1e-4", "--save-dir", str(tmp_path)])
    assert dcue._plan_n == 20 and dcue.nn_epoch >= 9
    assert dcue.feature_dim == 64 and dcue.conv_hidden == 128
    assert 0.0 <= dcue.best_val_auc <= 1.0
    assert os.listdir(tmp_path)


def test_train_dcue_reference_defaults(tmp_path):
    """train_dcue.py with the reference trainer's defaults (DCUE(feature_dim=100, conv_hidden=128,
    u_embdim=300, batch_size=64, ...), nn/dcue.py:44-50): only the synthetic data is chosen here.
    feature_dim = 100 runs at the library's 128-wide storage; the factors are d = 100 wide."""
    import train_dcue
    dcue = train_dcue.main(["--synthetic", "--synthetic-users", "300", "--synthetic-tracks", "600",
                            "--synthetic-pairs", "6000", "--num-epochs", "1", "--lr", "1e-4",
                            "--save-dir", str(tmp_path)])
    assert dcue.feature_dim == 100 and dcue.conv_hidden == 128 and dcue.u_embdim == 300
    assert dcue.model.conv.fc.weight.shape == (100, 100)
    assert dcue.user_factors.shape[1] == 100 and dcue.item_factors.shape[1] == 100
    assert 0.0 <= dcue.best_val_auc <= 1.0 and os.listdir(tmp_path)
    from test_gpu_parity import assert_storage_pads_zero
    assert_storage_pads_zero(dcue.model)


def test_saturated_user_raises_like_numpy(tmp_path):
    """40 tracks: the val split holds 3 songs and one user has all of them, so the reference's
    np.random.choice over that user's (empty) non-items raises ValueError
    (datasets/dcuedataset.py:219); the GPU sampler's host check raises the same error."""
    import train_dcue
    with pytest.raises(ValueError, match="cannot be empty"):
        train_dcue.main(["--synthetic", "--synthetic-users", "24", "--synthetic-tracks", "40",
                         "--synthetic-pairs", "300", "--feature-dim", "32", "--conv-hidden", "32",
                         "--batch-size", "8", "--neg-batch-size", "3", "--num-epochs", "1",
                         "--eval-pct", "1.0", "--lr", "1e-3", "--save-dir", str(tmp_path)])


def test_trainer_fit_matches_reference(golden, tmp_path):
    """DCUE.fit against the reference's own fit (tests/golden/fit.npz, num_workers=0 loaders): same
    seeds -> same chunks, shuffles and negative draws (numpy's stream continued on the GPU, torch's
    DataLoader draws mirrored), so every sub-epoch's numbers line up. Measured on MI355X: train loss
    1.1e-6 relative, val loss 1.7e-6, AUC / mAP 1.4e-4 absolute. Tolerances: losses 1e-5 relative
    (fp32 GPU vs CPU, compounded over the Adam steps), AUC / mAP 5e-4 (a score near-tie resolved
    differently moves a mean by ~1/(n_pos n_neg n_users)), final parameters 1e-3 of their largest
    magnitude (lr 1e-3 steps on rounding-level gradient differences)."""
    from dcrecommend.nn.dcue import DCUE
    g = golden("eval.npz")
    f = golden("fit.npz")
    from dcrecommend.datasets.dcuedataset import DCUEDataset
    train, val, items = _datasets(g, tmp_path)
    N, B = int(f["N"]), int(f["B"])
    trip = pd.DataFrame({"user_id": g["raw_users"], "song_id": g["raw_songs"], "score": g["raw_score"]})
    meta = items.metadata.copy()
    meta = pd.DataFrame({"idx": np.arange(len(g["meta_songs"])), "song_id": g["meta_songs"],
                         "data_mel": [os.path.join(str(tmp_path), "m%03d.pt" % k) for k in range(len(g["meta_songs"]))]})
    from dcrecommend.datasets.dcuepredset import DCUEPredset
    from dcrecommend.datasets.dcueitemset import DCUEItemset
    tr_ds = DCUEDataset(trip.copy(), meta, neg_samples=N, split="train")
    va_ds = DCUEDataset(trip.copy(), meta, neg_samples=N, split="val")
    te_ds = DCUEDataset(trip.copy(), meta, neg_samples=N, split="test")
    pred = DCUEPredset(trip.copy(), meta, split="val")
    truth = DCUEPredset(trip.copy(), meta, split="train")
    it_ds = DCUEItemset(trip.copy(), meta)

    rec = {"train": [], "update": [], "scores": [], "song": []}

    class Rec(DCUE):
        def _train_epoch(self, loader):
            out = DCUE._train_epoch(self, loader)
            rec["train"].append(out)
            return out

        def _update_best(self, val_map, val_auc, val_loss):
            rec["update"].append((val_map, val_auc, val_loss))
            return DCUE._update_best(self, val_map, val_auc, val_loss)

        def _compute_scores(self, split, *a, **k):
            out = DCUE._compute_scores(self, split, *a, **k)
            rec["scores"].append((0 if split == "val" else 1,) + tuple(out))
            return out

        def _compute_scores_song(self, *a, **k):
            out = DCUE._compute_scores_song(self, *a, **k)
            rec["song"].append(out)
            return out

    tr = Rec(feature_dim=32, conv_hidden=32, batch_size=B, neg_batch_size=N, lr=1e-3, num_epochs=1, eval_pct=1.0,
             device=DEV)
    np.random.seed(int(f["np_seed"]))
    torch.manual_seed(int(f["torch_seed"]))
    tr.fit(tr_ds, va_ds, te_ds, pred, truth, it_ds, len(tr_ds.user_index), len(tr_ds.item_index), "t", "m",
           str(tmp_path / "ck"))
    got = {k: np.array(v, dtype=np.float64) for k, v in rec.items()}
    assert got["train"].shape == f["train"].shape
    print("fit vs reference: train loss rel %.2e, val loss rel %.2e, AUC/mAP abs %.2e / %.2e / %.2e" % (
        float(np.abs(got["train"][:, 1] / f["train"][:, 1] - 1).max()),
        float(np.abs(got["update"][:, 2] / f["update"][:, 2] - 1).max()),
        float(np.abs(got["update"][:, :2] - f["update"][:, :2]).max()),
        float(np.abs(got["scores"] - f["scores"]).max()), float(np.abs(got["song"] - f["song"]).max())))
    np.testing.assert_array_equal(got["train"][:, 0], f["train"][:, 0])
    np.testing.assert_allclose(got["train"][:, 1], f["train"][:, 1], rtol=1e-5)
    np.testing.assert_allclose(got["update"][:, 2], f["update"][:, 2], rtol=1e-5)   # val loss
    np.testing.assert_allclose(got["update"][:, :2], f["update"][:, :2], atol=5e-4)  # val mAP, AUC
    np.testing.assert_allclose(got["scores"], f["scores"], atol=5e-4)
    np.testing.assert_allclose(got["song"], f["song"], atol=5e-4)
    sd = tr.model.state_dict()
    for k in f.files:
        if k.startswith("final.") and "num_batches" not in k:
            want = torch.from_numpy(np.array(f[k])).double()
            diff = float((sd[k[6:]].cpu().double() - want).abs().max())
            assert diff <= 1e-3 * max(float(want.abs().max()), 1.0), (k, diff)
