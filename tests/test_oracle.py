"""The oracle (CPU restatement) against the golden vectors produced by the reference."""
import numpy as np
import pytest
import torch

from oracle import dcue_oracle as O
from oracle import mt19937 as MT

torch.set_num_threads(4)


def _p(g, prefix):
    return {k[len(prefix):]: torch.from_numpy(np.array(g[k])) for k in g.files if k.startswith(prefix)}


def _inputs(g):
    return (torch.from_numpy(g["u"]), torch.from_numpy(g["pos"]).float(),
            torch.from_numpy(g["neg"]).float())


def _close(a, b, rtol=1e-4, atol_frac=1e-5):
    a = torch.as_tensor(np.asarray(a), dtype=torch.float64)
    b = torch.as_tensor(np.asarray(b), dtype=torch.float64)
    atol = atol_frac * max(float(b.abs().max()), 1e-30)
    return torch.allclose(a, b, rtol=rtol, atol=atol), float((a - b).abs().max())


def test_init_matches_reference(golden):
    g = golden("model_tiny.npz")
    torch.manual_seed(int(g["seed"]))
    p, b = O.init_params(int(g["d"]), int(g["H"]), 300, int(g["n_users"]))
    init = _p(g, "init.")
    for k, v in p.items():
        assert torch.equal(v, init[k]), k
    for k, v in b.items():
        assert torch.equal(v, init[k]), k


def test_init_h128_checksums(golden):
    g = golden("model_h128.npz")
    torch.manual_seed(int(g["seed"]))
    p, b = O.init_params(int(g["d"]), int(g["H"]), 300, int(g["n_users"]))
    for k, v in {**p, **b}.items():
        assert float(v.double().sum()) == pytest.approx(float(g["initsum." + k]), rel=1e-12, abs=1e-9), k


def _mt(g):
    return str(g["model_type"]) if "model_type" in g.files else "truedcuemel1dbn"


@pytest.mark.parametrize("name", ["model_plain.npz", "model_res.npz", "model_resbn.npz", "model_d100.npz",
                                  "model_w_plain.npz", "model_w_res.npz", "model_w_resbn.npz"])
def test_init_towers_checksums(golden, name):
    """The other wired towers (dcue/dcue.py:49-59): parameter names, order and init draws."""
    g = golden(name)
    torch.manual_seed(int(g["seed"]))
    p, b = O.init_params(int(g["d"]), int(g["H"]), 300, int(g["n_users"]), _mt(g))
    keys = {k[len("initsum."):] for k in g.files if k.startswith("initsum.")}
    assert keys == set(p) | set(b)
    for k, v in {**p, **b}.items():
        assert float(v.double().sum()) == pytest.approx(float(g["initsum." + k]), rel=1e-12, abs=1e-9), k


@pytest.mark.parametrize("name", ["model_tiny.npz", "model_h128.npz", "model_plain.npz", "model_res.npz",
                                  "model_resbn.npz", "model_d100.npz", "model_w_plain.npz", "model_w_res.npz",
                                  "model_w_resbn.npz"])
def test_forward_backward_step(golden, name):
    g = golden(name)
    torch.manual_seed(int(g["seed"]))
    p, b = O.init_params(int(g["d"]), int(g["H"]), 300, int(g["n_users"]), _mt(g))
    u, pos, neg = _inputs(g)
    loss, grads, (scores, uf, pf, nf) = O.loss_and_grads(p, b, u, pos, neg)
    for key, val in (("scores", scores), ("uf", uf), ("pf", pf), ("nf", nf), ("loss", loss)):
        ok, err = _close(val, g[key])
        assert ok, (key, err)
    for k, v in grads.items():
        ok, err = _close(v, g["grad." + k], rtol=1e-3, atol_frac=1e-4)
        assert ok, (k, err)
    for k, v in b.items():
        if "running" in k:
            ok, err = _close(v, g["fwd." + k])
            assert ok, (k, err)
    if "step1.conv.fc.weight" in g.files:
        adam = O.AdamState(p)
        adam.step(p, {k: torch.from_numpy(g["grad." + k]) for k in p}, float(g["lr"]))
        for k, v in p.items():
            ok, err = _close(v, g["step1." + k], rtol=1e-6, atol_frac=1e-7)
            assert ok, (k, err)
        adam.step(p, {k: torch.from_numpy(g["grad." + k]) for k in p}, float(g["lr"]), 1e-4)
        for k, v in p.items():
            ok, err = _close(v, g["step2." + k], rtol=1e-6, atol_frac=1e-7)
            assert ok, (k, err)
        with torch.no_grad():
            es, euf, epf, enf = O.forward(p, {k: torch.from_numpy(np.array(g["fwd." + k])) for k in b},
                                          u, pos, neg, train=False)
        ok, err = _close(es, g["eval_scores"])
        assert ok, err


def test_inbatch_model(golden):
    g = golden("inbatch_model.npz")
    torch.manual_seed(0)
    p, b = O.init_params(int(g["d"]), int(g["H"]), 300, int(g["n_users"]))
    u, pos = torch.from_numpy(g["u"]), torch.from_numpy(g["pos"]).float()
    r = torch.from_numpy(g["r"])
    B, N = r.shape
    neg = pos[r.reshape(-1)].reshape(B, N, 128, 131)
    loss, grads, (scores, *_r) = O.loss_and_grads(p, b, u, pos, neg)
    assert _close(scores, g["scores"])[0]
    for k, v in grads.items():
        ok, err = _close(v, g["grad." + k], rtol=1e-3, atol_frac=1e-4)
        assert ok, (k, err)


def test_train5(golden):
    g = golden("train5.npz")
    torch.manual_seed(0)
    p, b = O.init_params(int(g["d"]), int(g["H"]), 300, int(g["n_users"]))
    adam = O.AdamState(p)
    for s in range(5):
        loss = O.train_step(p, b, adam, torch.from_numpy(g["u"][s]), torch.from_numpy(g["pos"][s]).float(),
                            torch.from_numpy(g["neg"][s]).float(), float(g["lr"][s]))
        assert float(loss) == pytest.approx(float(g["loss"][s]), rel=1e-4)
    # Adam moves every element by up to ~lr per step whatever the gradient's size, so elements whose
    # gradient is rounding noise can move differently under a different summation order: the
    # absolute tolerance is a small fraction of the total lr budget (5 steps).
    budget = float(np.sum(g["lr"]))
    for k, v in {**p, **b}.items():
        ref = torch.from_numpy(np.array(g["final." + k])).double()
        err = (v.double() - ref).abs()
        tight = 1e-4 * float(ref.abs().max()) + 1e-3 * budget
        # e.g. a conv bias right before a train-mode BN whose inputs are all active has an
        # exactly-zero true gradient, so its sign (and Adam's +-lr move) is rounding noise.
        assert int((err > tight).sum()) <= max(2, err.numel() // 20), (k, float(err.max()))
        assert float(err.max()) <= 2 * budget, (k, float(err.max()))


def test_mt_stream_matches_numpy():
    for seed in (0, 1, 123456789, 2**32 - 1):
        ref = np.random.RandomState(seed).randint(0, 2**32, size=1500, dtype=np.uint64).astype(np.uint32)
        assert np.array_equal(MT.mt_stream(seed, 1500), ref)


def test_inbatch_draws(golden):
    g = golden("inbatch_draws.npz")
    for s in (0, 5, 99):
        assert np.array_equal(MT.inbatch(s, 64, 20), g["seed%d" % s])
        assert np.array_equal(O.inbatch_negatives(np.random.RandomState(s), 64, 20), g["seed%d" % s])
    assert np.array_equal(MT.inbatch(3, 8, 5), g["small_seed3"])


def _catalogue_csr(g):
    users = {u: i for i, u in enumerate(g["user_categories"])}
    songs = {s: i for i, s in enumerate(g["song_categories"])}
    uidx = np.array([users[u] for u in g["raw_users"]])
    sidx = np.array([songs[s] for s in g["raw_songs"]])
    order = np.lexsort((sidx, uidx))
    indptr = np.zeros(len(users) + 1, dtype=np.int64)
    np.add.at(indptr, uidx + 1, 1)
    return np.cumsum(indptr), sidx[order].astype(np.int64)


def test_catalogue_draws(golden):
    g = golden("catalogue.npz")
    indptr, indices = _catalogue_csr(g)
    users = g["users_seq"]
    N = int(g["N"])
    got = MT.catalogue(1234, True, g["split_items"], indptr, indices, users, N)
    assert np.array_equal(got, g["seeded"])
    got = MT.catalogue(77, False, g["split_items"], indptr, indices, users, N)
    assert np.array_equal(got, g["stream"])
    items = [indices[indptr[u]:indptr[u + 1]] for u in users]
    assert np.array_equal(O.catalogue_negatives(np.random.RandomState(77), g["split_items"], items, N), g["stream"])
