"""GPU parity: libdcue_hip (through its C ABI) against the reference's golden vectors.

Tolerances (written per check): forward outputs (scores, user/item feature vectors, loss) within
1e-4 relative to the output's largest magnitude -- the north-star bar; gradients within 1e-3 relative
(abs floor 1e-4 x max|ref|), since the reference's own CPU gradients move by that much between
thread counts; Adam-updated parameters as in tests/test_oracle.py (an element whose true gradient
is zero moves by +-lr on rounding noise in any implementation). Sampler draws are bit-exact.
"""
import numpy as np
import pytest
import torch

from oracle import mt19937 as MT

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _rel_err(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(np.asarray(b)).double()
    scale = float(b.abs().max()) if b.numel() else 0.0
    return float((a - b).abs().max()) / max(scale, 1e-30)


def _assert_close(a, b, rtol, afrac, what):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(np.asarray(b)).double()
    atol = afrac * max(float(b.abs().max()), 1e-30)
    err = (a - b).abs()
    bad = err > atol + rtol * b.abs()
    assert not bool(bad.any()), "%s: max err %.3e (rel-to-max %.3e)" % (what, float(err.max()), _rel_err(a, b))


def _net(g, seed=0):
    from dcrecommend.dcue.dcue import DCUENet
    torch.manual_seed(seed)
    mt = str(g["model_type"]) if "model_type" in g.files else "truedcuemel1dbn"
    net = DCUENet({"feature_dim": int(g["d"]), "conv_hidden": int(g["H"]), "user_embdim": 300,
                   "user_count": int(g["n_users"]), "model_type": mt})
    return net.cuda()


def assert_storage_pads_zero(net):
    """Outside the reference-shaped corners of the flat parameter, gradient and BN-statistics buffers
    (the storage channels past H / d, include/dcue.h dcue_storage_dims) everything is exactly zero."""
    from dcrecommend import _native as nat
    fl = net._flat
    named = dict(net.named_parameters())
    for buf, what in ((fl["P"], "params"), (fl["G"], "grads")):
        mask = torch.ones_like(buf, dtype=torch.bool)
        for s, name in enumerate(nat.DENSE_NAMES):
            if name in named:
                nat.corner(mask, fl["poff"][s], fl["shapes"][s], named[name].shape).fill_(False)
        assert not bool(buf[mask].any()), "%s: storage pads not zero" % what
    mask = torch.ones_like(fl["stats"], dtype=torch.bool)
    for l in range(nat.N_BN):
        bn = getattr(net.conv, "bn%d" % l, None)
        if bn is not None:
            for j in (2 * l, 2 * l + 1):
                mask[fl["boff"][j]:fl["boff"][j] + bn.num_features] = False
    assert not bool(fl["stats"][mask].any()), "BN statistics: storage pads not zero"


def _hinge(scores, margin=0.2):  # the reference's _loss_func, nn/dcue.py:167-170
    return torch.max(torch.zeros_like(scores), margin - scores).sum(dim=1).mean()


def _check_grads(net, g, prefix="grad."):
    named = dict(net.named_parameters())
    for name, p in named.items():
        ref = g[prefix + name]
        got = net.embedding_grad_dense() if name == "user_embd.embeddings.weight" else p.grad
        _assert_close(got, ref, 1e-3, 1e-4, name)


def _check_params_after_adam(net, g, prefix, lr_budget, skip_rows=None, grad_prefix=None):
    """Every element within 2 x the steps' summed lr (+1e-4 of the tensor's max): an element whose
    true gradient is rounding noise can take a +-lr Adam step either way in any implementation (the
    optimizer itself is held bit-exact on identical gradients in test_gpu_adam_exact.py). Where the
    golden step's gradient is given (grad_prefix), elements whose gradient is at least 1e-2 of the
    tensor's largest -- a sign no rounding flips -- must agree to 1e-4 of max + 1e-3 lr."""
    sd = net.state_dict()
    for k, v in sd.items():
        if prefix + k not in g.files:
            continue
        ref = torch.from_numpy(np.array(g[prefix + k])).double()
        got = v.double().cpu()
        grad = None
        if grad_prefix is not None and grad_prefix + k in g.files:
            grad = torch.from_numpy(np.array(g[grad_prefix + k])).double()
        if skip_rows is not None and k == "user_embd.embeddings.weight":
            keep = torch.ones(ref.shape[0], dtype=torch.bool)
            keep[skip_rows] = False
            ref, got = ref[keep], got[keep]
            grad = grad[keep] if grad is not None else None
        if k.endswith("num_batches_tracked"):
            assert int(got) == int(ref), k
            continue
        err = (got - ref).abs()
        assert float(err.max()) <= 2 * lr_budget + 1e-4 * float(ref.abs().max()), (k, float(err.max()))
        if grad is not None and float(grad.abs().max()) > 0:
            firm = grad.abs() >= 1e-2 * float(grad.abs().max())
            tight = 1e-4 * float(ref.abs().max()) + 1e-3 * lr_budget
            assert float(err[firm].max()) <= tight, ("firm-gradient elements", k, float(err[firm].max()))


@pytest.mark.parametrize("name", ["model_tiny.npz", "model_h128.npz", "model_plain.npz", "model_res.npz",
                                  "model_resbn.npz", "model_d100.npz", "model_w_plain.npz", "model_w_res.npz",
                                  "model_w_resbn.npz"])
def test_module_forward_backward(golden, name):
    """The reference's own fwd / hinge / bwd / Adam steps for each wired tower (dcue/dcue.py:49-59:
    truedcuemel1dbn at H = 32 and 128, truedcuemel1d, truedcuemel1dres, truedcuemel1dresbn), at the
    trainer's default widths (d = 100, H = 128: model_d100) and at odd H / d in the other towers
    (model_w_*: the library's zero-padded storage channels must stay invisible)."""
    g = golden(name)
    net = _net(g, int(g["seed"]))
    u = torch.from_numpy(g["u"]).to(DEV)
    pos = torch.from_numpy(g["pos"]).float().to(DEV)
    neg = torch.from_numpy(g["neg"]).float().to(DEV)
    net.train()
    net.zero_grad()
    scores, uf, pf, nf = net(u, pos, neg)
    for key, val in (("scores", scores), ("uf", uf), ("pf", pf), ("nf", nf)):
        _assert_close(val, g[key], 1e-4, 1e-4, key)
    loss = _hinge(scores)
    _assert_close(loss.detach(), g["loss"], 1e-4, 1e-4, "loss")
    loss.backward()
    torch.cuda.synchronize()
    _check_grads(net, g)
    for k, v in net.state_dict().items():
        if "fwd." + k in g.files:
            if k.endswith("num_batches_tracked"):
                assert int(v) == int(g["fwd." + k]), k
            else:
                _assert_close(v, g["fwd." + k], 1e-4, 1e-4, k)
    assert_storage_pads_zero(net)
    if "step1.conv.fc.weight" not in g.files:
        return
    from dcrecommend.optim import NativeAdam
    lr = float(g["lr"])
    opt = NativeAdam(net.parameters(), lr, (0.9, 0.99), 1e-8, 0)
    opt.step()
    torch.cuda.synchronize()
    _check_params_after_adam(net, g, "step1.", lr, grad_prefix="grad.")
    # second step on the same gradients with weight decay; the user rows of this batch consumed
    # their compact gradient in step 1, so they are excluded (the reference re-applies its dense one)
    opt.param_groups[0]["weight_decay"] = 1e-4
    opt.step()
    torch.cuda.synchronize()
    _check_params_after_adam(net, g, "step2.", 2 * lr, skip_rows=np.unique(g["u"]))
    assert_storage_pads_zero(net)


@pytest.mark.parametrize("H,d", [(64, 64), (128, 64), (256, 128), (128, 256)])  # (128, 64): config 1
def test_widths_against_oracle(H, d):
    """conv_hidden / feature_dim the golden fixtures do not cover (they hold 32 and 128): one train
    step's scores, loss and every dense gradient against the CPU oracle (oracle/dcue_oracle.py, the
    reference step restated). Covers the conv-1 weight gradient's output tiling (one, two or four
    64-channel o tiles) and the 256-wide fc/score paths. Tolerance as test_module_forward_backward."""
    from dcrecommend.dcue.dcue import DCUENet
    from oracle import dcue_oracle as O
    n_users, B, N = 7, 4, 3
    torch.manual_seed(1)
    net = DCUENet({"feature_dim": d, "conv_hidden": H, "user_embdim": 40, "user_count": n_users,
                   "model_type": "truedcuemel1dbn"})
    torch.manual_seed(1)
    p, b = O.init_params(d, H, 40, n_users)
    net = net.to(DEV).train()
    gen = torch.Generator().manual_seed(4)
    u = torch.randint(0, n_users, (B,), generator=gen)
    pos = torch.randn(B, 128, 131, generator=gen).half().float()
    neg = torch.randn(B, N, 128, 131, generator=gen).half().float()
    scores, _, _, _ = net(u.to(DEV), pos.to(DEV), neg.to(DEV))
    loss = torch.max(torch.zeros_like(scores), 0.2 - scores).sum(dim=1).mean()
    loss.backward()
    torch.cuda.synchronize()
    ref_loss, grads, (rs, _, _, _) = O.loss_and_grads(p, b, u, pos, neg)
    assert float((scores.detach().cpu() - rs).abs().max()) <= 1e-4 * float(rs.abs().max()) + 1e-6
    assert abs(float(loss.detach()) - float(ref_loss)) <= 1e-4 * abs(float(ref_loss)) + 1e-7
    named = dict(net.named_parameters())
    for k, g_ref in grads.items():
        if k not in named or named[k].grad is None:
            continue
        g = named[k].grad.detach().cpu()
        scale = float(g_ref.abs().max())
        if scale == 0.0:
            assert float(g.abs().max()) < 1e-6, k
            continue
        assert float((g - g_ref).abs().max()) <= 1e-3 * scale, "%s: %.3e" % (
            k, float((g - g_ref).abs().max()) / scale)


def test_eval_forward(golden):
    g = golden("model_tiny.npz")
    net = _net(g, int(g["seed"]))
    net.load_state_dict({k[len("step2."):]: torch.from_numpy(np.array(g[k])) for k in g.files
                         if k.startswith("step2.")})
    net.eval()
    u = torch.from_numpy(g["u"]).to(DEV)
    pos = torch.from_numpy(g["pos"]).float().to(DEV)
    neg = torch.from_numpy(g["neg"]).float().to(DEV)
    with torch.no_grad():
        scores, uf, pf, nf = net(u, pos, neg)
        feats = net.conv(pos)
        ufe = net.user_embd(u)
    _assert_close(scores, g["eval_scores"], 1e-4, 1e-4, "eval scores")
    _assert_close(uf, g["eval_uf"], 1e-4, 1e-4, "eval uf")
    _assert_close(pf, g["eval_pf"], 1e-4, 1e-4, "eval pf")
    _assert_close(nf, g["eval_nf"], 1e-4, 1e-4, "eval nf")
    _assert_close(feats, g["eval_pf"], 1e-4, 1e-4, "conv(X)")
    _assert_close(ufe, g["eval_uf"], 1e-4, 1e-4, "user_embd(u)")


def test_inbatch_gather_layout(golden):
    """In-batch negatives: the tower runs once per positive; BN stats weight each by its copies."""
    from dcrecommend import _native as nat
    g = golden("inbatch_model.npz")
    net = _net(g, 0)
    B, N = g["r"].shape
    pos = torch.from_numpy(g["pos"]).float().to(DEV)
    table = net._spectro_table(pos)
    users = torch.from_numpy(g["u"]).to(DEV)
    item_track = torch.arange(B, dtype=torch.int32, device=DEV)
    neg_item = torch.from_numpy(g["r"]).to(torch.int32).to(DEV)
    net.train()
    scores, uf, f, loss = net.native_forward(users, table, item_track, N, nat.LAYOUT_GATHER, neg_item,
                                             train=True, margin=0.2)
    _assert_close(scores, g["scores"], 1e-4, 1e-4, "scores")
    _assert_close(uf, g["uf"], 1e-4, 1e-4, "uf")
    _assert_close(f, g["pf"], 1e-4, 1e-4, "item feats")
    _assert_close(loss, g["loss"], 1e-4, 1e-4, "loss")
    net.native_backward(None)
    torch.cuda.synchronize()
    _check_grads(net, g)
    for k, v in net.state_dict().items():
        if "fwd." + k in g.files:
            _assert_close(v, g["fwd." + k], 1e-4, 1e-4, k)


def test_train5_fused_step(golden):
    """Five fused steps (dcue_forward + hinge + dcue_train_backward + dcue_adam_step)."""
    from dcrecommend import _native as nat
    from dcrecommend.optim import NativeAdam
    g = golden("train5.npz")
    net = _net(g, 0)
    opt = NativeAdam(net.parameters(), 1e-3, (0.9, 0.99), 1e-8, 0)
    net.train()
    B, N = int(g["B"]), int(g["N"])
    for s in range(5):
        pos = torch.from_numpy(g["pos"][s]).float().to(DEV)
        neg = torch.from_numpy(g["neg"][s]).float().to(DEV)
        X = torch.cat([pos, neg.reshape(B * N, 128, 131)])
        table = net._spectro_table(X)
        users = torch.from_numpy(g["u"][s]).to(DEV)
        item_track = torch.arange(B * (1 + N), dtype=torch.int32, device=DEV)
        _, _, _, loss = net.native_forward(users, table, item_track, N, nat.LAYOUT_CATALOGUE,
                                           train=True, margin=0.2)
        assert float(loss) == pytest.approx(float(g["loss"][s]), rel=1e-4)
        net.native_backward(None)
        opt.param_groups[0]["lr"] = float(g["lr"][s])
        opt.step()
    torch.cuda.synchronize()
    _check_params_after_adam(net, g, "final.", float(np.sum(g["lr"])))


def _mt_state(seed):
    from dcrecommend import _native as nat
    st = torch.empty(nat.MT_STATE_BYTES, dtype=torch.uint8, device=DEV)
    nat.check(nat.lib().dcue_mt_seed(nat.ptr(st), seed, nat.stream_handle()), "seed")
    return st


@pytest.mark.parametrize("seed", [0, 123456789, 4294967295])
def test_mt_stream(seed):
    from dcrecommend import _native as nat
    st = _mt_state(seed)
    out = torch.empty(2000, dtype=torch.int32, device=DEV)
    # two calls: the state must carry over exactly
    nat.check(nat.lib().dcue_mt_draw(nat.ptr(st), nat.ptr(out), 700, nat.stream_handle()), "draw")
    nat.check(nat.lib().dcue_mt_draw(nat.ptr(st), ctypes_off(out, 700), 1300, nat.stream_handle()), "draw")
    got = out.cpu().numpy().view(np.uint32)
    assert np.array_equal(got, MT.mt_stream(seed, 2000))


def ctypes_off(t, n):
    import ctypes
    return ctypes.c_void_p(t.data_ptr() + n * t.element_size())


@pytest.mark.parametrize("seed", [0, 5, 99])
def test_inbatch_sampler(golden, seed):
    from dcrecommend import _native as nat
    g = golden("inbatch_draws.npz")
    st = _mt_state(seed)
    out = torch.empty((64, 20), dtype=torch.int32, device=DEV)
    nat.check(nat.lib().dcue_sample_inbatch(nat.ptr(st), 64, 20, nat.ptr(out), nat.stream_handle()), "inbatch")
    assert np.array_equal(out.cpu().numpy(), g["seed%d" % seed])
    # the stream continues: a second batch equals numpy's next draws
    nat.check(nat.lib().dcue_sample_inbatch(nat.ptr(st), 64, 20, nat.ptr(out), nat.stream_handle()), "inbatch")
    rs = np.random.RandomState(seed)
    from oracle import dcue_oracle as O
    O.inbatch_negatives(rs, 64, 20)
    assert np.array_equal(out.cpu().numpy(), O.inbatch_negatives(rs, 64, 20))


def test_catalogue_sampler(golden):
    from dcrecommend import _native as nat
    from dcrecommend.datasets.csr import user_split_ranks
    g = golden("catalogue.npz")
    users = {u: i for i, u in enumerate(g["user_categories"])}
    songs = {s: i for i, s in enumerate(g["song_categories"])}
    uidx = np.array([users[u] for u in g["raw_users"]])
    sidx = np.array([songs[s] for s in g["raw_songs"]])
    indptr, ranks = user_split_ranks(uidx, sidx, len(users), g["split_items"])
    N = int(g["N"])
    dev = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(dt).to(DEV)  # noqa: E731
    split, ip, rk = dev(g["split_items"], torch.int64), dev(indptr, torch.int64), dev(ranks, torch.int32)
    us = dev(g["users_seq"], torch.int64)
    out = torch.empty((len(g["users_seq"]), N), dtype=torch.int64, device=DEV)
    nat.check(nat.lib().dcue_sample_catalogue(None, 1, 1234, nat.ptr(split), split.numel(), nat.ptr(ip),
                                              nat.ptr(rk), nat.ptr(us), us.numel(), N, nat.ptr(out),
                                              nat.stream_handle()), "catalogue seeded")
    assert np.array_equal(out.cpu().numpy(), g["seeded"])
    st = _mt_state(77)
    nat.check(nat.lib().dcue_sample_catalogue(nat.ptr(st), 0, 0, nat.ptr(split), split.numel(), nat.ptr(ip),
                                              nat.ptr(rk), nat.ptr(us), us.numel(), N, nat.ptr(out),
                                              nat.stream_handle()), "catalogue stream")
    assert np.array_equal(out.cpu().numpy(), g["stream"])


@pytest.mark.parametrize("N", [20, 1, 300])
def test_catalogue_sampler_groups_and_long_lists(N):
    """The global-stream sampler stages rank lists in LDS per group of samples: cover several
    groups, a list longer than the LDS stage (scanned in global memory), a user with one candidate
    (bounded draw over [0, 0]) and users with no split items, against the C MT19937 oracle
    (the algorithm of datasets/dcuedataset.py:207-220 on numpy's stream)."""
    from dcrecommend import _native as nat
    from dcrecommend.datasets.csr import user_split_ranks
    from oracle import mt19937 as MT
    rs = np.random.RandomState(5)
    n_songs, n_users = 12000, 300
    split = np.sort(rs.choice(n_songs, 10000, replace=False)).astype(np.int64)
    pairs = [(0, int(x)) for x in rs.choice(split, 9000, replace=False)]  # > the 8192-rank stage
    pairs += [(1, int(x)) for x in split[1:]]                              # one candidate left
    for u in range(3, n_users):                                            # user 2: none
        pairs += [(u, int(x)) for x in rs.choice(n_songs, rs.randint(0, 60), replace=False)]
    uidx = np.array([p[0] for p in pairs], dtype=np.int64)
    sidx = np.array([p[1] for p in pairs], dtype=np.int64)
    order = np.lexsort((sidx, uidx))
    uidx, sidx = uidx[order], sidx[order]
    indptr_items = np.zeros(n_users + 1, dtype=np.int64)
    np.add.at(indptr_items, uidx + 1, 1)
    indptr_items = np.cumsum(indptr_items)
    users_seq = rs.randint(0, n_users, 700).astype(np.int64)
    users_seq[[3, 250, 251, 600]] = [0, 1, 0, 2]
    want = MT.catalogue(77, False, split, indptr_items, sidx, users_seq, N)
    indptr, ranks = user_split_ranks(uidx, sidx, n_users, split)
    dev = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(dt).to(DEV)  # noqa: E731
    sp, ip, rk, us = (dev(split, torch.int64), dev(indptr, torch.int64), dev(ranks, torch.int32),
                      dev(users_seq, torch.int64))
    st = _mt_state(77)
    out = torch.empty((len(users_seq), N), dtype=torch.int64, device=DEV)
    nat.check(nat.lib().dcue_sample_catalogue(nat.ptr(st), 0, 0, nat.ptr(sp), sp.numel(), nat.ptr(ip),
                                              nat.ptr(rk), nat.ptr(us), us.numel(), N, nat.ptr(out),
                                              nat.stream_handle()), "catalogue stream")
    assert np.array_equal(out.cpu().numpy(), want)
    # the stream continues where the oracle's does: the next call equals its next samples
    nxt = rs.randint(3, n_users, 50).astype(np.int64)
    both = MT.catalogue(77, False, split, indptr_items, sidx, np.concatenate([users_seq, nxt]), N)
    us2 = dev(nxt, torch.int64)
    out2 = torch.empty((len(nxt), N), dtype=torch.int64, device=DEV)
    nat.check(nat.lib().dcue_sample_catalogue(nat.ptr(st), 0, 0, nat.ptr(sp), sp.numel(), nat.ptr(ip),
                                              nat.ptr(rk), nat.ptr(us2), us2.numel(), N, nat.ptr(out2),
                                              nat.stream_handle()), "catalogue stream 2")
    assert np.array_equal(out2.cpu().numpy(), both[len(users_seq):])
