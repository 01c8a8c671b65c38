"""GPU parity of the mixed audio + text item tower (BASELINE config 4, model_type
'truedcuemel1dbntext', csrc/text.hip) against oracle/text_oracle.py.

PARITY UNPINNED against the reference: it never published a text encoder (its text item set imports a
WordEmbeddings module that does not exist, reference datasets/dcuelmitemset.py:8). The token rows
follow its data contract (BOS + sentence + EOS, PAD-padded, dcuelmitemset.py:40-56) and the checks
hold the library to the fp64 restatement of this build's encoder at config 4's width d = 256:

  forward outputs (scores, user / item features, loss) within 1e-4 of the output's max (north_star);
  gradients within 1e-3 (abs floor 1e-4 of max), as tests/test_gpu_parity.py;
  one NativeAdam step: every parameter within 2 lr (+1e-4 of max) of the oracle's torch.optim.Adam.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
D, H, E_U = 256, 128, 300
TD, WD, T, V, PAD = 256, 300, 64, 500, 0


def _close(got, ref, rtol, afrac, what):
    got = torch.as_tensor(got).double().cpu()
    ref = torch.as_tensor(ref).double().cpu()
    atol = afrac * max(float(ref.abs().max()), 1e-30)
    err = (got - ref).abs()
    bad = err > atol + rtol * ref.abs()
    assert not bool(bad.any()), "%s: max err %.3e of max %.3e" % (what, float(err.max()), float(ref.abs().max()))


def _args(n_users, td=TD, wd=WD, t=T):
    return {"feature_dim": D, "conv_hidden": H, "user_embdim": E_U, "user_count": n_users,
            "model_type": "truedcuemel1dbntext", "text_dim": td, "word_dim": wd, "text_len": t,
            "n_words": V, "pad_idx": PAD}


def _pair(n_users, seed=0, **kw):
    from dcrecommend.dcue.dcue import DCUENet
    from oracle import text_oracle as TO
    a = _args(n_users, **kw)
    torch.manual_seed(seed)
    net = DCUENet(a)
    torch.manual_seed(seed)
    p, b = TO.init_params(D, H, E_U, n_users, a["text_dim"], a["word_dim"], V)
    return net, p, b


def test_text_init_matches_oracle():
    """DCUENet's text tower builds the oracle's parameters in the same RNG order (bit-exact)."""
    net, p, b = _pair(7)
    sd = net.state_dict()
    for k, v in p.items():
        assert torch.equal(sd[k], v), k
    assert not net.text.embeddings.weight.requires_grad


@pytest.mark.parametrize("td,wd,t", [(TD, WD, T), (100, 64, 20), (40, 128, 128)])
def test_text_module_step(td, wd, t):
    """Catalogue-layout step through DCUENet.forward (the reference's [pos; neg] stack, with each
    item's token row): scores / features / loss 1e-4, every trainable gradient 1e-3 of the fp64
    oracle, then one NativeAdam step within the lr budget. Widths: config 4 (256 / 300 / 64) and two
    odd ones (padded text channels, a 64-wide and a 128-wide word width, short and long sentences)."""
    from dcrecommend.optim import NativeAdam
    from oracle import text_oracle as TO
    from oracle import dcue_oracle as O
    n_users, B, N = 9, 4, 3
    net, p, b = _pair(n_users, td=td, wd=wd, t=t)
    net = net.to(DEV).train()
    gen = torch.Generator().manual_seed(11)
    u = torch.randint(0, n_users, (B,), generator=gen)
    pos = torch.randn(B, 128, 131, generator=gen).half().float()
    neg = torch.randn(B, N, 128, 131, generator=gen).half().float()
    pt = TO.sentences(gen, B, t, V, PAD, min_len=0)
    nt = TO.sentences(gen, B * N, t, V, PAD, min_len=0).reshape(B, N, t)
    scores, uf, pf, nf = net(u.to(DEV), pos.to(DEV), neg.to(DEV), pt.to(DEV), nt.to(DEV))
    loss = torch.max(torch.zeros_like(scores), 0.2 - scores).sum(dim=1).mean()
    loss.backward()
    torch.cuda.synchronize()
    p64 = {k: v.double() for k, v in p.items()}
    b64 = {k: (v.double() if v.is_floating_point() else v.clone()) for k, v in b.items()}
    ref_loss, g64, (rs, ruf, rpf, rnf) = TO.loss_and_grads(p64, b64, u, pos.double(), neg.double(), pt, nt, PAD)
    _close(scores.detach(), rs, 1e-4, 1e-4, "scores")
    _close(uf.detach(), ruf, 1e-4, 1e-4, "user feats")
    _close(pf.detach(), rpf, 1e-4, 1e-4, "positive feats")
    _close(nf.detach(), rnf, 1e-4, 1e-4, "negative feats")
    _close(loss.detach(), ref_loss, 1e-4, 1e-4, "loss")
    named = dict(net.named_parameters())
    for k, g_ref in g64.items():
        got = net.embedding_grad_dense() if k == "user_embd.embeddings.weight" else named[k].grad
        _close(got, g_ref, 1e-3, 1e-4, "grad " + k)
    assert named["text.embeddings.weight"].grad is None
    # one Adam step (NativeAdam) against the oracle's torch.optim.Adam on the oracle's fp32 gradients
    lr = 1e-3
    opt = NativeAdam(net.parameters(), lr, (0.9, 0.99), 1e-8, 0)
    opt.step()
    torch.cuda.synchronize()
    _, g32, _ = TO.loss_and_grads(p, {k: v.clone() for k, v in b.items()}, u, pos, neg, pt, nt, PAD)
    trainable = {k: v for k, v in p.items() if k in g32}
    adam = O.AdamState(trainable)
    adam.step(trainable, g32, lr)
    sd = net.state_dict()
    for k, ref in trainable.items():
        diff = (sd[k].double().cpu() - ref.double()).abs()
        assert float(diff.max()) <= 2 * lr + 1e-4 * float(ref.abs().max()), (k, float(diff.max()))
    assert torch.equal(sd["text.embeddings.weight"].cpu(), p["text.embeddings.weight"]), "frozen words moved"
    from test_gpu_parity import assert_storage_pads_zero
    assert_storage_pads_zero(net)


def test_text_eval_tower():
    """Eval-mode item features (running BN statistics, DCUENet.conv(X, tokens)) at 1e-4."""
    from oracle import text_oracle as TO
    net, p, b = _pair(5, seed=3)
    net = net.to(DEV).eval()
    gen = torch.Generator().manual_seed(4)
    X = torch.randn(12, 128, 131, generator=gen).half().float()
    tok = TO.sentences(gen, 12, T, V, PAD)
    with torch.no_grad():
        f = net.item_features(X.to(DEV), tok.to(DEV))
    p64 = {k: v.double() for k, v in p.items()}
    b64 = {k: (v.double() if v.is_floating_point() else v.clone()) for k, v in b.items()}
    ref = TO.item_tower(p64, b64, X.double(), tok, PAD, train=False)
    _close(f, ref, 1e-4, 1e-4, "eval item features")


def test_text_plan_inbatch_bench_shape():
    """The bench's in-batch plan (B = 64, N = 20, compact tower over the 64 positives, deferred
    user table) with the text tower at config 4's widths: step 0 scores and loss 1e-4 and every
    gradient 1e-3 of the fp64 oracle on the reference's literal [pos; neg] stack; steps 1-2 (plan.step
    with the fused Adam) loss 1e-4 of the oracle's trajectory."""
    from dcrecommend import _native as nat
    from dcrecommend.dcue.plan import TrainPlan
    from dcrecommend.optim import NativeAdam
    from oracle import dcue_oracle as O
    from oracle import text_oracle as TO
    B, N, n_users, n_tracks = 64, 20, 300, 500
    net, p, b = _pair(n_users, seed=2)
    net = net.to(DEV).train()
    opt = NativeAdam(net.parameters(), 1e-4, (0.9, 0.99), 1e-8, 0, defer_embedding=True)
    gen = torch.Generator().manual_seed(8)
    X = torch.randn(n_tracks, 128, 131, generator=gen).half().float()
    table = X.half().transpose(1, 2).contiguous().to(DEV)
    toks = TO.sentences(gen, n_tracks, T, V, PAD)
    tok_d = toks.to(DEV)
    mt = torch.empty(nat.MT_STATE_BYTES, dtype=torch.uint8, device=DEV)
    nat.check(nat.lib().dcue_mt_seed(nat.ptr(mt), 21, nat.stream_handle()), "mt_seed")
    rs = np.random.RandomState(21)
    plan = TrainPlan(net, table, B, N, mt_state=mt, optimizer=opt, tokens=tok_d)
    off = nat.workspace_outputs(net._flat["dims"], B, N, B)
    adam = None
    lrs = [1e-4, 2e-4, 1e-4]
    for step, lr in enumerate(lrs):
        u = torch.randint(0, n_users, (B,), generator=gen)
        items = torch.randint(0, n_tracks, (B,), generator=gen)
        r = torch.from_numpy(O.inbatch_negatives(rs, B, N))
        neg_items = items[r.reshape(-1)].reshape(B, N)
        pos, neg = X[items], X[neg_items.reshape(-1)].reshape(B, N, 128, 131)
        pt, nt = toks[items], toks[neg_items.reshape(-1)].reshape(B, N, T)
        opt.param_groups[0]["lr"] = lr
        if step == 0:
            plan.launch(u.to(DEV), items.to(torch.int32).to(DEV))
            torch.cuda.synchronize()
            assert torch.equal(plan.neg_item.cpu().long(), r), "in-batch draws differ from numpy"
            p64 = {k: v.double() for k, v in p.items()}
            b64 = {k: (v.double() if v.is_floating_point() else v.clone()) for k, v in b.items()}
            ref_loss, g64, (rsc, ruf, rpf, rnf) = TO.loss_and_grads(p64, b64, u, pos.double(), neg.double(),
                                                                     pt, nt, PAD)
            sc = net._ws[off[0]:off[0] + 4 * B * N].view(torch.float32).view(B, N)
            _close(sc, rsc, 1e-4, 1e-4, "scores")
            _close(plan.loss, ref_loss, 1e-4, 1e-4, "loss")
            named = dict(net.named_parameters())
            for k, g_ref in g64.items():
                got = net.embedding_grad_dense() if k == "user_embd.embeddings.weight" else named[k].grad
                _close(got, g_ref, 1e-3, 1e-4, "grad " + k)
            opt.step()
            _, g32, _ = TO.loss_and_grads(p, b, u, pos, neg, pt, nt, PAD)
            trainable = {k: v for k, v in p.items() if k in g32}
            adam = O.AdamState(trainable)
            adam.step(trainable, g32, lr)
        else:
            plan.step(u.to(DEV), items.to(torch.int32).to(DEV))
            torch.cuda.synchronize()
            trainable = {k: v for k, v in p.items() if k != "text.embeddings.weight"}
            leaves_loss, g32, _ = TO.loss_and_grads(p, b, u, pos, neg, pt, nt, PAD)
            adam.step(trainable, g32, lr)
            _close(plan.loss, leaves_loss, 1e-4, 1e-4, "step %d loss" % step)
    plan.close()


def test_text_fwd_kernels_bit_identical(tmp_path):
    """The gather-once text forward (k_text_fwd_full, the default), its two-position-part form
    (DCUE_TEXT_PARTS=2: halves of the positions merged through tickets), a two-column-tile shape
    (DCUE_TEXT_FWD=4x2), a deeper weight prefetch (DCUE_TEXT_BPD=15) and the chunked kernel
    (DCUE_TEXT_FWD=chunked) run the same MFMA sequence per accumulator and the same first-maximum
    rule: five plan steps of the text tower (tests/race_worker.py) give bit-identical losses, dense
    parameters and user table."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys, torch; sys.path.insert(0, %r); import race_worker as W; r = W.run('text'); "
            "torch.save({k: r[k] for k in ('loss', 'P', 'emb')}, sys.argv[1])" % os.path.join(root, "tests"))
    res = []
    for i, extra in enumerate(({}, {"DCUE_TEXT_FWD": "chunked"}, {"DCUE_TEXT_PARTS": "2"},
                               {"DCUE_TEXT_FWD": "4x2"}, {"DCUE_TEXT_BPD": "15"})):
        out = str(tmp_path / ("t%d.pt" % i))
        env = dict(os.environ, **extra)
        for k in ("DCUE_TEXT_FWD", "DCUE_TEXT_PARTS", "DCUE_TEXT_BPD"):
            if k not in extra:
                env.pop(k, None)
        p = subprocess.run([sys.executable, "-c", code, out], env=env, stdout=subprocess.PIPE,
                           stderr=subprocess.STDOUT, text=True, timeout=100)
        assert p.returncode == 0, p.stdout[-3000:]
        res.append(torch.load(out, weights_only=True))
    for r in res[1:]:
        for k in ("loss", "P", "emb"):
            assert torch.equal(res[0][k], r[k]), k
