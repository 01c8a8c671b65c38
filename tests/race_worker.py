"""Schedule-perturbation runs for tests/test_gpu_races.py: a few back-to-back plan steps (nothing
synchronised between them, as in training and the bench) at fixed seeds, with spin kernels injected
ahead of the work at chosen sites (include/dcue.h dcue_debug_delay). Returns the per-step losses, the
dense parameters and the flushed user table.

Run as a script (the parent sets DCUE_LEGACY_ORDERS=1 to get round 4's cross-stream orders) it prints
one JSON line: for each delayed site, whether the run matched the undelayed one bit for bit and
whether it stayed finite."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "amplifai-deepcontentrecommenders_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

DEV = "cuda:0"
TOWERS = {
    "bn": {"feature_dim": 64, "conv_hidden": 64, "model_type": "truedcuemel1dbn"},
    "res": {"feature_dim": 64, "conv_hidden": 64, "model_type": "truedcuemel1dresbn"},
    "text": {"feature_dim": 64, "conv_hidden": 64, "model_type": "truedcuemel1dbntext", "text_dim": 64,
             "word_dim": 32, "text_len": 16, "n_words": 50, "pad_idx": 0},
    # 32 positions: two 16-position tiles, so DCUE_TEXT_PARTS=2 splits each item over two workgroups
    # that merge through the accumulator block's tickets (text.hip k_text_fwd_full)
    "text32": {"feature_dim": 64, "conv_hidden": 64, "model_type": "truedcuemel1dbntext", "text_dim": 64,
               "word_dim": 32, "text_len": 32, "n_words": 50, "pad_idx": 0},
}


def run(tower="bn", delays=None, steps=5, inbatch=True, check=None, B=16, N=5):
    """Steps of one fresh model under `delays` ({site: microseconds}); returns loss / P / emb (CPU)."""
    from dcrecommend import _native as nat
    from dcrecommend.dcue.dcue import DCUENet
    from dcrecommend.dcue.plan import TrainPlan
    from dcrecommend.optim import NativeAdam
    n_users, n_tracks = 40, 60
    args = dict(TOWERS[tower], user_embdim=48, user_count=n_users)
    torch.manual_seed(0)
    net = DCUENet(args).to(DEV).train()
    opt = NativeAdam(net.parameters(), 1e-3, (0.9, 0.99), 1e-8, 0, defer_embedding=True, flush_every=3)
    gen = torch.Generator().manual_seed(1)
    X = torch.randn(n_tracks, 128, 131, generator=gen).half()
    table = X.transpose(1, 2).contiguous().to(DEV)
    tokens = None
    if tower.startswith("text"):
        from oracle import text_oracle as TO
        tokens = TO.sentences(gen, n_tracks, args["text_len"], args["n_words"], args["pad_idx"]).to(DEV)
    M = B if inbatch else B * (1 + N)
    users = [torch.randint(0, n_users, (B,), generator=gen).to(DEV) for _ in range(steps + 1)]
    items = [torch.randint(0, n_tracks, (M,), generator=gen).to(torch.int32).to(DEV) for _ in range(steps + 1)]
    if inbatch:
        mt = torch.empty(nat.MT_STATE_BYTES, dtype=torch.uint8, device=DEV)
        nat.check(nat.lib().dcue_mt_seed(nat.ptr(mt), 7, nat.stream_handle()), "mt_seed")
        plan = TrainPlan(net, table, B, N, mt_state=mt, optimizer=opt, tokens=tokens, check=check)
    else:
        plan = TrainPlan(net, table, B, N, item_track=items[0], optimizer=opt, tokens=tokens, check=check)
    torch.cuda.synchronize()
    for site, us in (delays or {}).items():
        nat.debug_delay(site, us)
    losses = []
    try:
        for s in range(steps):
            if inbatch:
                plan.set_next(items[s + 1])
            plan.step(users[s], items[s])
            losses.append(plan.loss.detach().clone())
        torch.cuda.synchronize()
    finally:
        nat.debug_clear_delays()
    probes = plan.probe_report()
    if plan._probes is not None:
        plan._probes.reset()  # reported here: close() need not raise
    opt.flush()
    sd = net.state_dict()
    out = {"loss": torch.stack(losses).cpu(), "P": net._flat["P"].detach().cpu(),
           "emb": sd["user_embd.embeddings.weight"].cpu(), "probes": probes}
    plan.close()
    torch.cuda.synchronize()
    return out


def same(a, b):
    return all(torch.equal(a[k], b[k]) for k in ("loss", "P", "emb"))


def finite(a):
    return all(bool(torch.isfinite(a[k]).all()) for k in ("loss", "P", "emb"))


def main():
    tower = sys.argv[1] if len(sys.argv) > 1 else "bn"
    sites = sys.argv[2].split(",") if len(sys.argv) > 2 else ["wgrad_2", "dgrad_2"]
    us = int(sys.argv[3]) if len(sys.argv) > 3 else 5000
    base = run(tower)
    res = {"legacy_orders": os.environ.get("DCUE_LEGACY_ORDERS", "0"), "base_finite": finite(base)}
    for site in sites:
        r = run(tower, {site: us}, check="probe")
        res[site] = {"identical": same(r, base), "finite": finite(r), "loss": [float(x) for x in r["loss"]],
                     "first_bad": [p[0] for p in r["probes"]][:3]}
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())
