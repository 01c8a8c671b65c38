"""Worker for tests/test_gpu_schedule.py: five in-batch plan steps (B = 16, N = 5, deferred user
table, fused Adam) at fixed seeds under whatever scheduling environment the parent set
(DCUE_SIDE_THREAD, DCUE_SCORE_FORK, DCUE_PROLOGUE_FIRST, DCUE_LATE_WAIT, DCUE_AHEAD_AT,
DCUE_USER_FWD); saves the losses, the dense parameters and the flushed user table to $OUT."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "amplifai-deepcontentrecommenders_amd"))


def main():
    from dcrecommend import _native as nat
    from dcrecommend.dcue.dcue import DCUENet
    from dcrecommend.dcue.plan import TrainPlan
    from dcrecommend.optim import NativeAdam
    dev = "cuda:0"
    B, N, n_users, n_tracks = 16, 5, 40, 60
    torch.manual_seed(0)
    net = DCUENet({"feature_dim": 64, "conv_hidden": 64, "user_embdim": 48, "user_count": n_users,
                   "model_type": "truedcuemel1dbn"}).to(dev).train()
    opt = NativeAdam(net.parameters(), 1e-3, (0.9, 0.99), 1e-8, 0, defer_embedding=True, flush_every=3)
    gen = torch.Generator().manual_seed(1)
    X = torch.randn(n_tracks, 128, 131, generator=gen).half()
    table = X.transpose(1, 2).contiguous().to(dev)
    mt = torch.empty(nat.MT_STATE_BYTES, dtype=torch.uint8, device=dev)
    nat.check(nat.lib().dcue_mt_seed(nat.ptr(mt), 7, nat.stream_handle()), "mt_seed")
    plan = TrainPlan(net, table, B, N, mt_state=mt, optimizer=opt)
    users = [torch.randint(0, n_users, (B,), generator=gen).to(dev) for _ in range(6)]
    items = [torch.randint(0, n_tracks, (B,), generator=gen).to(torch.int32).to(dev) for _ in range(6)]
    losses = []
    for s in range(5):
        plan.set_next(items[s + 1])
        plan.step(users[s], items[s])
        losses.append(plan.loss.detach().clone())
    torch.cuda.synchronize()
    opt.flush()
    sd = net.state_dict()
    torch.save({"loss": torch.stack(losses).cpu(), "P": net._flat["P"].detach().cpu(),
                "emb": sd["user_embd.embeddings.weight"].cpu(), "fail_flags": nat.debug_fail_flags()},
               os.environ["OUT"])
    plan.close()
    print("schedule worker ok", os.environ.get("DCUE_SIDE_THREAD"), os.environ.get("DCUE_SCORE_FORK"),
          [float(x) for x in losses])
    return 0


if __name__ == "__main__":
    sys.exit(main())
