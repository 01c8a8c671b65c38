"""Rank of tests/test_gpu_dp.py (a child process; RANK, WORLD_SIZE, MASTER_* and OUT in the env).

Two ranks share cuda:0 over gloo. Each launches the same catalogue-layout step twice on its own
users: the first time the local gradient is synchronised and all-reduced plainly (the reference
mean); the second time dcrecommend.distributed.allreduce_mean_overlapped_ all-reduces it in two
buckets straight behind the launch, the larger one ordered only by the plan's side-stream event.
"""
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "amplifai-deepcontentrecommenders_amd"))


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dcrecommend import distributed as D
    from dcrecommend.dcue.dcue import DCUENet
    from dcrecommend.dcue.plan import TrainPlan
    dev = "cuda:0"
    B, N, n_users, n_tracks = 8, 3, 40, 48
    torch.manual_seed(5)
    net = DCUENet({"feature_dim": 32, "conv_hidden": 32, "user_embdim": 40, "user_count": n_users,
                   "model_type": "truedcuemel1dbn"}).cuda().train()
    gen = torch.Generator(device=dev).manual_seed(11)
    tracks = torch.randn((n_tracks, 131, 128), generator=gen, device=dev).half()
    gen.manual_seed(100 + rank)  # each rank its own batch
    users = torch.randint(0, n_users, (B,), generator=gen, device=dev)
    items = torch.randint(0, n_tracks, (B * (1 + N),), generator=gen, device=dev).to(torch.int32)
    plan = TrainPlan(net, tracks, B, N, mt_state=None, emb_grad_scale=1.0 / world)
    G = net._flat["G"]
    late = D.late_grad_floats(net)
    plan.launch(users, items)
    torch.cuda.synchronize()
    ref = G.clone()
    D.allreduce_mean_(ref)
    for _ in range(3):  # the same step again: overlapped buckets right behind the launch
        plan.launch(users, items)
        D.allreduce_mean_overlapped_(plan, G, late)
        torch.cuda.synchronize()
        if not torch.equal(G, ref):
            bad = (G != ref).nonzero().flatten()
            print("rank %d: %d mismatches, first at %d (late = %d)" % (rank, bad.numel(), int(bad[0]), late))
            sys.exit(3)
    torch.save({"G": G.cpu(), "late": late}, os.path.join(os.environ["OUT"], "r%d.pt" % rank))
    plan.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
