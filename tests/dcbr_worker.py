"""Rank of tests/test_gpu_dcbr_dp.py (a child process; RANK, WORLD_SIZE, MASTER_*, OUT in the env).

Two ranks share cuda:0 over gloo; the library's communicator runs over its host transport
(distributed.HostComm: the same exchange code as over RCCL, each collective summed by gloo).

WRMF, row-sharded (config 5's ALS over 2 ranks): two iterations with the communicator bound against
a one-rank fit of the same data on every rank: user and item factors bit-exact (each row is solved
exactly as on one GPU, then all-gathered).

DCBR regression, data parallel: each rank steps its own item batches with the communicator bound
(dense gradient averaged over the ranks before Adam) against a twin model stepped with
loss_and_grads + a plain all-reduce mean + NativeAdam.step(): bit-exact, and one replica across the
ranks.
"""
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "amplifai-deepcontentrecommenders_amd"))

DEV = "cuda:0"


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from dcrecommend import distributed as D
    from dcrecommend.dcbr import DCBR, WRMF
    comm = D.HostComm()
    # ---- WRMF: the same interactions on every rank
    g = torch.Generator().manual_seed(3)
    n_users, n_items, nnz, dim = 37, 53, 400, 24
    u = torch.randint(0, n_users, (nnz,), generator=g)
    i = torch.randint(0, n_items, (nnz,), generator=g)
    v = torch.rand(nnz, generator=g) * 3
    dp = WRMF(factors=dim, regularization=0.05, alpha=10.0, iterations=2, seed=1, device=DEV, comm=comm)
    dp.fit(u, i, v, n_users=n_users, n_items=n_items)
    one = WRMF(factors=dim, regularization=0.05, alpha=10.0, iterations=2, seed=1, device=DEV)
    one.fit(u, i, v, n_users=n_users, n_items=n_items)
    torch.cuda.synchronize()
    wrmf_ok = torch.equal(dp.user_factors, one.user_factors) and torch.equal(dp.item_factors, one.item_factors)
    # ---- DCBR regression: rank-local item batches, twin models
    n_tracks, M = 40, 12
    tg = torch.Generator(device=DEV).manual_seed(9)
    tracks = torch.randn(n_tracks, 131, 128, generator=tg, device=DEV).half()
    targets = torch.randn(n_tracks, 32, generator=tg, device=DEV) * 0.3
    torch.manual_seed(4)
    a = DCBR(feature_dim=32, conv_hidden=32, lr=1e-3, device=DEV, comm=comm)
    torch.manual_seed(4)
    b = DCBR(feature_dim=32, conv_hidden=32, lr=1e-3, device=DEV)
    bg = torch.Generator().manual_seed(100 + rank)
    for _ in range(3):
        items = torch.randint(0, n_tracks, (M,), generator=bg).to(torch.int32).to(DEV)
        a.step(tracks, items, targets[items.long()])
        b.loss_and_grads(tracks, items, targets[items.long()])
        torch.cuda.synchronize()
        D.allreduce_mean_(b.net._flat["G"])
        b.opt.step()
    torch.cuda.synchronize()
    same_twin = torch.equal(a.net._flat["P"], b.net._flat["P"])
    same, lo, hi = D.replica_checksums(a.net._flat["P"])
    torch.save({"wrmf_ok": wrmf_ok, "twin": same_twin, "replicas": same, "P": a.net._flat["P"].cpu()},
               os.path.join(os.environ["OUT"], "r%d.pt" % rank))
    print("rank %d: wrmf bit-exact %s, dcbr twin bit-exact %s, replicas identical %s" % (rank, wrmf_ok, same_twin, same),
          flush=True)
    comm.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
