#!/usr/bin/env python
"""DCUE training-step throughput on MI355X (BASELINE.json config 2; weak scaling over GPUs).

One step = the reference's per-batch hot loop (nn/dcue.py:202-210) on one batch of synthetic
input already resident in HBM: in-batch negative draws (MT19937, bit-exact with numpy) ->
forward (item ConvNet over the batch's tracks, user tower, cosine scores, hinge loss) -> backward ->
[RCCL all-reduce of the dense gradient when N>1] -> Adam over every parameter incl. the whole user
table -> cyclic LR schedule. Prints ONE JSON line on rank 0.

  python bench.py [--gpus N --steps K --warmup W]         (N>1: torch.distributed.run, one rank/GPU)
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "amplifai-deepcontentrecommenders_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--mode", choices=["inbatch", "catalogue"], default="inbatch")
    ap.add_argument("--users", type=int, default=100_000)
    ap.add_argument("--tracks", type=int, default=200_000)
    ap.add_argument("--interactions", type=int, default=5_000_000)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--neg", type=int, default=20)
    ap.add_argument("--feature-dim", type=int, default=128)
    ap.add_argument("--hidden", type=int, default=128)
    ap.add_argument("--user-embdim", type=int, default=300)
    ap.add_argument("--cpu-steps", type=int, default=6)
    ap.add_argument("--dense-embedding-adam", action="store_true",
                    help="step every user row every step (the literal sweep) instead of the deferred, "
                         "bit-identical replay")
    ap.add_argument("--flush-every", type=int, default=64)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def synthetic_tracks(n, device, seed):
    """[n][131][128] fp16 spectrograms (randn rounded to fp16: lossless in the fp16 table)."""
    gen = torch.Generator(device=device).manual_seed(seed)
    table = torch.empty((n, 131, 128), dtype=torch.float16, device=device)
    step = 8192
    for s in range(0, n, step):
        e = min(n, s + step)
        table[s:e] = torch.randn((e - s, 131, 128), generator=gen, device=device).half()
    return table


def cpu_baseline(args, n_users_local):
    """The oracle (torch-CPU restatement of the reference step) on a bounded sample of the same
    workload: in-batch negatives are copies of positives run through the tower, as the reference's
    in-batch sampler builds them (nn/dcue.py:698-709)."""
    from oracle import dcue_oracle as O
    torch.manual_seed(0)
    B, N = args.batch, args.neg
    p, b = O.init_params(args.feature_dim, args.hidden, args.user_embdim, n_users_local)
    adam = O.AdamState(p)
    rs = np.random.RandomState(0)
    gen = torch.Generator().manual_seed(1)
    batches = []
    for _ in range(args.cpu_steps + 2):
        u = torch.randint(0, n_users_local, (B,), generator=gen)
        pos = torch.randn(B, 128, 131, generator=gen).half().float()
        r = torch.from_numpy(O.inbatch_negatives(rs, B, N))
        batches.append((u, pos, pos[r.reshape(-1)].reshape(B, N, 128, 131)))
    for u, pos, neg in batches[:2]:
        O.train_step(p, b, adam, u, pos, neg, 1e-5)
    t0 = time.perf_counter()
    for u, pos, neg in batches[2:]:
        O.train_step(p, b, adam, u, pos, neg, 1e-5)
    dt = time.perf_counter() - t0
    rows = B * args.cpu_steps / dt
    return {"value": rows * N, "unit": "triplets/s", "rows_per_s": rows, "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": "%d oracle train steps (after 2 warm-up) at B=%d, N=%d in-batch, d=%d, H=%d, "
                      "%d users, torch-CPU fp32, %.1f s" % (args.cpu_steps, B, N, args.feature_dim,
                                                            args.hidden, n_users_local, dt)}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from dcrecommend import _native as nat
    from dcrecommend.dcue.dcue import DCUENet
    from dcrecommend.optim import NativeAdam
    from dcrecommend.optim.cyclic_scheduler import CyclicLRWithRestarts

    B, N = args.batch, args.neg
    # users are sharded across ranks (row u of rank r = global user u*world + r): each rank owns its
    # users' embedding rows + Adam moments; the track table is replicated
    n_users_local = (args.users + world - 1 - rank) // world
    tracks = synthetic_tracks(args.tracks, dev, seed=1234)
    gen = torch.Generator(device=dev).manual_seed(100 + rank)
    n_pairs = args.interactions // world
    pair_user = torch.randint(0, n_users_local, (n_pairs,), generator=gen, device=dev)
    pair_track = torch.randint(0, args.tracks, (n_pairs,), generator=gen, device=dev, dtype=torch.int64)

    torch.manual_seed(0)  # identical dense init on every rank (DDP-style replicas)
    net = DCUENet({"feature_dim": args.feature_dim, "conv_hidden": args.hidden,
                   "user_embdim": args.user_embdim, "user_count": n_users_local,
                   "model_type": "truedcuemel1dbn"}).to(dev)
    net.train()
    defer = not args.dense_embedding_adam
    opt = NativeAdam(net.parameters(), 1e-5, (0.9, 0.99), 1e-8, 0, defer_embedding=defer,
                     flush_every=args.flush_every)
    epoch_size = (int(math.ceil(n_pairs / 10)) // B) * B
    sched = CyclicLRWithRestarts(opt, B, epoch_size=epoch_size, restart_period=30, t_mult=2, policy="cosine")
    sched.step()

    # batch composition (DataLoader shuffle over the interaction rows) is prepared ahead, like the
    # reference's worker processes; the step consumes HBM-resident index vectors
    total = args.warmup + args.steps
    perm = torch.randperm(n_pairs, generator=gen, device=dev)[: total * B].view(total, B)
    users_b = pair_user[perm].contiguous()
    items_b = pair_track[perm].to(torch.int32).contiguous()
    mt = torch.empty(nat.MT_STATE_BYTES, dtype=torch.uint8, device=dev)
    nat.check(nat.lib().dcue_mt_seed(nat.ptr(mt), 10 + rank, nat.stream_handle()), "mt_seed")
    neg_item = torch.empty((B, N), dtype=torch.int32, device=dev)
    G = net._flat["G"]
    adam_state = opt._adam_state()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]

    if args.mode == "catalogue":
        raise SystemExit("catalogue mode bench: use --mode inbatch (config 2); catalogue runs in tests")

    def step(s, timed):
        nat.check(nat.lib().dcue_sample_inbatch(nat.ptr(mt), B, N, nat.ptr(neg_item), nat.stream_handle()),
                  "sample_inbatch")
        net.native_forward(users_b[s], tracks, items_b[s], N, nat.LAYOUT_GATHER, neg_item, train=True,
                           margin=0.2, copy_outputs=False)
        net.native_backward(None, emb_grad_scale=1.0 / world)
        if world > 1:
            dist.all_reduce(G)
            G.div_(world)
        g = opt.param_groups[0]
        opt.step_count += 1
        model = net._model_struct(adam_state)
        emb_args = nat.AdamArgs(float(g["lr"]), 0.9, 0.99, 1e-8, float(g["weight_decay"]), opt.step_count,
                                nat.ADAM_EMBEDDING)
        dense_args = nat.AdamArgs(float(g["lr"]), 0.9, 0.99, 1e-8, float(g["weight_decay"]), opt.step_count,
                                  nat.ADAM_DENSE)
        if timed is not None:
            ev[timed][0].record()
        nat.check(nat.lib().dcue_adam_step(ctypes_ref(model), ctypes_ref(emb_args), nat.stream_handle()), "adam")
        if timed is not None:
            ev[timed][1].record()
        nat.check(nat.lib().dcue_adam_step(ctypes_ref(model), ctypes_ref(dense_args), nat.stream_handle()), "adam")
        sched.batch_step()

    for s in range(args.warmup):
        step(s, None)
    opt.flush()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(args.warmup + k, k)
    opt.flush()  # deferred user-table steps still pending are part of the timed work
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    rows = world * B * args.steps / dt
    emb_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps
    E = args.user_embdim
    # algorithmic bytes of one user-table Adam sweep: read p, m, v + write p, m, v for every row,
    # the row's slot word, and the batch's compact gradient rows
    emb_bytes = n_users_local * E * 4 * 6 + n_users_local * 4 + B * E * 4
    achieved = emb_bytes / (emb_ms * 1e-3) / 1e9
    traffic = None
    tf_path = os.path.join(ROOT, "profiles", "pmc_adam_embed.json")
    if os.path.exists(tf_path):
        try:
            traffic = json.load(open(tf_path)).get("hbm_bytes_per_launch")
        except (ValueError, OSError):
            traffic = None

    result = {
        "metric": "training triplets/sec (whole node) + AUC@val, DCUE d=128 at 1/2/4/8 MI355X",
        "value": rows * N,
        "unit": "triplets/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "rows_per_s": rows,
        "auc_val": None,
        "config": {"workload": "DCUE truedcuemel1dbn d=%d H=%d E=%d, %d users x %d tracks (fp16 table), "
                               "%d interactions, in-batch negatives N=%d"
                               % (args.feature_dim, args.hidden, E, args.users, args.tracks,
                                  args.interactions, N),
                   "batch_per_gpu": B, "global_batch": B * world, "neg": N,
                   "parallelism": "dp%d (users sharded, dense grads all-reduced)" % world},
        "roofline": {"kernel": "k_adam_embed (user-table Adam sweep)", "bound": "hbm",
                     "achieved": achieved, "peak": 8000.0, "unit": "GB/s", "frac": achieved / 8000.0,
                     "traffic": traffic, "avg_ms": emb_ms, "algorithmic_bytes": emb_bytes},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args, n_users_local)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def ctypes_ref(x):
    import ctypes
    return ctypes.byref(x)


if __name__ == "__main__":
    main()
