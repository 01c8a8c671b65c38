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
    ap.add_argument("--no-eval", action="store_true", help="skip AUC@val after the timed steps")
    ap.add_argument("--eval-pct", type=float, default=0.025, help="users sampled for AUC@val (eval_pct)")
    ap.add_argument("--gpu-only", action="store_true",
                    help="diagnostic: hold the stream behind a sleep kernel while the steps are "
                         "enqueued, then report the GPU's own time for them (no host in the loop)")
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


def song_split(n_tracks):
    """Split code per track (0 train, 1 val, 2 test) by the reference's song split
    (datasets/dcuedataset.py:146-164): two masks drawn right after seeding with 10."""
    rs = np.random.RandomState(10)
    in_train = rs.rand(n_tracks) < 0.80
    rs = np.random.RandomState(10)
    in_val = rs.rand(int(in_train.sum())) < 0.1 / 0.8
    code = np.full(n_tracks, 2, dtype=np.int8)
    train_ids = np.nonzero(in_train)[0]
    code[train_ids] = 0
    code[train_ids[in_val]] = 1
    return code


def evaluate_val(args, net, tracks, pair_user, pair_track, split, n_users, dev):
    """Item factors of every track (eval tower), user factors of every user, then the split-weighted
    AUC / mAP of DCUE.score for an eval_pct sample of the users with train and val interactions."""
    import ctypes
    from dcrecommend import _native as nat
    from dcrecommend.nn import rank
    t0 = time.perf_counter()
    net.sync_user_table()
    net.eval()
    d = args.feature_dim
    n_tracks = tracks.shape[0]
    model = net._model_struct()
    tr = nat.Tracks(tracks.data_ptr(), n_tracks, 0 if tracks.dtype == torch.float16 else 1, 0)
    item_f = torch.empty((n_tracks, d), device=dev)
    step = 8192
    ws = torch.empty(nat.workspace_bytes(net._flat["dims"], step, 0, step), dtype=torch.uint8, device=dev)
    for s in range(0, n_tracks, step):
        n = min(step, n_tracks - s)
        it = torch.arange(s, s + n, dtype=torch.int32, device=dev)
        nat.check(nat.lib().dcue_item_tower_eval(ctypes.byref(model), ctypes.byref(tr), nat.ptr(it), n, nat.ptr(ws),
                                                 ws.numel(), nat.ptr(item_f[s:s + n]), nat.stream_handle()),
                  "dcue_item_tower_eval")
    nat.check(nat.lib().dcue_factor_repeat_mean(nat.ptr(item_f), item_f.numel(), 10, nat.stream_handle()),
              "dcue_factor_repeat_mean")
    torch.cuda.synchronize()
    t_items = time.perf_counter() - t0
    user_f = torch.empty((n_users, d), device=dev)
    for s in range(0, n_users, step):
        n = min(step, n_users - s)
        u = torch.arange(s, s + n, dtype=torch.int64, device=dev)
        nat.check(nat.lib().dcue_user_tower(ctypes.byref(model), nat.ptr(u), n, nat.ptr(ws), ws.numel(),
                                            nat.ptr(user_f[s:s + n]), nat.stream_handle()), "dcue_user_tower")
    torch.cuda.synchronize()
    t_factors = time.perf_counter() - t0
    # all-split interaction CSR over users (duplicate pairs collapse, as the reference's csr_matrix)
    pu, pt = pair_user.cpu().numpy(), pair_track.cpu().numpy()
    key = np.unique(pu * np.int64(n_tracks) + pt)
    u_of, t_of = key // n_tracks, (key % n_tracks).astype(np.int32)
    ptr = np.zeros(n_users + 1, np.int64)
    np.add.at(ptr, u_of + 1, 1)
    ptr = np.cumsum(ptr)
    cls = np.where(split == 1, rank.LIST_PRED, 0).astype(np.uint8) | np.where(split == 0, rank.LIST_TRUTH, 0).astype(np.uint8)
    sp = split[t_of]
    has_train = np.zeros(n_users, bool)
    has_val = np.zeros(n_users, bool)
    has_train[u_of[sp == 0]] = True
    has_val[u_of[sp == 1]] = True
    users = np.nonzero(has_train & has_val)[0]
    sample = np.random.RandomState(0).choice(users, int(len(users) * args.eval_pct))
    t1 = time.perf_counter()
    ev = rank.RankEvaluator({"pos_ptr": ptr, "pos_idx": t_of, "cand_class": cls}, dev)
    auc, ap, ok = ev.metrics(user_f, item_f, sample, nat.RANK_SPLIT)
    t_rank = time.perf_counter() - t1
    net.train()
    H = args.hidden
    # eval item tower FLOPs per track at full conv lengths (23.2 MFLOP at H=d=128)
    flops = 2 * (128 * 4 * H * 132 + H * 4 * H * 34 + H * 4 * H * 9 + H * 2 * H * 3 + H * d + d * d)
    return {"auc": rank.mean_until_missing(auc, ok), "map_val": rank.mean_until_missing(ap, ok),
            "users": int(len(sample)), "candidates": int(n_tracks), "factors_s": t_factors, "rank_s": t_rank,
            "item_tower_s": t_items, "item_tower_tflops": flops * n_tracks / t_items / 1e12,
            "note": "random-init model after the bench steps on synthetic data: AUC ~0.5 is expected"}


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
    # one process per GPU; DCUE_DIST_BACKEND=gloo rehearses the N>1 path with several ranks on one
    # GPU (local ranks wrap over the visible devices), RCCL ("nccl") otherwise
    backend = os.environ.get("DCUE_DIST_BACKEND", "nccl")
    local = local % torch.cuda.device_count() if backend != "nccl" else local
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from dcrecommend import _native as nat
    from dcrecommend import distributed as D
    from dcrecommend.dcue.dcue import DCUENet
    from dcrecommend.optim import NativeAdam
    from dcrecommend.optim.cyclic_scheduler import CyclicLRWithRestarts
    from dcrecommend.dcue.plan import TrainPlan

    B, N = args.batch, args.neg
    # users are sharded across ranks (row u of rank r = global user u*world + r): each rank owns its
    # users' embedding rows + Adam moments; the track table is replicated
    n_users_local = D.local_user_count(args.users, rank, world)
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
    # song split of the reference (datasets/dcuedataset.py:146-164): 80% train of which 1/8 is val,
    # the rest test; training batches draw only train-split interactions, AUC@val ranks val songs
    split = song_split(args.tracks)
    split_d = torch.from_numpy(split).to(dev)
    train_pairs = torch.nonzero(split_d[pair_track] == 0).squeeze(1)
    epoch_size = (int(math.ceil(n_pairs / 10)) // B) * B
    sched = CyclicLRWithRestarts(opt, B, epoch_size=epoch_size, restart_period=30, t_mult=2, policy="cosine")
    sched.step()

    # batch composition (DataLoader shuffle over the interaction rows) is prepared ahead, like the
    # reference's worker processes; the step consumes HBM-resident index vectors
    total = args.warmup + args.steps
    perm = train_pairs[torch.randperm(train_pairs.numel(), generator=gen, device=dev)[: total * B]].view(total, B)
    users_b = pair_user[perm].contiguous()
    items_b = pair_track[perm].to(torch.int32).contiguous()
    mt = torch.empty(nat.MT_STATE_BYTES, dtype=torch.uint8, device=dev)
    nat.check(nat.lib().dcue_mt_seed(nat.ptr(mt), 10 + rank, nat.stream_handle()), "mt_seed")
    G = net._flat["G"]
    G_late = D.late_grad_floats(net)
    TIMED = nat.TIMED_CONV1_WGRAD  # the roofline kernel, timed live by HIP events in the library
    TIMER_STRIDE = 8

    catalogue = args.mode == "catalogue"
    if catalogue:
        # the reference's live sampler (datasets/dcuedataset.py:207-220): N negatives per row drawn
        # from the train split's songs the user never interacted with; the conv runs on all
        # M = B(1+N) distinct items. The user -> split-rank CSR covers every interaction.
        from dcrecommend.datasets.csr import user_split_ranks
        split_items = np.nonzero(split == 0)[0].astype(np.int64)
        indptr, ranks = user_split_ranks(pair_user.cpu().numpy(), pair_track.cpu().numpy(), n_users_local,
                                         split_items)
        split_d64 = torch.from_numpy(split_items).to(dev)
        indptr_d = torch.from_numpy(indptr).to(dev)
        ranks_d = torch.from_numpy(ranks).to(dev)
        items_b64 = items_b.long()
        negs = torch.empty((B, N), dtype=torch.int64, device=dev)

    # The roofline kernel's timer is on before the plan is built. It binds a HIP event pair to every
    # TIMER_STRIDE-th launch of the kernel (its own dispatch's start and end, on the stream it runs
    # on); a timed launch costs the stream a few microseconds, so a sample is timed, not every step.
    nat.timer_enable(TIMED, TIMER_STRIDE)
    plan = TrainPlan(net, tracks, B, N, mt_state=None if catalogue else mt, emb_grad_scale=1.0 / world,
                     optimizer=opt)

    def sample_catalogue(s):
        nat.check(nat.lib().dcue_sample_catalogue(nat.ptr(mt), 0, 0, nat.ptr(split_d64), split_d64.numel(),
                                                  nat.ptr(indptr_d), nat.ptr(ranks_d), nat.ptr(users_b[s]), B, N,
                                                  nat.ptr(negs), nat.stream_handle()), "dcue_sample_catalogue")
        nat.check(nat.lib().dcue_build_catalogue_batch(nat.ptr(items_b64[s]), nat.ptr(negs), B, N,
                                                       nat.ptr(plan.item_track), nat.stream_handle()),
                  "dcue_build_catalogue_batch")

    def step(s):
        if catalogue:
            sample_catalogue(s)
            src = (users_b[s], None)
        else:
            src = (users_b[s], items_b[s])
        if world > 1:
            plan.launch(*src)
            # RCCL: the one exchange of the step (1.57 MB), in two buckets; the larger one overlaps
            # the conv-1 weight gradient
            D.allreduce_mean_overlapped_(plan, G, G_late)
            opt.step()
        else:
            plan.step(*src)  # sample + forward + backward + Adam, one host call
        sched.batch_step()

    for s in range(args.warmup):
        step(s)
    opt.flush()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    nat.timer_read(TIMED)  # drop the warm-up records
    if args.gpu_only:
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(int(2.4e6 * args.steps))  # ~1 ms of GPU per step (2.4 GHz cycles)
        ev0.record()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(args.warmup + k)
    opt.flush()  # deferred user-table steps still pending are part of the timed work
    t_enq = time.perf_counter() - t0  # host time to enqueue the steps (diagnostic)
    if args.gpu_only:
        ev1.record()
    torch.cuda.synchronize()
    if args.gpu_only:
        print(json.dumps({"gpu_only_ms_per_step": ev0.elapsed_time(ev1) / args.steps,
                          "host_enqueue_ms_per_step": t_enq / args.steps * 1e3}))
    nat.timer_enable(TIMED, False)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    dt = D.max_over_ranks(dt, dev)

    rows = world * B * args.steps / dt
    wg_ms, wg_n = nat.timer_read(TIMED)
    wg_ms = wg_ms / max(wg_n, 1)
    # algorithmic FLOPs of one conv-1 weight-gradient launch: dW1[o][c][k] summed over every conv-1
    # output row (item, position) of the batch's distinct items -- B items x 132 positions (131
    # frames, kernel 4, padding 2) x 128 mel inputs x 4 taps x H outputs, 2 FLOP per product
    M_items = B * (1 + N) if catalogue else B
    wg_flops = 2.0 * args.hidden * 128 * 4 * (M_items * 132)
    achieved = wg_flops / (wg_ms * 1e-3) / 1e12
    traffic = None
    tf_path = os.path.join(ROOT, "profiles", "pmc_conv1_wgrad.json")
    if os.path.exists(tf_path) and not catalogue:  # collected on the default (in-batch) workload
        try:
            traffic = json.load(open(tf_path)).get("hbm_bytes_per_launch")
        except (ValueError, OSError):
            traffic = None
    E = args.user_embdim

    result = {
        "metric": "training triplets/sec (whole node) + AUC@val, DCUE d=128 at 1/2/4/8 MI355X",
        "value": rows * N,
        "unit": "triplets/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "host_enqueue_ms_per_step": t_enq / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "rows_per_s": rows,
        "auc_val": None,
        "config": {"workload": "DCUE truedcuemel1dbn d=%d H=%d E=%d, %d users x %d tracks (fp16 table), "
                               "%d interactions, %s negatives N=%d"
                               % (args.feature_dim, args.hidden, E, args.users, args.tracks,
                                  args.interactions, "catalogue" if catalogue else "in-batch", N),
                   "batch_per_gpu": B, "global_batch": B * world, "neg": N,
                   "parallelism": "dp%d (users sharded, dense grads all-reduced)" % world},
        "roofline": {"kernel": "k_conv1_wgrad (conv layer 1 weight gradient, f32 MFMA 32x32x2)", "bound": "mfma",
                     "achieved": achieved, "peak": 157.3, "unit": "TFLOP/s", "frac": achieved / 157.3,
                     "traffic": traffic, "avg_ms": wg_ms, "launches": wg_n, "algorithmic_flops": wg_flops},
    }
    if rank == 0 and not args.no_eval:
        # AUC@val of the trained model (outside the timed region): DCUE.score over an eval_pct
        # sample of this rank's users (nn/dcue.py:380-449, 580-603) on the GPU evaluator
        ev = evaluate_val(args, net, tracks, pair_user, pair_track, split, n_users_local, dev)
        result["auc_val"] = ev.pop("auc")
        result["eval"] = ev
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
