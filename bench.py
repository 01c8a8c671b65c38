#!/usr/bin/env python
"""DCUE training-step throughput on MI355X (BASELINE.json config 2; weak scaling over GPUs).

One step = the reference's per-batch hot loop (nn/dcue.py:202-210) on one batch of synthetic input
already resident in HBM: negative draws (MT19937, bit-exact with numpy) -> forward (item ConvNet,
user tower, cosine scores, hinge loss) -> backward -> [N>1: RCCL all-reduce of the dense gradient,
overlapped with the conv-1 weight gradient] -> Adam over every parameter incl. the whole user table
-> cyclic LR schedule. The whole step, exchange included, is one host call (TrainPlan.step).

Phases, each W untimed warm-up steps then EXACTLY K timed steps between barrier + synchronize:
  1. in-batch negatives, cold user table (a fresh optimizer: most user rows have zero moments);
  2. in-batch negatives after a pass over every local user (steady state: every row's Adam
     moments are live) -- `value` and `ms_per_step`;
  3. catalogue negatives (the reference's live sampler, datasets/dcuedataset.py:207-256: M =
     B(1+N) distinct items per step) -- the `catalogue` object.
Rank 0 prints ONE JSON line.

  python bench.py [--gpus N --steps K --warmup W]
N>1 runs one process per GPU: under torch.distributed.run (RANK/WORLD_SIZE set) or, when started
directly, bench.py launches the N ranks itself before touching any GPU.
"""
import argparse
import gc
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "amplifai-deepcontentrecommenders_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

F32_PEAK_TFLOPS = 157.3   # MI355X dense FP32 (matrix and vector), MI355X_MICROARCH.md
HBM_PEAK_GBS = 8000.0
F16_PEAK_TFLOPS = 2500.0  # MI355X dense FP16/BF16 MFMA (no sparsity), MI355X_MICROARCH.md
# conv forwards run on split-f16 MFMA (three f16 products per f32 product) unless DCUE_CONV_F16=0
CONV_F16 = os.environ.get("DCUE_CONV_F16", "1")[:1] != "0"
WGRAD_F16 = os.environ.get("DCUE_WGRAD_F16", "1")[:1] != "0"
W1K = WGRAD_F16 and os.environ.get("DCUE_W1K", "0")[:1] == "1"  # conv 1: k_conv_wgrad1k (round 6, A/B)



def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--modes", default="inbatch,catalogue,text,dcbr",
                    help="comma list of phases after the cold one: inbatch (warm), catalogue, text "
                         "(config 4's mixed audio + text tower), dcbr (config 5)")
    ap.add_argument("--text-dim", type=int, default=256)
    ap.add_argument("--text-feature-dim", type=int, default=256, help="config 4: d = 256")
    ap.add_argument("--word-dim", type=int, default=300)
    ap.add_argument("--text-len", type=int, default=64)
    ap.add_argument("--spin-sync", type=int, default=1,
                    help="1 (default): poll for the GPU's idle before the pre-timing synchronize, so the "
                         "issuing thread is not asleep in the driver when the timed steps start (its "
                         "wake-up cost the first timed step 0.5-0.9 ms of host time; DESIGN.md §7); "
                         "0: synchronize directly")
    ap.add_argument("--n-words", type=int, default=20000)
    ap.add_argument("--users", type=int, default=100_000)
    ap.add_argument("--tracks", type=int, default=200_000)
    ap.add_argument("--interactions", type=int, default=5_000_000)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--neg", type=int, default=20)
    ap.add_argument("--feature-dim", type=int, default=128)
    ap.add_argument("--hidden", type=int, default=128)
    ap.add_argument("--user-embdim", type=int, default=300)
    ap.add_argument("--cpu-steps", type=int, default=10)
    ap.add_argument("--dense-embedding-adam", action="store_true",
                    help="step every user row every step (the literal sweep) instead of the deferred, "
                         "bit-identical replay")
    ap.add_argument("--flush-every", type=int, default=12,
                    help="deferred user-table Adam: rolling-flush cadence (NativeAdam flush_every). A "
                         "batch's user rows are at most this many steps behind, so their replay inside "
                         "the step is short; the rolling slices' total work does not depend on it "
                         "(A/B: 64 -> 12 is 0.261 -> 0.232 ms/step at 100 steps, profiles/r04_ab_flush_every.txt)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-eval", action="store_true", help="skip AUC@val after the timed steps")
    ap.add_argument("--no-f32-probe", action="store_true",
                    help="skip the exact-f32 comparison run (DCUE_CONV_F16=0 DCUE_WGRAD_F16=0 "
                         "DCUE_DGRAD_F16=0, in-batch + catalogue, in a child process)")
    ap.add_argument("--eval-pct", type=float, default=0.025, help="users sampled for AUC@val (eval_pct)")
    ap.add_argument("--timer-stride", type=int, default=8,
                    help="time every n-th launch of the roofline kernels live (HIP events)")
    ap.add_argument("--gc-mode", choices=["on", "off"], default="on",
                    help="diagnostic: off = gc.collect() then gc.disable() around each phase's timed steps")
    ap.add_argument("--host-trace", action="store_true",
                    help="diagnostic: report each timed step's host issue time (host_issue_us per phase)")
    ap.add_argument("--gpu-only", action="store_true",
                    help="diagnostic: hold the stream behind a sleep kernel while the warm in-batch "
                         "steps are enqueued, then report the GPU's own time for them")
    ap.add_argument("--profile-phase", choices=["inbatch_cold", "inbatch", "catalogue", "text"],
                    help="under `rocprofv3 --kernel-trace`: bracket this phase's timed steps with a "
                         "marker kernel (profiles/summarize_pmc.py keeps what lies between)")
    ap.add_argument("--sync-bn", action="store_true",
                    help="N > 1 with the native exchange: SyncBN over the ranks (dcue_plan_set_sync_bn); "
                         "default per-replica BatchNorm (DDP semantics)")
    ap.add_argument("--py-exchange", action="store_true",
                    help="N>1: all-reduce from Python over torch.distributed instead of the plan's RCCL")
    ap.add_argument("--stall-s", type=float, default=180.0,
                    help="N>1: a rank that makes no progress for this long reports where and exits 3")
    ap.add_argument("--deadline-s", type=float, default=1500.0,
                    help="bench.py --gpus N started directly: end every rank after this long")
    return ap.parse_args()


# ----------------------------------------------------------------------------------- launching
def spawn_ranks(n, deadline_s):
    """`bench.py --gpus N` started directly: one child process per GPU with the torch.distributed
    env (rendezvous on 127.0.0.1), before this process touches a GPU; rank 0 prints the line. The
    children are polled, never waited on blindly: one failing rank ends the others (they would wait
    in a collective forever), and past `deadline_s` every rank is ended with a message."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    t0 = time.monotonic()
    try:
        while any(p.poll() is None for p in procs):
            failed = [(i, p.returncode) for i, p in enumerate(procs) if p.returncode]
            if failed or time.monotonic() - t0 > deadline_s:
                why = ("rank %d exited with %d" % failed[0]) if failed else "deadline of %.0f s passed" % deadline_s
                print("bench.py: %s; ending the other ranks" % why, file=sys.stderr, flush=True)
                rc = failed[0][1] if failed else 124
                for q in procs:
                    if q.poll() is None:
                        q.terminate()
                t1 = time.monotonic()
                while any(q.poll() is None for q in procs) and time.monotonic() - t1 < 20:
                    time.sleep(0.2)
                break
            time.sleep(0.2)
        rc = rc or next((p.returncode for p in procs if p.returncode), 0)
    finally:
        for q in procs:
            if q.poll() is None:
                q.kill()
    return rc


class Watchdog:
    """Per-rank deadline on progress. The ranks meet in RCCL collectives (the plan's gradient
    exchange, two buckets per step, and the barriers around each timed phase); a rank stuck there
    never returns to Python. Every step reports its position here; if none arrives for `limit_s`,
    the watchdog thread prints where the rank stopped -- phase, step, and which collective was
    pending -- and ends the process with status 3 (no re-exec; the parent or torchrun sees it)."""

    def __init__(self, rank, limit_s):
        import threading
        self.rank, self.limit = rank, limit_s
        self.where = "start-up"
        self.t = time.monotonic()
        self.lock = threading.Lock()
        th = threading.Thread(target=self._run, daemon=True)
        th.start()

    def mark(self, where):
        with self.lock:
            self.where, self.t = where, time.monotonic()

    def _run(self):
        while True:
            time.sleep(1.0)
            with self.lock:
                idle, where = time.monotonic() - self.t, self.where
            if idle > self.limit:
                print("bench.py rank %d: no progress for %.0f s; last position: %s" % (self.rank, idle, where),
                      file=sys.stderr, flush=True)
                os._exit(3)


# ------------------------------------------------------------------------------ synthetic data
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


def item_flops(H, d):
    """Forward FLOPs of the item tower per spectrogram at full conv lengths (23.2 MFLOP at H=d=128)."""
    return 2 * (128 * 4 * H * 132 + H * 4 * H * 34 + H * 4 * H * 9 + H * 2 * H * 3 + H * d + d * d)


def text_conv_flops(T, E, C):
    """Forward FLOPs of the text conv per item: T positions x (3 taps x E) x C."""
    return 2.0 * T * 3 * E * C


def synthetic_sentences(n, T, n_words, device, seed, pad=0, bos=1, eos=2):
    """[n][T] int32 token rows in the reference's shape (datasets/dcuelmitemset.py:40-56): BOS, a
    sentence of 1..T-2 random word ids (>= 3), EOS, then PAD."""
    gen = torch.Generator(device=device).manual_seed(seed)
    lens = torch.randint(1, T - 1, (n, 1), generator=gen, device=device)
    pos = torch.arange(T, device=device).unsqueeze(0)
    words = torch.randint(3, n_words, (n, T), generator=gen, device=device, dtype=torch.int32)
    tok = torch.where(pos <= lens, words, torch.full_like(words, pad))
    tok[:, 0] = bos
    tok.scatter_(1, lens + 1, eos)
    return tok.to(torch.int32).contiguous()


DGRAD_F16 = os.environ.get("DCUE_DGRAD_F16", "1")[:1] != "0"


def fail_flag_failures(flags):
    """The library's device fail word (dcue_debug_fail_flags) as checks.failed entries: bit 0 is a
    bounded wait in the fused user-tower forward that gave up (adam.hip k_user_fwd) -- its rows may
    then have been read before their Adam replay; bit 1 a plan's device-side cross-stream wait that
    gave up (dcue_common.h DevWait) -- its kernel then read a producer's data early. Either fails the
    run, whatever its throughput."""
    out = []
    if flags & 1:
        out.append("fail flags: the fused user-tower forward's bounded wait for a claimed row gave up (bit 0)")
    if flags & 2:
        out.append("fail flags: a plan's device-side cross-stream wait (DevWait) gave up (bit 1)")
    if flags & ~3:
        out.append("fail flags: unknown bits 0x%x" % (flags & ~3))
    return out


def executed_work(args, items_per_row, M):
    """The FLOPs one row's step actually executes and their time at the ceiling of the arithmetic
    that runs them: forwards on split-f16 MFMA (3 f16 products per f32 product: 2500/3
    TFLOP/s f32-equivalent), the conv-1 weight gradient on the raw fp16 table (2 products: 2500/2),
    the other weight gradients split-f16 (2500/3), input gradients of layers 5..2 split-f16 where a
    launch writes >= 8,192 rows (catalogue layers 2-3) and f32 MFMA (157.3) otherwise, the user tower
    f32 MFMA; conv 1's input gradient is never computed (§4.2). Returns (flops, seconds) per row."""
    H, d, E = args.hidden, args.feature_dim, args.user_embdim
    lp_in = {2: 33, 3: 8, 4: 2, 5: 1}  # rows of g_{l-1} written by layer l's dgrad, per item
    f = {1: 2 * 128 * 4 * H * 132, 2: 2 * H * 4 * H * 34, 3: 2 * H * 4 * H * 9, 4: 2 * H * 2 * H * 3,
         5: 2 * H * d, "fc": 2 * d * d}
    fwd_peak = F16_PEAK_TFLOPS / 3 if CONV_F16 else F32_PEAK_TFLOPS
    w16 = F16_PEAK_TFLOPS / 3 if WGRAD_F16 else F32_PEAK_TFLOPS
    w1 = F16_PEAK_TFLOPS / 2 if WGRAD_F16 else F32_PEAK_TFLOPS
    flops = t = 0.0
    for k, v in f.items():
        flops += v
        t += v / (fwd_peak * 1e12)                                   # forward
        flops += v
        t += v / ((w1 if k == 1 else w16) * 1e12)                    # weight gradient
        if k != 1:                                                   # input gradient (none for conv 1)
            split = DGRAD_F16 and k in lp_in and M * lp_in[k] >= 8192
            flops += v
            t += v / ((F16_PEAK_TFLOPS / 3 if split else F32_PEAK_TFLOPS) * 1e12)
    flops *= items_per_row
    t *= items_per_row
    u = 3 * 2 * (E * E + E * d)
    return flops + u, t + u / (F32_PEAK_TFLOPS * 1e12)


def row_flops(args, items_per_row):
    """SURVEY §8(d) canonical work per row: 3 x forward (fwd + bwd) of the item tower over the
    row's items plus the user tower (1.462 GFLOP catalogue, 70.4 MFLOP compact in-batch)."""
    E, d = args.user_embdim, args.feature_dim
    return 3 * item_flops(args.hidden, d) * items_per_row + 3 * 2 * (E * E + E * d)


F64_PEAK_TFLOPS = 78.6  # MI355X fp64 vector and matrix (AMD spec: the two are equal on MI355X)


def wrmf_half_step_flops(indptr, d, n_fixed):
    """Algorithmic fp64 FLOPs of one WRMF half-step: the Gram matrix F^T F (lower
    triangle, n_fixed rows), and per row with pairs its rank-1 terms (nnz x (d(d+1)/2 + d) FMAs),
    the Cholesky (d^3/6) and the two triangular solves (d^2)."""
    nnz = (indptr[1:] - indptr[:-1]).double()
    rows = float((nnz > 0).sum())
    fma = float(nnz.sum()) * (d * (d + 1) / 2 + d) + rows * (d ** 3 / 6 + d * d) + n_fixed * d * (d + 1) / 2
    return 2.0 * fma


def wrmf_half_step_flops_executed(indptr, d, n_fixed, woodbury_max=32):
    """fp64 FLOPs one default WRMF half-step executes, each row counted by the path
    that solves it: the Gram matrix (n_fixed x d(d+1)/2 FMAs); M = (G + lambda I)^-1 by Gauss-Jordan
    (d^3); a row with 1..32 pairs by the Woodbury identity (k_wrmf_solve_lowrank: P = F_r M n d^2,
    S = P F_r^T n^2 d, b / P b / x 3 n d, the n x (n + 1) elimination n^2 (n + 1)); a row with more by
    the block Cholesky (k_wrmf_solve_mfma: n (d(d+1)/2 + d) + d^3/6 + d^2)."""
    nnz = (indptr[1:] - indptr[:-1]).double()
    low = (nnz > 0) & (nnz <= woodbury_max)
    high = nnz > woodbury_max
    nl = nnz[low]
    fma = float((nl * d * d + nl * nl * d + 3 * nl * d + nl * nl * (nl + 1)).sum())
    nh = nnz[high]
    fma += float(nh.sum()) * (d * (d + 1) / 2 + d) + float(high.sum()) * (d ** 3 / 6 + d * d)
    fma += n_fixed * d * (d + 1) / 2 + float(d) ** 3
    return 2.0 * fma


# --------------------------------------------------------------------------------- evaluation
def dcbr_phase(args, tracks, pair_user, pair_track, n_users, dev, M, comm=None, world=1, rank=0):
    """BASELINE config 5 at this run's shape (no reference numbers exist: dcrecommend/dcbr is
    unpublished): WRMF (factors = d, alpha 40, lambda 0.1) on the interactions -- one untimed
    iteration, then two timed ALS iterations (users, then items) -- and the DCBR regression of the
    item tower onto those factors, `warmup` + `steps` Adam steps over random M-item batches per
    rank. N > 1 (comm: the library's communicator): every rank holds the same interactions, each
    half-step solves 1/N of the rows and all-gathers them, and the regression averages its dense
    gradient over the ranks before Adam (DDP) -- whole-job rates, the slowest rank's time."""
    from dcrecommend import distributed as D
    from dcrecommend.dcbr import DCBR, WRMF
    d = args.feature_dim
    w = WRMF(factors=d, regularization=0.1, alpha=40.0, iterations=1, seed=0, device=dev, comm=comm)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    w.fit(pair_user, pair_track, None, n_users=n_users, n_items=args.tracks)
    torch.cuda.synchronize()
    t_fit1 = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(2):
        w.half_step(w.user_factors, w.item_factors, w.by_user)
        w.half_step(w.item_factors, w.user_factors, w.by_item)
    torch.cuda.synchronize()
    t_iter = D.max_over_ranks((time.perf_counter() - t0) / 2, dev)
    gen = torch.Generator(device="cpu").manual_seed(17 + rank)
    n = args.warmup + args.steps
    items = torch.randint(0, args.tracks, (n, M), generator=gen, dtype=torch.int32).to(dev)
    torch.manual_seed(3)  # the same ConvNet on every rank
    model = DCBR(feature_dim=d, conv_hidden=args.hidden, lr=1e-4, device=dev, comm=comm)
    targets = w.item_factors
    losses = []
    for s in range(args.warmup):
        losses.append(model.step(tracks, items[s], targets[items[s].long()]))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for s in range(args.warmup, n):
        losses.append(model.step(tracks, items[s], targets[items[s].long()]))
    torch.cuda.synchronize()
    dt = D.max_over_ranks(time.perf_counter() - t0, dev)
    same, _, _ = D.replica_checksums(model.net._flat["P"])
    finite = bool(torch.isfinite(model.net._flat["P"]).all()) and all(
        bool(torch.isfinite(torch.as_tensor(l)).all()) for l in losses) and bool(
        torch.isfinite(w.user_factors).all()) and bool(torch.isfinite(w.item_factors).all())
    nnz = int(pair_user.shape[0])
    # rooflines: the ALS iteration against the fp64 vector peak (its solve is fp64 VALU work); the
    # regression step against the ceiling of the arithmetic its kernels run (executed_work, per item,
    # the user tower left out)
    f_chol = (wrmf_half_step_flops(w.by_user[0], d, args.tracks) +
              wrmf_half_step_flops(w.by_item[0], d, n_users))
    tile = os.environ.get("DCUE_WRMF_SOLVE", "")[:1] == "t"
    woodbury = not tile and os.environ.get("DCUE_WRMF_LOWRANK", "1")[:1] != "0"
    # `achieved` / `frac`: the FLOPs the kernels execute, each row by its own path (Woodbury rows
    # never form or factor the d x d system); the Cholesky formulation's count for every row, divided
    # by the same time, is kept beside it as an effective rate
    f_iter = (wrmf_half_step_flops_executed(w.by_user[0], d, args.tracks) +
              wrmf_half_step_flops_executed(w.by_item[0], d, n_users)) if woodbury else f_chol
    ach = f_iter / t_iter / 1e12
    wroof = {"kernel": "dcue_wrmf_half_step x 2 (k_wrmf_gram_mfma + %s)" % (
                 "k_wrmf_solve: fp64 register-tile Cholesky" if tile else
                 "k_wrmf_solve_lowrank: Woodbury identity for rows with <= 32 pairs, k_wrmf_solve_mfma: "
                 "fp64-MFMA block Cholesky for the rest; v_mfma_f64_16x16x4_f64"),
             "bound": "valu (fp64)" if tile else "mfma (fp64; MI355X's fp64 matrix and vector peaks are equal)",
             "achieved": ach, "peak": F64_PEAK_TFLOPS, "unit": "TFLOP/s (fp64)",
             "frac": ach / F64_PEAK_TFLOPS, "algorithmic_flops": f_iter,
             "flops_counted": "executed per path (Woodbury rows: n d^2 + n^2 d + n^3; Cholesky rows)"
                              if woodbury else "Cholesky formulation (every row)",
             "effective_tflops_cholesky_formulation": f_chol / t_iter / 1e12, "traffic": None}
    pmc = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "pmc_wrmf_solve.json")
    if os.path.exists(pmc):
        with open(pmc) as fh:
            wroof["traffic_per_solve_launch"] = json.load(fh).get("hbm_bytes")
    ex_f, ex_t = executed_work(args, 1, M)
    u = 3 * 2 * (args.user_embdim ** 2 + args.user_embdim * d)
    ex_f, ex_t = ex_f - u, ex_t - u / (F32_PEAK_TFLOPS * 1e12)
    r_ach = world * M * args.steps * ex_f / dt / 1e12
    rroof = {"kernel": "DCBR regression step (item-tower train forward + MSE head + item-only backward)",
             "bound": "mfma", "achieved": r_ach, "peak": ex_f / ex_t / 1e12,
             "unit": "TFLOP/s (f32-equivalent, executed work; peak = the blended ceiling of its kernels)",
             "frac": r_ach / (ex_f / ex_t / 1e12), "flops_per_item": ex_f}
    return {"workload": "WRMF d=%d over %d users x %d tracks, %d interactions; DCBR regression of the "
                        "truedcuemel1dbn item tower (H=%d) onto the item factors, %d-item batches per GPU, %d GPU(s)"
                        % (d, n_users, args.tracks, nnz, args.hidden, M, world),
            "wrmf_ms_per_iteration": t_iter * 1e3, "wrmf_rows_per_s": (n_users + args.tracks) / t_iter,
            "wrmf_first_iteration_ms_incl_csr_build": t_fit1 * 1e3,
            "regression_ms_per_step": dt / args.steps * 1e3, "regression_items_per_s": world * M * args.steps / dt,
            "wrmf_roofline": wroof, "regression_roofline": rroof,
            "loss_first": float(losses[0]), "loss_last": float(losses[-1]), "replicas_identical": same,
            "finite": finite,
            "parity": "unpinned against the reference (never published); pinned against oracle/wrmf_oracle.py "
                      "and the fp64 oracle item tower (tests/test_gpu_dcbr.py); N>1 bit-exact with one rank "
                      "(WRMF) and with an explicit all-reduce (regression), tests/test_gpu_dcbr_dp.py"}


def evaluate_val(args, net, tracks, pair_user, pair_track, split, n_users, dev):
    """Item factors of every track (eval tower), user factors of every user, then the split-weighted
    AUC / mAP of DCUE.score for an eval_pct sample of the users with train and val interactions."""
    import ctypes
    from dcrecommend import _native as nat
    from dcrecommend.nn import rank
    t0 = time.perf_counter()
    net.sync_user_table()
    net.eval()
    d = nat.storage_dims(net._flat["dims"]).feature_dim  # factor rows at the storage width (zero past d)
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
    ptr[1:] = np.cumsum(np.bincount(u_of, minlength=n_users))
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
    flops = item_flops(args.hidden, d)
    return {"auc": rank.mean_until_missing(auc, ok), "map_val": rank.mean_until_missing(ap, ok),
            "users": int(len(sample)), "candidates": int(n_tracks), "factors_s": t_factors, "rank_s": t_rank,
            "item_tower_s": t_items, "item_tower_tflops": flops * n_tracks / t_items / 1e12,
            "note": "random-init model after the bench steps on synthetic data: AUC ~0.5 is expected"}


def exact_f32_probe(args):
    """What the split-f16 emulation buys: the same in-batch and catalogue steps with every conv on
    exact f32 MFMA (DCUE_CONV_F16=0 DCUE_WGRAD_F16=0 DCUE_DGRAD_F16=0; the library reads them at load,
    so in a child process, after this one's timed phases)."""
    env = dict(os.environ, DCUE_CONV_F16="0", DCUE_WGRAD_F16="0", DCUE_DGRAD_F16="0")
    cmd = [sys.executable, os.path.abspath(__file__), "--modes", "inbatch,catalogue", "--no-eval",
           "--no-cpu-baseline", "--no-f32-probe", "--steps", str(args.steps), "--warmup", str(args.warmup),
           "--users", str(args.users), "--tracks", str(args.tracks), "--interactions", str(args.interactions)]
    try:
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
        d = json.loads(line)
        return {"ms_per_step": d["ms_per_step"], "catalogue_ms_per_step": d.get("catalogue", {}).get("ms_per_step"),
                "inbatch_cold_ms_per_step": d["inbatch_cold"]["ms_per_step"],
                "env": "DCUE_CONV_F16=0 DCUE_WGRAD_F16=0 DCUE_DGRAD_F16=0 (every conv on f32 MFMA 16x16x4 / 32x32x2)"}
    except (subprocess.SubprocessError, IndexError, ValueError, KeyError) as e:
        return {"error": "%s: %s" % (type(e).__name__, str(e)[:200])}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(args, n_users_local):
    """The oracle (torch-CPU restatement of the reference step, pinned to the reference's golden
    vectors) on the host cores: warm-up 2 steps, then the median of --cpu-steps steps (SURVEY
    §8(d)). Like the reference, it runs the item tower over the literal [pos; neg] stack of
    B(1+N) spectrograms, in-batch negatives being copies of positives (nn/dcue.py:698-709) --
    the GPU's compact in-batch layout runs the tower once per distinct item (B = 64), so part of
    the in-batch GPU/CPU ratio is that 21x reuse; catalogue mode does the same work on both."""
    from oracle import dcue_oracle as O
    affinity = len(os.sched_getaffinity(0))
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or affinity
    threads = max(1, min(threads, affinity))
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    B, N = args.batch, args.neg
    p, b = O.init_params(args.feature_dim, args.hidden, args.user_embdim, n_users_local)
    adam = O.AdamState(p)
    rs = np.random.RandomState(0)
    gen = torch.Generator().manual_seed(1)
    times = []
    for s in range(args.cpu_steps + 2):
        u = torch.randint(0, n_users_local, (B,), generator=gen)
        pos = torch.randn(B, 128, 131, generator=gen).half().float()
        r = torch.from_numpy(O.inbatch_negatives(rs, B, N))
        neg = pos[r.reshape(-1)].reshape(B, N, 128, 131)
        t0 = time.perf_counter()
        O.train_step(p, b, adam, u, pos, neg, 1e-5)
        times.append(time.perf_counter() - t0)
    med = float(np.median(times[2:]))
    rows = B / med
    return {"value": rows * N, "unit": "triplets/s", "rows_per_s": rows, "cores": threads, "kind": "port",
            "host_cpus_visible": affinity, "cpu_model": cpu_model(),
            "sample": "median of %d oracle train steps (after 2 warm-up) at B=%d, N=%d, d=%d, H=%d, %d users, "
                      "torch-CPU fp32 on %d threads; the reference-literal %d-item [pos; neg] stack per step "
                      "(the GPU's in-batch step runs the compact %d-item tower)"
                      % (args.cpu_steps, B, N, args.feature_dim, args.hidden, n_users_local, threads, B * (1 + N), B),
            "ms_per_step_median": med * 1e3}


# ---------------------------------------------------------------------------------------- main
def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus, args.deadline_s))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; DCUE_DIST_BACKEND=gloo rehearses the N>1 path with several ranks on one
    # GPU (local ranks wrap over the visible devices; the exchange then runs from Python)
    backend = os.environ.get("DCUE_DIST_BACKEND", "nccl")
    local = local % torch.cuda.device_count() if backend != "nccl" else local
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    wd = Watchdog(rank, args.stall_s) if world > 1 else None

    def mark(where):
        if wd is not None:
            wd.mark(where)

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
    modes = [m for m in args.modes.split(",") if m]
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

    def sched_step():
        try:
            sched.batch_step()
        except StopIteration:  # the sub-epoch's batch count is spent: the trainer's next sched.step()
            sched.step()
            sched.batch_step()

    # batch composition (DataLoader shuffle over the interaction rows) is prepared ahead, like the
    # reference's worker processes; every step consumes HBM-resident index vectors
    def batches(n_steps):
        perm = train_pairs[torch.randint(0, train_pairs.numel(), (n_steps * B,), generator=gen, device=dev)]
        return pair_user[perm].view(n_steps, B).contiguous(), pair_track[perm].to(torch.int32).view(n_steps, B).contiguous()

    # one pass over every local user with a train interaction (the steady state's precondition)
    u_t = pair_user[train_pairs]
    order = torch.argsort(u_t, stable=True)
    first = torch.ones_like(order, dtype=torch.bool)
    first[1:] = u_t[order][1:] != u_t[order][:-1]
    cover = train_pairs[order[first]]
    cover = cover[torch.randperm(cover.numel(), generator=gen, device=dev)]
    n_cover = cover.numel() // B * B
    warm_users = pair_user[cover[:n_cover]].view(-1, B).contiguous()
    warm_items = pair_track[cover[:n_cover]].to(torch.int32).view(-1, B).contiguous()

    mt = torch.empty(nat.MT_STATE_BYTES, dtype=torch.uint8, device=dev)
    nat.check(nat.lib().dcue_mt_seed(nat.ptr(mt), 10 + rank, nat.stream_handle()), "mt_seed")
    G = net._flat["G"]
    G_late = D.late_grad_floats(net)
    native_exchange = world > 1 and backend == "nccl" and not args.py_exchange
    comm, comm_error = None, None
    if native_exchange:
        try:
            comm = D.NativeComm()
        except RuntimeError as e:  # reported in the line; the step then all-reduces from Python
            comm_error = str(e)

    timed = [nat.TIMED_CONV1_WGRAD, nat.TIMED_CONV1_FWD, nat.TIMED_EMB_SLICE, nat.TIMED_EMB_FLUSH,
             nat.TIMED_ALLREDUCE, nat.TIMED_TEXT_FWD, nat.TIMED_USER_FWD, nat.TIMED_TEXT_WGRAD]
    # every stride-th launch of each class is timed live (a timed launch costs its stream a few us)
    stride = max(1, min(args.timer_stride, args.steps // 4))
    if args.timer_stride <= 0:  # (diagnostic: no live kernel timing at all)
        timed = []

    def make_plan(catalogue):
        plan = TrainPlan(net, tracks, B, N, mt_state=None if catalogue else mt, emb_grad_scale=1.0 / world,
                         optimizer=opt)
        if comm is not None:
            plan.set_comm(comm)
            if args.sync_bn:
                plan.set_sync_bn(True)
        return plan

    def run(plan, step_fn, n, phase="warm-up", stamps=None):
        for s in range(n):
            # a step's exchange is issued inside plan.step; a rank stuck in it stops here or in the
            # synchronize after the loop, with that step's two buckets (bn0/conv1/bn1 and the rest)
            # pending on the communicator's stream
            if wd is not None:
                mark("%s step %d/%d issued (its RCCL buckets: late segments then bn0/conv-1/bn1)" % (phase, s + 1, n))
            step_fn(plan, s)
            if stamps is not None:
                stamps.append(time.perf_counter())

    def inbatch_step(users_b, items_b):
        # per-step batch views made once, outside the timed region (the batch composition is prepared
        # ahead, as the reference's DataLoader workers do): a step issues no tensor indexing
        users_b, items_b = list(users_b.unbind(0)), list(items_b.unbind(0))
        n_b = len(users_b)

        def fn(plan, s):
            if world > 1 and comm is None:
                plan.launch(users_b[s], items_b[s])
                D.allreduce_mean_overlapped_(plan, G, G_late)
                opt.step()
            else:
                if s + 1 < n_b:  # the next batch is known: its bn0 inputs ride beside this step
                    plan.set_next(items_b[s + 1])
                plan.step(users_b[s], items_b[s])  # sample + fwd + bwd (+ RCCL) + Adam: one host call
            sched_step()
        return fn

    def profile_mark():
        """--profile-phase: a short sleep kernel (torch's spin_kernel) that brackets the phase's
        timed steps in a rocprofv3 kernel trace; profiles/summarize_pmc.py keeps the dispatches
        between the two marks."""
        torch.cuda.synchronize()
        torch.cuda._sleep(1000)
        torch.cuda.synchronize()

    launches = {}  # kernel launches per timed step, per phase (libdcue_hip's own count)
    host_trace = {}  # --host-trace: per-step host issue times, per phase

    def timed_phase(name, plan, step_fn, gpu_only=False, optim=None):
        """W warm-up steps, then EXACTLY K timed steps between barrier + synchronize on both
        sides; max over ranks. Returns (seconds, host enqueue seconds, gpu-only ms or None)."""
        optim = opt if optim is None else optim
        run(plan, step_fn, args.warmup, name + " warm-up")
        optim.flush()
        if args.gc_mode == "off":  # (A/B: Python's cyclic collector held off over the timed steps)
            gc.collect()
            gc.disable()
        mark(name + ": barrier before the timed steps")
        if world > 1:
            dist.barrier()
        # (outside the timed region) wait for the GPU by polling, so the host thread stays awake on its
        # core, then synchronize: a thread put to sleep in the driver's wait issued the first timed step
        # 2-4x slower (profiles/r06_ab_spin_sync.txt)
        if args.spin_sync:
            done = torch.cuda.Event()
            done.record()
            while not done.query():
                pass
        torch.cuda.synchronize()
        for k in timed:
            nat.timer_enable(k, stride)  # from the first timed step on (restarts the stride count)
        profiled = args.profile_phase == name
        if profiled:
            profile_mark()
        ev0 = ev1 = None
        if gpu_only:
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(int(2.4e6 * args.steps))  # ~1 ms of GPU per step (2.4 GHz cycles)
            ev0.record()
        l0 = nat.lib().dcue_launch_count()
        t0 = time.perf_counter()
        stamps = [] if args.host_trace else None
        run(plan, lambda p, s: step_fn(p, args.warmup + s), args.steps, name + " timed", stamps)
        if stamps is not None:  # --host-trace: each timed step's host issue time (us)
            host_trace[name] = [round((b - a) * 1e6, 1) for a, b in zip([t0] + stamps[:-1], stamps)]
        optim.flush()  # deferred user-table steps still pending are part of the timed work
        t_enq = time.perf_counter() - t0
        if args.gc_mode == "off":
            gc.enable()
        launches[name] = (nat.lib().dcue_launch_count() - l0) / args.steps
        if gpu_only:
            ev1.record()
        mark(name + ": synchronize after the timed steps (every issued step's exchange pending)")
        torch.cuda.synchronize()
        if profiled:
            profile_mark()
        mark(name + ": barrier after the timed steps")
        if world > 1:
            dist.barrier()
        dt = D.max_over_ranks(time.perf_counter() - t0, dev)
        kern = {k: nat.timer_samples(k) for k in timed}
        for k in timed:
            nat.timer_enable(k, False)
        return dt, t_enq, (ev0.elapsed_time(ev1) / args.steps if gpu_only else None), kern

    frozen_frac = [None]

    def replay_bytes(optim):
        """Bytes the user-table replay moves over the whole table (k_emb_flush; adam.hip): m and v
        read for every element, p read and m, v written for the float4 groups whose moments are not
        the idle (+0, +0) fixed point (the replay skips those), the row clocks read. p's store
        (only where the replay changed it) is left out: a lower bound, so the fraction stays
        physical. Counted after the phase's final flush (an idle group stays idle)."""
        st = optim._adam_state()
        em, ev = st["em"], st["ev"]
        if st.get("emb_step") is not None:  # frozen rows (csrc/adam_replay.h): clock bit 30
            frozen_frac[0] = float(((st["emb_step"] & 0x40000000) != 0).float().mean())
        n = em.numel()
        if n % 4:
            act = int(((em.view(torch.int32) | ev.view(torch.int32)) != 0).sum())
        else:
            act = 4 * int((((em.view(torch.int32) | ev.view(torch.int32)) != 0).view(-1, 4).any(1)).sum())
        return 8.0 * n + 12.0 * act + 4.0 * em.shape[0], act / max(n, 1)

    def kernel_rooflines(kern, M, steps, optim=None, d=None):
        """Live HIP-event timing of the candidate kernels: per launch and per step, with each
        one's algorithmic work against its roofline."""
        H, E = args.hidden, args.user_embdim
        d = args.feature_dim if d is None else d
        Tt, Ew, Ct = args.text_len, args.word_dim, args.text_dim
        conv1 = 2.0 * H * 128 * 4 * (M * 132)
        rows_slice = n_users_local / args.flush_every
        table_bytes, active = replay_bytes(opt if optim is None else optim)
        spec = {
            nat.TIMED_CONV1_WGRAD: (("k_conv_wgrad1k (conv-1 weight gradient, one tap per workgroup: 32 o x 128 c "
                                     "tiles, split-K over 64-row stages, split-f16 MFMA 16x16x32 on the raw fp16 "
                                     "table: two f16 products per f32 product, dz hi+lo x exact x; peak = f16 dense "
                                     "peak / 2)") if W1K else
                                    ("k_conv_wgrad16 layer 1 (conv-1 weight gradient, split-f16 MFMA 16x16x32 on "
                                     "the raw fp16 table: two f16 products per f32 product, dz hi+lo x exact x; "
                                     "peak = f16 dense peak / 2)") if WGRAD_F16 else
                                    "k_conv1_wgrad (conv-1 weight gradient, f32 MFMA 32x32x2)", "mfma", conv1),
            nat.TIMED_CONV1_FWD: (("k_conv_rows<0,0> layer 1 (conv-1 forward + pool + BN partials, split-f16 "
                                   "MFMA 16x16x32: three f16 products per f32 product; peak = f16 dense peak / 3)")
                                  if CONV_F16 else
                                  "k_conv_rows<0,0> layer 1 (conv-1 forward + pool + BN partials, f32 MFMA)",
                                  "mfma", conv1),
            nat.TIMED_EMB_SLICE: ("k_emb_flush_rows (deferred user-table Adam, one rolling slice; user "
                                  "stream, beside the item tower: its duration includes waiting behind the "
                                  "priority-2 critical-path kernels; bytes: the table's at its active fraction)",
                                  "valu", table_bytes * rows_slice / max(n_users_local, 1)),
            nat.TIMED_EMB_FLUSH: ("k_emb_flush (deferred user-table Adam, full-table flush at the phase end, "
                                  "alone on its stream: the replay's uncontended per-element rate)", "valu",
                                  table_bytes),
            nat.TIMED_ALLREDUCE: ("RCCL all-reduce of the dense gradient (per bucket)", "xgmi", None),
            nat.TIMED_TEXT_FWD: ("k_text_fwd (config 4 text conv: word-vector gather + Conv1d(%d -> %d, k 3) "
                                 "over %d positions + masked max, split-f16 MFMA 16x16x32: three f16 products "
                                 "per f32 product; peak = f16 dense peak / 3)"
                                 % (args.word_dim, args.text_dim, args.text_len), "mfma",
                                 M * text_conv_flops(args.text_len, args.word_dim, args.text_dim)),
            # user stream, beside the item tower (the score kernel waits for it): B rows x (E x E + E x d)
            # MACs on f32 MFMA (k_tgemm's 16x16x4 blocks), plus the batch rows' deferred Adam replay
            nat.TIMED_USER_FWD: ("k_user_fwd (fused user-tower forward: the batch rows' deferred Adam replay, "
                                 "then Linear(%d,%d)+ReLU+Linear(%d,%d) on f32 MFMA; user stream)" % (E, E, E, d),
                                 "mfma", B * 2.0 * (E * E + E * d)),
            # wgrad stream 1: dW[o][c][k] = sum_i g[i][o] e[i][t*(i,o)+k-1][c], exact f32 FMAs (VALU);
            # bytes: the batch's sentences' word rows, tokens, g and argmax codes read once, dW + db written
            nat.TIMED_TEXT_WGRAD: ("k_text_wgrad (config 4 text conv weight gradient: max-routed gather of "
                                   "word rows x dL/ds, f32 FMAs; wgrad stream 1)", "valu",
                                   M * (Tt * Ew * 4.0 + Tt * 4.0 + Ct * 5.0) + Ct * Ew * 3 * 4.0 + Ct * 4.0),
        }
        side_stream = (nat.TIMED_EMB_SLICE, nat.TIMED_EMB_FLUSH, nat.TIMED_USER_FWD, nat.TIMED_TEXT_WGRAD)
        out = []
        for k, samples in kern.items():
            n = len(samples)
            if n == 0:
                continue
            name, bound, work = spec[k]
            avg = sum(samples) / n
            # launches per step from the timer stride (every stride-th launch is timed); the full flush
            # runs once per phase (opt.flush() after the timed steps)
            per_step = 1.0 / steps if k == nat.TIMED_EMB_FLUSH else n * stride / steps
            srt = sorted(samples)
            med = (srt[(n - 1) // 2] + srt[n // 2]) / 2
            # The launch's start stamp (hipExtLaunchKernel's start event) is taken when the command
            # processor reaches the packet; in the first timed step the GPU is still running the work
            # the host queued ahead, so that sample can span the preceding kernels too (up to 180 us
            # against 19 in the same run's rocprofv3 trace). The rooflines use the
            # median launch, which rocprofv3's average of the same kernel matches; the average stays
            # beside it with every sample.
            ent = {"kernel": name, "bound": bound, "avg_ms": avg, "launches_timed": n,
                   "median_ms": med, "min_ms": srt[0], "max_ms": srt[-1],
                   "samples_ms": [round(v, 5) for v in samples[:64]],
                   "ms_per_step": med * per_step,
                   "critical_path": k not in side_stream}
            if bound == "mfma":
                # split-f16 kernels: f32-equivalent FLOPs against the f16 peak over their products per
                # f32 product (forward: 3; conv-1 weight gradient on the fp16 table: 2)
                nprod = 3 if ((k == nat.TIMED_CONV1_FWD and CONV_F16) or k == nat.TIMED_TEXT_FWD) else 2 if (
                    k == nat.TIMED_CONV1_WGRAD and WGRAD_F16) else 0
                split = nprod > 0
                peak = F16_PEAK_TFLOPS / nprod if split else F32_PEAK_TFLOPS
                ent.update(achieved=work / (med * 1e-3) / 1e12, peak=peak,
                           unit="TFLOP/s (f32-equivalent)" if split else "TFLOP/s", algorithmic_flops=work)
                ent["frac"] = ent["achieved"] / peak
            elif bound in ("hbm", "valu"):
                # the user-table replay (k_emb_flush*) is classed "valu": correctly rounded sqrt / div
                # per replayed element-step; its HBM fraction is informational
                ent.update(achieved=work / (med * 1e-3) / 1e9, peak=HBM_PEAK_GBS, unit="GB/s",
                           algorithmic_bytes=work)
                if k in (nat.TIMED_EMB_SLICE, nat.TIMED_EMB_FLUSH):
                    ent["active_fraction"] = active  # of the table's elements with live moments
                    ent["frozen_row_fraction"] = frozen_frac[0]  # rows the slices skip (adam_replay.h)
                ent["frac" if bound == "hbm" else "hbm_frac"] = ent["achieved"] / HBM_PEAK_GBS
                if k == nat.TIMED_TEXT_WGRAD:  # its f32 FMAs against the f32 vector peak, for information
                    fl = 2.0 * M * Ct * Ew * 3
                    ent.update(algorithmic_flops=fl, achieved_tflops=fl / (med * 1e-3) / 1e12,
                               valu_frac=fl / (med * 1e-3) / 1e12 / F32_PEAK_TFLOPS)
            out.append(ent)
        byk = {e["kernel"]: e for e in out}
        sl = byk.get(spec[nat.TIMED_EMB_SLICE][0])
        fl = byk.get(spec[nat.TIMED_EMB_FLUSH][0])
        if sl is not None and fl is not None:
            # same session: the slice's rows at the full flush's uncontended per-row rate, against its
            # live duration on the user stream beside the priority-2 critical-path kernels
            iso = fl["avg_ms"] * rows_slice / max(n_users_local, 1)
            sl["isolated_ms_estimate"] = iso
            sl["live_over_isolated"] = sl["avg_ms"] / iso if iso > 0 else None
        out.sort(key=lambda e: -e["ms_per_step"])
        return out

    def traffic_for(kernel_name, mode):
        tag = {"k_conv1_wgrad": "conv1_wgrad", "k_conv_wgrad16": "conv1_wgrad16", "k_conv_wgrad1k": "conv1_wgrad1k",
               "k_emb_flush_rows": "emb_flush_rows",
               "k_conv_rows<0,0>": "conv1_fwd", "k_text_fwd": "text_fwd", "k_user_fwd": "user_fwd",
               "k_text_wgrad": "text_wgrad"}.get(kernel_name.split(" ")[0])
        path = os.path.join(ROOT, "profiles", "pmc_%s_%s.json" % (tag, mode)) if tag else None
        if path and os.path.exists(path):
            try:
                return json.load(open(path)).get("hbm_bytes_per_launch")
            except (ValueError, OSError):
                return None
        return None

    def summary(dt, t_enq, kern, M, items_per_row, mode, phase):
        rows = world * B * args.steps / dt
        ks = kernel_rooflines(kern, M, args.steps)
        for k in ks:  # the committed PMC summary's HBM bytes per launch, where one exists
            k["traffic"] = traffic_for(k["kernel"], mode)
        # the roofline line names the largest kernel on the step's critical path (the caller's stream);
        # side-stream kernels that the step does not wait for are listed in "kernels" only
        mf = [k for k in ks if k["bound"] in ("mfma", "hbm") and k["critical_path"]]
        roof = dict(mf[0]) if mf else {}
        if roof:
            roof["traffic"] = traffic_for(roof["kernel"], mode)
        # the step against the ceiling of the arithmetic it runs (FLOP-weighted over split-f16 and f32
        # MFMA, executed FLOPs: conv 1's input gradient is elided); the canonical SURVEY §8(d) figure
        # (3 x forward, f32 peak) beside it
        flops_row = row_flops(args, items_per_row)
        ex_flops, ex_t = executed_work(args, items_per_row, M)
        roof["step_frac"] = rows / world * ex_t
        roof["step_flops_executed_per_row"] = ex_flops
        roof["step_ceiling_tflops"] = ex_flops / ex_t / 1e12
        roof["step_flops_per_row"] = flops_row
        roof["canonical_tflops_per_gpu"] = rows / world * flops_row / 1e12
        res = {"ms_per_step": dt / args.steps * 1e3, "host_enqueue_ms_per_step": t_enq / args.steps * 1e3,
               "launches_per_step": launches.get(phase), "rows_per_s": rows, "triplets_per_s": rows * N,
               "roofline": roof, "kernels": ks}
        ar = [k for k in ks if k["bound"] == "xgmi"]
        if ar:
            res["allreduce_ms_per_step"] = ar[0]["ms_per_step"]
        return res

    out = {}
    if world > 1 and os.environ.get("DCUE_BENCH_STALL_RANK") == str(rank):
        # fault injection for the self-diagnosis test (tests/test_gpu_dp.py): this rank stops, as if
        # stuck in a collective; the watchdogs and the launcher must end the job with a report
        mark("DCUE_BENCH_STALL_RANK: held before the first step")
        while True:
            time.sleep(1.0)
    # ---- phase 1: in-batch, cold user table
    plan = make_plan(False)
    ub, ib = batches(args.warmup + args.steps)
    # (--gpu-only applies to the cold phase when that is the profiled one: its GPU-only timeline)
    cold_gpu_only = args.gpu_only and args.profile_phase == "inbatch_cold"
    dt, t_enq, gpu_ms_c, kern = timed_phase("inbatch_cold", plan, inbatch_step(ub, ib), gpu_only=cold_gpu_only)
    out["inbatch_cold"] = summary(dt, t_enq, kern, B, 1, "inbatch", "inbatch_cold")
    if gpu_ms_c is not None:
        out["inbatch_cold"]["gpu_only_ms_per_step"] = gpu_ms_c
    # ---- phase 2: every local user once (outside any timed region), then in-batch steady state
    warm = inbatch_step(warm_users, warm_items)
    run(plan, warm, warm_users.shape[0])
    if "inbatch" in modes:
        ub, ib = batches(args.warmup + args.steps)
        dt, t_enq, gpu_ms, kern = timed_phase("inbatch", plan, inbatch_step(ub, ib),
                                              gpu_only=args.gpu_only and not cold_gpu_only)
        out["inbatch"] = summary(dt, t_enq, kern, B, 1, "inbatch", "inbatch")
        if gpu_ms is not None:
            out["inbatch"]["gpu_only_ms_per_step"] = gpu_ms
    checks = {"after": [], "failed": []}

    def check_state(p, phase):
        """Correctness signal of the full-size run, outside the timed region (check mode's probes,
        dcrecommend.check): the last step's loss, the dense parameters and gradients, and the
        flushed user table with both Adam moments, all finite."""
        from dcrecommend.check import StepCheck
        net._sync_plan()
        opt.flush()
        ck = StepCheck(dev)
        ck.finite(p.loss.view(1), "loss")
        ck.finite(net._flat["P"], "dense parameters")
        ck.finite(G, "dense gradients")
        st = opt._adam_state()
        ck.finite(net.user_embd.embeddings.weight, "user table")
        for k in ("em", "ev"):
            ck.finite(st[k], "user table Adam " + k)
        checks["after"].append(phase)
        checks["failed"] += [phase + ": " + f for f in ck.failed()]
        checks["failed"] += [phase + ": " + f for f in fail_flag_failures(nat.debug_fail_flags())]
        checks["last_loss_" + phase] = float(p.loss)

    if os.environ.get("DCUE_BENCH_FORCE_FAIL_FLAG") == "1":
        # test hook (tests/test_gpu_bench_checks.py): raise the device's fail word as a gave-up wait would
        nat.check(nat.lib().dcue_debug_raise_fail_flags(1), "dcue_debug_raise_fail_flags")
    check_state(plan, "inbatch")
    plan.close()
    # ---- phase 3: catalogue negatives (the reference's live sampler)
    if "catalogue" in modes:
        from dcrecommend.datasets.csr import check_catalogue_users, saturated_users, user_split_ranks
        split_items = np.nonzero(split == 0)[0].astype(np.int64)
        indptr, ranks_ = user_split_ranks(pair_user.cpu().numpy(), pair_track.cpu().numpy(), n_users_local,
                                          split_items)
        sat = saturated_users(indptr, len(split_items))
        split_d64 = torch.from_numpy(split_items).to(dev)
        indptr_d = torch.from_numpy(indptr).to(dev)
        ranks_d = torch.from_numpy(ranks_).to(dev)
        cplan = make_plan(True)
        ub, ib = batches(args.warmup + args.steps)
        check_catalogue_users(ub.cpu().numpy(), sat)
        ib64 = ib.long()
        # catalogue negatives are drawn two steps ahead on a sampling stream, as the reference's
        # DataLoader workers draw them (datasets/dcuedataset.py:207-256, in __getitem__) ahead of the
        # training step: same draw order on the one numpy-compatible stream, so the same negatives.
        # Three batch buffers; step s+1's items are built before step s is launched, so the plan
        # also prepares step s+1's bn0 statistics beside step s (dcue_plan_set_next).
        main = torch.cuda.current_stream(dev)
        samp = torch.cuda.Stream(device=dev)
        negs = [torch.empty((B, N), dtype=torch.int64, device=dev) for _ in range(3)]
        items = [torch.empty(B * (1 + N), dtype=torch.int32, device=dev) for _ in range(3)]
        ready = [torch.cuda.Event() for _ in range(3)]
        done = [torch.cuda.Event() for _ in range(3)]
        n_all = ub.shape[0]

        def draw(s):
            k = s % 3
            with torch.cuda.stream(samp):
                nat.check(nat.lib().dcue_sample_catalogue(
                    nat.ptr(mt), 0, 0, nat.ptr(split_d64), split_d64.numel(), nat.ptr(indptr_d), nat.ptr(ranks_d),
                    nat.ptr(ub[s]), B, N, nat.ptr(negs[k]), samp.cuda_stream), "dcue_sample_catalogue")
                nat.check(nat.lib().dcue_build_catalogue_batch(nat.ptr(ib64[s]), nat.ptr(negs[k]), B, N,
                                                               nat.ptr(items[k]), samp.cuda_stream),
                          "dcue_build_catalogue_batch")
                ready[k].record(samp)

        samp.wait_stream(main)  # the batch tensors and the sampler state are written on the main stream
        draw(0)
        if n_all > 1:
            draw(1)

        def cat_step(plan, s):
            last = min(s + 1, n_all - 1)
            main.wait_event(ready[last % 3])  # step s's batch and (lookahead) step s+1's
            if s + 1 < n_all:
                plan.set_next(items[(s + 1) % 3])
            if world > 1 and comm is None:
                plan.launch(ub[s], items[s % 3])
                D.allreduce_mean_overlapped_(plan, G, G_late)
                opt.step()
            else:
                plan.step(ub[s], items[s % 3])
            done[s % 3].record(main)
            if s + 2 < n_all:  # buffer (s+2) % 3 was step s-1's: free once that step is done
                if s >= 1:
                    samp.wait_event(done[(s - 1) % 3])
                draw(s + 2)
            sched_step()
        dt, t_enq, _, kern = timed_phase("catalogue", cplan, cat_step)
        out["catalogue"] = summary(dt, t_enq, kern, B * (1 + N), 1 + N, "catalogue", "catalogue")
        check_state(cplan, "catalogue")
        cplan.close()
    # ---- phase 4: BASELINE config 4, the mixed audio + text item tower at d = 256,
    # in-batch steps as phase 2 on the same users, tracks and interactions, each track with a synthetic
    # sentence (BOS + words + EOS + PAD) and random 300-d word vectors in place of the LM-pretrained
    # ones (caller-supplied; none can be fetched here)
    if "text" in modes:
        mark("text phase")
        Dt = args.text_feature_dim
        torch.manual_seed(0)
        tnet = DCUENet({"feature_dim": Dt, "conv_hidden": args.hidden, "user_embdim": args.user_embdim,
                        "user_count": n_users_local, "model_type": "truedcuemel1dbntext",
                        "text_dim": args.text_dim, "word_dim": args.word_dim, "text_len": args.text_len,
                        "n_words": args.n_words, "pad_idx": 0}).to(dev)
        tnet.train()
        with torch.no_grad():
            tnet.text.embeddings.weight.copy_(torch.randn(args.n_words, args.word_dim, generator=gen, device=dev) * 0.3)
        tokens = synthetic_sentences(args.tracks, args.text_len, args.n_words, dev, seed=77)
        topt = NativeAdam(tnet.parameters(), 1e-5, (0.9, 0.99), 1e-8, 0, defer_embedding=defer,
                          flush_every=args.flush_every)
        tsched = CyclicLRWithRestarts(topt, B, epoch_size=epoch_size, restart_period=30, t_mult=2, policy="cosine")
        tsched.step()
        tplan = TrainPlan(tnet, tracks, B, N, mt_state=mt, emb_grad_scale=1.0 / world, optimizer=topt,
                          tokens=tokens)
        if comm is not None:
            tplan.set_comm(comm)

        def text_step(users_b, items_b):
            users_b, items_b = list(users_b.unbind(0)), list(items_b.unbind(0))

            def fn(plan, s):
                if world > 1 and comm is None:
                    plan.launch(users_b[s], items_b[s])
                    D.allreduce_mean_overlapped_(plan, tnet._flat["G"], D.late_grad_floats(tnet))
                    topt.step()
                else:
                    if s + 1 < len(users_b):
                        plan.set_next(items_b[s + 1])
                    plan.step(users_b[s], items_b[s])
                try:
                    tsched.batch_step()
                except StopIteration:
                    tsched.step()
                    tsched.batch_step()
            return fn
        ub, ib = batches(args.warmup + args.steps)
        dt, t_enq, _, kern = timed_phase("text", tplan, text_step(ub, ib), optim=topt)
        rows = world * B * args.steps / dt
        ks = kernel_rooflines(kern, B, args.steps, optim=topt, d=Dt)
        for k in ks:
            k["traffic"] = traffic_for(k["kernel"], "text")
        tk = [k for k in ks if k["kernel"].startswith("k_text_fwd")]
        troof = dict(tk[0]) if tk else {}
        if troof:
            troof["traffic"] = traffic_for(troof["kernel"], "text")
        tflops_row = 3 * (item_flops(args.hidden, Dt) + 2.0 * args.text_dim * Dt
                          + text_conv_flops(args.text_len, args.word_dim, args.text_dim)) \
            + 3 * 2 * (args.user_embdim ** 2 + args.user_embdim * Dt)
        troof["step_flops_per_row"] = tflops_row
        tnet._sync_plan()
        topt.flush()
        out["text"] = {
            "workload": "DCUE truedcuemel1dbntext (config 4): d=%d H=%d E=%d + text Conv1d(%d -> %d, k 3) over "
                        "%d-token sentences of a %d-word vocabulary, fc(%d + %d -> %d); %d users x %d tracks, "
                        "in-batch N=%d" % (Dt, args.hidden, args.user_embdim, args.word_dim, args.text_dim,
                                           args.text_len, args.n_words, args.text_dim, Dt, Dt, args.users,
                                           args.tracks, N),
            "ms_per_step": dt / args.steps * 1e3, "host_enqueue_ms_per_step": t_enq / args.steps * 1e3,
            "launches_per_step": launches.get("text"), "rows_per_s": rows, "triplets_per_s": rows * N,
            "roofline": troof, "kernels": ks, "last_loss": float(tplan.loss),
            "finite": bool(torch.isfinite(tnet._flat["P"]).all()) and bool(torch.isfinite(tplan.loss)),
            "data": "synthetic: random word vectors (N(0, 0.09)) stand in for the LM-pretrained ones",
            "parity": "unpinned against the reference (its text encoder was never published, "
                      "datasets/dcuelmitemset.py:8); pinned against oracle/text_oracle.py (tests/test_gpu_text.py)"}
        if not out["text"]["finite"]:
            checks["failed"].append("text: non-finite dense parameters or loss")
        checks["failed"] += ["text: " + f for f in fail_flag_failures(nat.debug_fail_flags())]
        tplan.close()
        del tplan, topt, tnet, tokens
    # ---- phase 5 (N = 1): the DCBR path (BASELINE config 5): WRMF target factors of
    # the same interactions, then the audio ConvNet regressing them (catalogue-sized item batches)
    if "dcbr" in modes and (world == 1 or comm is not None) and args.feature_dim <= 128:
        mark("dcbr phase")
        if world == 1:
            out["dcbr"] = dcbr_phase(args, tracks, pair_user, pair_track, n_users_local, dev, B * (1 + N))
        else:  # every rank the same (global) interaction set, solved row-sharded
            g_all = torch.Generator(device=dev).manual_seed(4242)
            all_u = torch.randint(0, args.users, (args.interactions,), generator=g_all, device=dev)
            all_t = torch.randint(0, args.tracks, (args.interactions,), generator=g_all, device=dev, dtype=torch.int64)
            out["dcbr"] = dcbr_phase(args, tracks, all_u, all_t, args.users, dev, B * (1 + N), comm=comm,
                                     world=world, rank=rank)
            del all_u, all_t
        if not out["dcbr"]["finite"]:
            checks["failed"].append("dcbr: non-finite WRMF factors, regression parameters or loss")
    head = out.get("inbatch", out["inbatch_cold"])
    E = args.user_embdim
    result = {
        "metric": "training triplets/sec (whole node) + AUC@val, DCUE d=128 at 1/2/4/8 MI355X",
        "value": head["triplets_per_s"],
        "unit": "triplets/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": head["ms_per_step"],
        "host_enqueue_ms_per_step": head["host_enqueue_ms_per_step"],
        "launches_per_step": head["launches_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": ("f32 (conv forwards, input and weight gradients: f32 values as power-of-two-scaled split "
                  "fp16 hi+lo pairs on f16 MFMA, f32 accumulate)") if CONV_F16 or WGRAD_F16 else "f32",
        "data": "synthetic",
        "rows_per_s": head["rows_per_s"],
        "auc_val": None,
        "config": {"workload": "DCUE truedcuemel1dbn d=%d H=%d E=%d, %d users x %d tracks (fp16 table), "
                               "%d interactions, in-batch negatives N=%d"
                               % (args.feature_dim, args.hidden, E, args.users, args.tracks, args.interactions, N),
                   "regime": ("steady state: every local user's Adam moments live (one pass over all users "
                              "before the timed steps)") if "inbatch" in out else "cold user table",
                   "batch_per_gpu": B, "global_batch": B * world, "neg": N,
                   "parallelism": "dp%d (users sharded, dense grads all-reduced)" % world,
                   "exchange": ("RCCL inside the plan step (libdcue_hip)" if comm is not None else
                                "torch.distributed (%s) from Python%s" % (
                                    backend, "; native RCCL failed: " + comm_error if comm_error else ""))
                               if world > 1 else None,
                   "batchnorm": "sync (global batch)" if (comm is not None and args.sync_bn) else "per replica",
                   "process_group_world": dist.get_world_size() if world > 1 else 1},
        "roofline": head["roofline"],
        "kernels": head["kernels"],
        "inbatch_cold": {k: out["inbatch_cold"][k] for k in ("ms_per_step", "rows_per_s", "triplets_per_s",
                                                             "host_enqueue_ms_per_step", "launches_per_step")},
    }
    if host_trace:
        result["host_issue_us"] = host_trace
    if "allreduce_ms_per_step" in head:
        result["allreduce_ms_per_step"] = head["allreduce_ms_per_step"]
    if "gpu_only_ms_per_step" in head:
        result["gpu_only_ms_per_step"] = head["gpu_only_ms_per_step"]
    if "catalogue" in out:
        result["catalogue"] = out["catalogue"]
    if "text" in out:
        result["text"] = out["text"]
    if "dcbr" in out:
        result["dcbr"] = out["dcbr"]
    # every roofline fraction in the line must be physically possible: a fraction above 1 is an
    # algorithmic-work count that overstates what the kernel did
    def over_one(o, path):
        if isinstance(o, dict):
            for k, v in o.items():
                if k in ("frac", "hbm_frac", "step_frac") and isinstance(v, (int, float)) and v > 1.0:
                    yield "%s.%s = %.3f" % (path, k, v)
                else:
                    yield from over_one(v, path + "." + k if path else k)
        elif isinstance(o, list):
            for i, v in enumerate(o):
                yield from over_one(v, "%s[%d]" % (path, i))
    bad_frac = list(over_one(result, ""))
    if bad_frac:
        checks["failed"].append("roofline fractions above 1: " + "; ".join(bad_frac))
    checks["finite"] = not any(not f.startswith("roofline") for f in checks["failed"])
    result["checks"] = checks
    # data parallelism's invariant: every rank steps the same dense replica (the exchange averaged
    # the same gradient into every rank's Adam); a broken exchange shows up here as differing replicas
    mark("replica checksum all-reduce")
    net._sync_plan()
    same, lo, hi = D.replica_checksums(net._flat["P"])
    result["replicas_identical"] = same
    if not same:
        result["replica_fingerprint_min_max"] = [lo, hi]
    if world > 1:
        D.broadcast_buffers_(net)  # DDP semantics: evaluate with rank 0's BN statistics
    if rank == 0 and not args.no_eval:
        # AUC@val of the trained model (outside the timed region): DCUE.score over an eval_pct
        # sample of this rank's users (nn/dcue.py:380-449, 580-603) on the GPU evaluator
        ev = evaluate_val(args, net, tracks, pair_user, pair_track, split, n_users_local, dev)
        result["auc_val"] = ev.pop("auc")
        result["eval"] = ev
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args, n_users_local)
    if rank == 0 and world == 1 and not args.no_f32_probe:
        result["exact_f32"] = exact_f32_probe(args)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if comm is not None:
        comm.close()
    if world > 1:
        dist.destroy_process_group()
    if checks["failed"]:  # a diverged phase is a failed run, whatever its throughput
        print("bench: checks failed: %s" % "; ".join(checks["failed"]), file=sys.stderr, flush=True)
        sys.exit(1)


if __name__ == "__main__":
    main()
