"""Data-parallel gradient exchange with overlap (row e, dcrecommend.distributed): two ranks on one
GPU (gloo), the bucketed all-reduce issued behind the step against a plain post-step all-reduce.

Bar: bit-exact (two addends per element either way). The ranks are child processes
(tests/dp_worker.py), started with subprocess like any other program.
"""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_overlapped_allreduce_matches_plain(tmp_path):
    world, port = 2, _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), OUT=str(tmp_path))
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "dp_worker.py")], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out)
    for r, p in enumerate(procs):
        assert p.returncode == 0, "rank %d failed:\n%s" % (r, outs[r][-3000:])
    parts = [torch.load(os.path.join(tmp_path, "r%d.pt" % r), weights_only=True) for r in range(world)]
    assert torch.equal(parts[0]["G"], parts[1]["G"])  # the mean is the same on every rank
    assert 0 < parts[0]["late"] < parts[0]["G"].numel()


def _pair_nets(n_users=40, E=40):
    from dcrecommend.dcue.dcue import DCUENet
    nets = []
    for _ in range(2):
        torch.manual_seed(5)
        nets.append(DCUENet({"feature_dim": 32, "conv_hidden": 32, "user_embdim": E, "user_count": n_users,
                             "model_type": "truedcuemel1dbn"}).cuda().train())
    return nets


def _full_state(net, opt):
    out = {k: v.detach().clone() for k, v in net.state_dict().items()}
    st = opt._adam_state()
    for k in ("m", "v", "em", "ev"):
        out["adam." + k] = st[k].clone()
    out["grad"] = net._flat["G"].clone()
    return out


def test_native_exchange_in_plan_step_world1():
    """The plan's own RCCL exchange (dcue_plan_set_comm) on a one-rank communicator: the step with
    the exchange bound (events, comm stream, both buckets, Adam's divide) is bit-exact with the step
    without it. (RCCL refuses two ranks on one GPU, so the multi-rank numbers come from the 8-GPU
    bench; the bucket arithmetic itself is covered by test_overlapped_allreduce_matches_plain.)"""
    import torch.distributed as dist
    from dcrecommend import distributed as D
    from dcrecommend.dcue.plan import TrainPlan
    from dcrecommend.optim import NativeAdam
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % _free_port(), rank=0, world_size=1)
    try:
        comm = D.NativeComm()
        assert comm.world == 1 and comm.rank == 0
        a, b = _pair_nets()
        gen = torch.Generator(device="cuda:0").manual_seed(11)
        tracks = torch.randn((48, 131, 128), generator=gen, device="cuda:0").half()
        opts = [NativeAdam(n.parameters(), 1e-3, (0.9, 0.99), 1e-8, 0, defer_embedding=True, flush_every=4)
                for n in (a, b)]
        B, N = 8, 3
        plans = [TrainPlan(n, tracks, B, N, mt_state=None, optimizer=o) for n, o in zip((a, b), opts)]
        plans[0].set_comm(comm)
        for _ in range(6):
            users = torch.randint(0, 40, (B,), generator=gen, device="cuda:0")
            items = torch.randint(0, 48, (B * (1 + N),), generator=gen, device="cuda:0").to(torch.int32)
            for p in plans:
                p.step(users, items)
        for o in opts:
            o.flush()
        torch.cuda.synchronize()
        sa, sb = _full_state(a, opts[0]), _full_state(b, opts[1])
        for k in sa:
            assert torch.equal(sa[k], sb[k]), k
        t = torch.arange(1000, dtype=torch.float32, device="cuda:0")
        comm.allreduce_mean_(t)
        assert torch.equal(t.cpu(), torch.arange(1000, dtype=torch.float32))
        for p in plans:
            p.close()
        comm.close()
    finally:
        dist.destroy_process_group()


def test_adam_grad_div_is_the_ddp_mean():
    """dcue_adam_args.grad_div = W on a summed gradient == the step on the mean (W a power of two:
    both exact), and the gradient buffer holds the mean afterwards (grad.div_(world) semantics)."""
    import ctypes
    from dcrecommend import _native as nat
    from dcrecommend.optim import NativeAdam
    a, b = _pair_nets()
    gen = torch.Generator(device="cuda:0").manual_seed(3)
    tracks = torch.randn((48, 131, 128), generator=gen, device="cuda:0").half()
    users = torch.randint(0, 40, (8,), generator=gen, device="cuda:0")
    items = torch.randint(0, 48, (32,), generator=gen, device="cuda:0").to(torch.int32)
    opts = []
    for n in (a, b):
        n.native_forward(users, tracks, items, 3, nat.LAYOUT_CATALOGUE, None, train=True)
        n.native_backward(None)
        opts.append(NativeAdam(n.parameters(), 1e-3, (0.9, 0.99), 1e-8, 0))
    a._flat["G"].mul_(4.0)  # as if 4 ranks had summed this rank's gradient
    for n, o, div in ((a, opts[0], 4.0), (b, opts[1], 0.0)):
        st = o._adam_state()
        args = nat.AdamArgs(1e-3, 0.9, 0.99, 1e-8, 0.0, 1, nat.ADAM_DENSE, div)
        nat.check(nat.lib().dcue_adam_step(ctypes.byref(n._model_struct(st)), ctypes.byref(args),
                                           nat.stream_handle()), "dcue_adam_step")
    torch.cuda.synchronize()
    assert torch.equal(a._flat["G"], b._flat["G"])
    assert torch.equal(a._flat["P"], b._flat["P"])


def _bench(args, env=None, timeout=240):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                         timeout=timeout, env=dict(os.environ, **(env or {})))
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    import json
    return json.loads(lines[0])


SMALL = ["--steps", "3", "--warmup", "1", "--no-eval", "--no-cpu-baseline", "--users", "3000", "--tracks",
         "4000", "--interactions", "60000"]


def test_bench_single_gpu_line():
    """The bench line's contract fields at a small workload: the steady-state in-batch value, the
    cold in-batch and the catalogue phases, kernel rooflines with the step-level fraction."""
    r = _bench(SMALL)
    assert r["n_gpus"] == 1 and r["value"] > 0 and r["unit"] == "triplets/s"
    assert r["catalogue"]["rows_per_s"] > 0 and r["inbatch_cold"]["rows_per_s"] > 0
    assert 0 < r["roofline"]["step_frac"] < 1
    assert r["kernels"] and all(k["avg_ms"] > 0 for k in r["kernels"])


def test_bench_launches_its_own_ranks():
    """`bench.py --gpus 2` started directly (no torch.distributed.run) spawns two ranks before any
    GPU call; here both share the one GPU over gloo with the Python exchange (RCCL needs a GPU per
    rank); rank 0 prints the single line with the whole-job numbers."""
    r = _bench(["--gpus", "2"] + SMALL, env={"DCUE_DIST_BACKEND": "gloo"})
    assert r["n_gpus"] == 2 and r["config"]["process_group_world"] == 2
    assert r["config"]["global_batch"] == 2 * r["config"]["batch_per_gpu"]
    assert r["value"] > 0 and r["catalogue"]["rows_per_s"] > 0
    assert r["replicas_identical"] is True  # every rank stepped the same dense replica


def test_bench_stalled_rank_reports_and_exits():
    """a rank that stops making progress (here rank 1 is held before its first
    step by DCUE_BENCH_STALL_RANK, as a hung collective would hold it) is reported -- which rank,
    how long, its last position -- and every rank ends with a non-zero status instead of waiting
    for the driver's kill."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--stall-s", "15"] + SMALL,
                         capture_output=True, text=True, timeout=200,
                         env=dict(os.environ, DCUE_DIST_BACKEND="gloo", DCUE_BENCH_STALL_RANK="1"))
    assert out.returncode != 0
    assert "no progress for" in out.stderr and "last position" in out.stderr, out.stderr[-3000:]
    assert not [l for l in out.stdout.splitlines() if l.startswith("{")]


@pytest.mark.parametrize("kind", ["sgd", "ranger"])
def test_plan_launch_with_comm_feeds_other_optimizers_world1(kind):
    """TrainPlan.step with NativeSGD / NativeRanger runs launch() then the optimizer's own
    sweep. With a communicator bound, launch() now exchanges the dense gradient and leaves the mean
    (dcue_plan_launch + comm_divide), so no optimizer sees an un-averaged gradient. At world 1 the
    step is bit-exact with the unbound one (the exchange path runs; the mean is the identity)."""
    import torch.distributed as dist
    from dcrecommend import distributed as D
    from dcrecommend.dcue.plan import TrainPlan
    from dcrecommend.optim import NativeRanger, NativeSGD
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % _free_port(), rank=0, world_size=1)
    try:
        comm = D.NativeComm()
        a, b = _pair_nets()
        gen = torch.Generator(device="cuda:0").manual_seed(12)
        tracks = torch.randn((48, 131, 128), generator=gen, device="cuda:0").half()
        mk = ((lambda ps: NativeSGD(ps, 1e-3, momentum=0.9, nesterov=True)) if kind == "sgd"
              else (lambda ps: NativeRanger(ps, 1e-3)))
        opts = [mk(n.parameters()) for n in (a, b)]
        B, N = 8, 3
        plans = [TrainPlan(n, tracks, B, N, mt_state=None, optimizer=o) for n, o in zip((a, b), opts)]
        plans[0].set_comm(comm)
        for _ in range(4):
            users = torch.randint(0, 40, (B,), generator=gen, device="cuda:0")
            items = torch.randint(0, 48, (B * (1 + N),), generator=gen, device="cuda:0").to(torch.int32)
            for p in plans:
                p.step(users, items)
        torch.cuda.synchronize()
        for k, v in a.state_dict().items():
            assert torch.equal(v, b.state_dict()[k]), k
        assert torch.equal(a._flat["G"], b._flat["G"])
        for p in plans:
            p.close()
        comm.close()
    finally:
        dist.destroy_process_group()


def test_bench_forced_fail_flag_fails_the_line():
    """a non-zero device fail word (dcue_debug_fail_flags: the fused user-tower
    forward's bounded wait gave up) fails the bench line -- checks.failed names it and the exit status
    is 1 -- instead of being visible to the tests only. DCUE_BENCH_FORCE_FAIL_FLAG raises the word
    through dcue_debug_raise_fail_flags after the in-batch phase."""
    import json
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--modes", "inbatch", "--no-f32-probe"]
                         + SMALL, capture_output=True, text=True, timeout=240,
                         env=dict(os.environ, DCUE_BENCH_FORCE_FAIL_FLAG="1"))
    assert out.returncode == 1, out.stdout[-2000:] + out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    r = json.loads(lines[0])
    assert any("fail flags" in f for f in r["checks"]["failed"]), r["checks"]
    assert "fail flags" in out.stderr
