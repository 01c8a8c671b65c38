"""Data-parallel layout of the DCUE step: one process per GPU, users sharded, dense grads all-reduced.

SURVEY.md §8(e). The interaction set is sharded BY USER: global user u lives on rank u % W as local
row u // W, so each rank owns its users' embedding rows and their Adam moments (the user table and
its optimizer state never cross xGMI), and the per-rank user-table Adam work is 1/W. The track table
is replicated. The one exchange per step is the all-reduce (sum, then / W) of the replicated dense
gradient -- the flat buffer DCUENet keeps (393,276 fp32 at d=H=128) -- which together with
emb_grad_scale = 1/W on the local rows reproduces DDP's mean-over-ranks gradient.

Two ways to run the exchange:
* NativeComm + TrainPlan.set_comm (the production path): libdcue_hip owns an RCCL communicator and
  the whole data-parallel step -- sample, forward, backward, the two-bucket all-reduce overlapped
  with the conv-1 weight gradient, Adam with the divide by W fused in -- stays ONE host call
  (TrainPlan.step), exactly as the single-GPU step.
* HostComm + TrainPlan.set_comm: the same native plan step and exchange code, with the library
  handing each bucket to a torch.distributed all-reduce on the host (gloo): for several ranks that
  share one GPU, which RCCL does not allow (tests), not for speed.
* allreduce_mean_overlapped_ over a torch.distributed group: the same buckets from Python (gloo
  on CPU tests, or several ranks sharing one GPU).

BatchNorm running statistics are per replica during training, as under DDP without SyncBN; DDP's
default broadcast_buffers makes every rank use rank 0's buffers, which broadcast_buffers_ does
before evaluation or a checkpoint.
"""
import ctypes

import torch
import torch.distributed as dist


def local_user_count(n_users, rank, world):
    """Rows of the user table rank `rank` owns: global users u with u % world == rank."""
    return (n_users - rank + world - 1) // world if n_users > rank else 0


def to_local_user(u, world):
    return u // world


def to_global_user(u_local, rank, world):
    return u_local * world + rank


def shard_interactions(user_idx, item_idx, rank, world):
    """This rank's (local user, item) pairs of a global interaction list (tensors or arrays)."""
    user_idx = torch.as_tensor(user_idx)
    item_idx = torch.as_tensor(item_idx)
    keep = (user_idx % world) == rank
    return user_idx[keep] // world, item_idx[keep]


def allreduce_mean_(grad, group=None):
    """In-place mean of a replicated gradient over the ranks (RCCL on GPU, gloo in CPU tests)."""
    world = dist.get_world_size(group)
    if world > 1:
        dist.all_reduce(grad, group=group)
        grad.div_(world)
    return grad


def late_grad_floats(net):
    """Floats at the head of the flat gradient that the step's end writes (bn0, conv layer 1, bn1:
    segments [0, SEG_LATE) of the reference order); everything after is final once the plan's side
    streams are in."""
    from . import _native as nat
    dims = net._flat["dims"] if net._flat is not None else nat.make_dims(
        net.conv_hidden, net.feature_dim, net.user_embdim, net.user_count, net.model_type)
    return nat.param_layout(dims)[nat.SEG_LATE]


_COMM_STREAMS = {}


def allreduce_mean_overlapped_(plan, grad, late, group=None):
    """In-place mean over the ranks of the flat gradient of the step `plan` last launched, in two
    buckets. grad[late:] -- every gradient but bn0/conv1/bn1 -- is all-reduced as soon as the
    plan's side streams are in, from a stream of its own, so it overlaps the step's conv-1 weight
    gradient on the caller's stream; grad[:late] follows after the step's end. The caller's stream
    then waits for both (RCCL runs them in issue order on the process group's stream). On CPU
    tensors (gloo tests) the buckets run in order."""
    world = dist.get_world_size(group)
    if world == 1:
        return grad
    if grad.is_cuda:
        dev = grad.device
        comm = _COMM_STREAMS.get(dev)
        if comm is None:
            comm = _COMM_STREAMS[dev] = torch.cuda.Stream(device=dev)
        plan.wait_side(comm)
        with torch.cuda.stream(comm):
            w_early = dist.all_reduce(grad[late:], group=group, async_op=True)
        w_late = dist.all_reduce(grad[:late], group=group, async_op=True)
        w_early.wait()
        w_late.wait()
    else:
        plan.wait_side(None)
        dist.all_reduce(grad[late:], group=group)
        dist.all_reduce(grad[:late], group=group)
    grad.div_(world)
    return grad


def max_over_ranks(value, device, group=None):
    """Max of a host scalar over the ranks (bench timing: the slowest rank defines the step)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def replica_checksums(buf, group=None):
    """Whether every rank holds the same dense replica: a per-rank fingerprint of `buf` (fp64 sum,
    sum of squares and a position-weighted sum, so a permutation or a sign flip shows), reduced
    with MIN and MAX over the ranks. Returns (identical, fingerprint min, fingerprint max)."""
    x = buf.detach().double().reshape(-1)
    w = torch.arange(1, x.numel() + 1, dtype=torch.float64, device=x.device) / max(x.numel(), 1)
    fp = torch.stack([x.sum(), (x * x).sum(), (x * w).sum()])
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        v = fp.cpu().tolist()
        return True, v, v
    lo, hi = fp.clone(), fp.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    lo, hi = lo.cpu().tolist(), hi.cpu().tolist()
    return lo == hi, lo, hi


def broadcast_buffers_(net, group=None, src=0):
    """Every rank takes rank `src`'s BN running statistics and batch counters (DDP's
    broadcast_buffers semantics), e.g. before evaluation or saving on rank 0."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return net
    for _, b in net.named_buffers():
        dist.broadcast(b.data, src=src, group=group)
    return net


class NativeComm:
    """An RCCL communicator owned by libdcue_hip (include/dcue.h dcue_comm_*) over the ranks of a
    torch.distributed group, which only carries the unique id from rank 0."""

    def __init__(self, group=None):
        from . import _native as nat
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        obj = [None]
        if self.rank == 0:
            buf = (ctypes.c_ubyte * nat.COMM_ID_BYTES)()
            nat.check(nat.lib().dcue_comm_unique_id(buf), "dcue_comm_unique_id")
            obj[0] = bytes(buf)
        dist.broadcast_object_list(obj, src=0, group=group)
        buf = (ctypes.c_ubyte * nat.COMM_ID_BYTES).from_buffer_copy(obj[0])
        handle = ctypes.c_void_p()
        nat.check(nat.lib().dcue_comm_create(buf, self.world, self.rank, ctypes.byref(handle)),
                  "dcue_comm_create")
        self.handle = handle
        self._lib = nat.lib()

    def allreduce_mean_(self, t):
        """In place: the mean of a GPU float32 tensor over the ranks (ordered on the current stream)."""
        from . import _native as nat
        if t.dtype != torch.float32 or not t.is_cuda or not t.is_contiguous():
            raise ValueError("allreduce_mean_ needs a contiguous float32 GPU tensor")
        nat.check(self._lib.dcue_comm_allreduce_mean(self.handle, nat.ptr(t), t.numel(), nat.stream_handle()),
                  "dcue_comm_allreduce_mean")
        return t

    def allgather_(self, t):
        """In place: t holds world equal parts along dim 0, this rank's at index `rank`; afterwards
        every rank holds all of them (dcue_comm_allgather)."""
        from . import _native as nat
        if t.dtype != torch.float32 or not t.is_cuda or not t.is_contiguous() or t.numel() % self.world:
            raise ValueError("allgather_ needs a contiguous float32 GPU tensor of world equal parts")
        nat.check(self._lib.dcue_comm_allgather(self.handle, nat.ptr(t), t.numel() // self.world,
                                                nat.stream_handle()), "dcue_comm_allgather")
        return t

    def close(self):
        if getattr(self, "handle", None) is not None:
            self._lib.dcue_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HostComm(NativeComm):
    """A libdcue_hip communicator whose transport is a torch.distributed group on the host
    (dcue_comm_create_host): the plan's native exchange -- both buckets, their event order, Adam's
    divide by the world size -- runs unchanged, each bucket summed by `dist.all_reduce` on a CPU view
    of the library's pinned staging buffer. uint64 buffers are summed as int64 (the same bits: two's
    complement addition wraps identically)."""

    def __init__(self, group=None):
        from . import _native as nat
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self._group = group

        def _allreduce(ctx, host_buf, n, dtype):
            try:
                ct = ctypes.c_float if dtype == nat.COMM_F32 else ctypes.c_int64
                arr = (ct * int(n)).from_address(host_buf)
                t = torch.frombuffer(arr, dtype=torch.float32 if dtype == nat.COMM_F32 else torch.int64)
                dist.all_reduce(t, group=self._group)
                return 0
            except Exception as e:  # reported through the library's error path (non-zero)
                print("HostComm all-reduce failed: %r" % (e,), flush=True)
                return 1

        self._cb = nat.HOST_ALLREDUCE_FN(_allreduce)  # kept alive as long as the communicator
        handle = ctypes.c_void_p()
        nat.check(nat.lib().dcue_comm_create_host(self.world, self.rank, self._cb, None, ctypes.byref(handle)),
                  "dcue_comm_create_host")
        self.handle = handle
        self._lib = nat.lib()
