"""Bound replay of the DCUE training step's sample + forward + backward (include/dcue.h dcue_plan_*).

The reference trainer runs, per batch, `model(u, pos, neg)` -> `loss.backward()` (nn/dcue.py:202-208)
after its in-batch sampler drew the negatives (nn/dcue.py:698-709). TrainPlan binds exactly that
work -- the GPU MT19937 draw, dcue_forward(train) and dcue_train_backward -- to fixed batch buffers
once and replays it with one host call per step: issued from C++ (default) or as a captured HIP
graph (graph=True; slower on ROCm 7.2). The optimizer step (NativeAdam.step) and any
gradient all-reduce stay outside, between replays.

Build the optimizer (and with it any deferred user-table state) BEFORE the plan: the graph binds the
buffers that exist at creation and refuses to run if the model or optimizer state was rebuilt.
"""
import collections
import ctypes

import torch

from dcrecommend import _native as nat
from dcrecommend.check import ProbeCheck, StepCheck, enabled_by_env


class TrainPlan:

    def __init__(self, net, tracks, n_rows, n_neg, mt_state=None, item_track=None, margin=0.2,
                 emb_grad_scale=1.0, graph=False, optimizer=None, check=None, tokens=None):
        """tracks: HBM track table [n_tracks][131][128] (fp16/fp32). In-batch mode (mt_state given):
        positives are items 0..B-1 of item_track, negatives drawn in-graph. Otherwise item_track holds
        B*(1+N) items in catalogue order (datasets/dcuedataset.py:242-250). tokens: the text tower's
        [n_tracks][text_len] int32 token table (BASELINE config 4), bound like `tracks`."""
        fl = net._require_device()
        dev = fl["P"].device
        B, N = int(n_rows), int(n_neg)
        self.inbatch = mt_state is not None
        M = B if self.inbatch else B * (1 + N)
        self.net, self.tracks, self.tokens = net, tracks, tokens
        self.users = torch.zeros(B, dtype=torch.int64, device=dev)
        self.item_track = torch.zeros(M, dtype=torch.int32, device=dev)
        if item_track is not None:
            self.item_track.copy_(item_track)
        self.neg_item = torch.zeros((B, N), dtype=torch.int32, device=dev) if self.inbatch else None
        self.mt_state = mt_state
        self.ws = net._workspace(B, N, M)
        off = nat.workspace_outputs(fl["dims"], B, N, M)
        # the last launched step's mean hinge loss (nn/dcue.py:167-170), a device view into the workspace
        self.loss = self.ws[off[3]:off[3] + 4].view(torch.float32)[0]
        self.optimizer = optimizer
        # with an optimizer the plan also owns the Adam step (step()); the struct then carries its state
        self._fused_adam = optimizer is not None and hasattr(optimizer, "_adam_state")
        model = net._model_struct(optimizer._adam_state() if self._fused_adam else None)
        opt = net._deferred_opt() if getattr(net, "_deferred_opt", None) is not None else None
        self._bound = (fl, self.ws, fl["emb_grad"], opt._moments if opt is not None else None)
        self._keep = (fl["emb_grad"], fl["emb_rows"])
        batch = nat.Batch(B, N, M, nat.LAYOUT_GATHER if self.inbatch else nat.LAYOUT_CATALOGUE,
                          self.users.data_ptr(), self.item_track.data_ptr(),
                          self.neg_item.data_ptr() if self.inbatch else None)
        tr = net._tracks(tracks, tokens)
        flags = (nat.PLAN_SAMPLE_INBATCH if self.inbatch else 0) | (nat.PLAN_GRAPH if graph else 0)
        cfg = nat.PlanConfig(flags, float(margin),
                             float(emb_grad_scale), 0, mt_state.data_ptr() if self.inbatch else None)
        handle = ctypes.c_void_p()
        nat.check(nat.lib().dcue_plan_create(ctypes.byref(model), ctypes.byref(batch), ctypes.byref(tr),
                                             nat.ptr(self.ws), self.ws.numel(), ctypes.byref(cfg),
                                             ctypes.byref(handle)), "dcue_plan_create")
        self._handle = handle
        self._lib = nat.lib()
        # the stream the plan issues on: torch's current stream at creation (pass stream= to override)
        self._stream = nat.stream_handle()
        self._adam_args = nat.AdamArgs()
        # source batches stay referenced for a few steps: the plan's side streams read them
        # asynchronously (the caching allocator must not hand their memory out meanwhile)
        self._hold = collections.deque(maxlen=4)
        # the replayed backward writes the flat gradient: expose the reference-shaped .grad views
        net._expose_grads()
        net.user_embd.embeddings.weight.grad = None
        net._grad_users = self.users
        # check mode (dcrecommend.check): ids validated before each step, loss/params/grads after
        if check is None:
            check = enabled_by_env()
        # check="probe": in-stream output probes only, read at close() / probe_report()
        self._probes = ProbeCheck(dev) if check == "probe" else None
        self._check = StepCheck(dev) if check and check != "probe" else None
        self._n_users = int(fl["dims"].n_users)

    def _check_before(self, users, item_track):
        ck = self._check
        ck.ids(self.users if users is None else users, self._n_users, "user ids outside the table")
        ck.ids(self.item_track if item_track is None else item_track, self.tracks.shape[0],
               "item ids outside the track table")
        ck.raise_if_any()

    def _check_after(self):
        self.sync()
        ck, fl = self._check, self.net._flat
        ck.finite(self.loss.view(1), "non-finite loss")
        ck.finite(fl["P"], "non-finite dense parameters")
        ck.finite(fl["G"], "non-finite dense gradients")
        ck.raise_if_any()

    def _check_bound(self):
        net = self.net
        opt = net._deferred_opt() if getattr(net, "_deferred_opt", None) is not None else None
        now = (net._flat, net._ws, net._flat["emb_grad"] if net._flat else None,
               opt._moments if opt is not None else None)
        if any(a is not b for a, b in zip(now, self._bound)):
            raise RuntimeError("TrainPlan: the model's device buffers or the optimizer state were rebuilt "
                               "after the plan was created; create a new plan")

    def launch(self, users=None, item_track=None, stream=None):
        """One training step's sample + forward + backward. users [B] int64 / item_track [M] int32
        (device tensors, optional) are copied into the bound batch buffers first."""
        if self._handle is None:
            raise RuntimeError("TrainPlan was closed")
        self._check_bound()
        if self._check is not None:
            self._check_before(users, item_track)
        self._hold.append((users, item_track))
        st = self._lib.dcue_plan_launch(self._handle, None if users is None else users.data_ptr(),
                                        None if item_track is None else item_track.data_ptr(),
                                        self._stream if stream is None else stream)
        if st != 0:
            nat.check(st, "dcue_plan_launch")
        if self._check is not None:
            self._check_after()

    def step(self, users=None, item_track=None, stream=None):
        """One whole single-GPU training step in one host call: launch() + the optimizer step
        (NativeAdam semantics with the optimizer's current param_group lr / weight_decay)."""
        opt = self.optimizer
        if opt is None:
            raise RuntimeError("TrainPlan.step needs the plan built with optimizer=...")
        if not self._fused_adam:  # NativeSGD / NativeRanger: the replay, then their own sweep
            self.launch(users, item_track, stream)
            opt.step()
            return
        if self._handle is None:
            raise RuntimeError("TrainPlan was closed")
        self._check_bound()
        if self._check is not None:
            self._check_before(users, item_track)
        self._hold.append((users, item_track))
        g = opt.param_groups[0]
        opt.step_count += 1
        args = self._adam_args
        args.lr, (args.beta1, args.beta2) = g["lr"], g["betas"]
        args.eps, args.weight_decay, args.step, args.parts = g["eps"], g["weight_decay"], opt.step_count, 0
        st = self._lib.dcue_plan_step(self._handle, None if users is None else users.data_ptr(),
                                      None if item_track is None else item_track.data_ptr(),
                                      ctypes.byref(args), self._stream if stream is None else stream)
        if st != 0:
            nat.check(st, "dcue_plan_step")
        # the step's last Adam work may still run on the library's user stream (include/dcue.h
        # dcue_plan_step); the model joins it before anything reads the parameters from torch
        self.net._pending_plan = self
        if self._check is not None:
            self._check_after()

    def sync(self, stream=None):
        """`stream` (default: the plan's) waits for the work the last step left on the library's side
        streams (include/dcue.h dcue_plan_sync): the parameters are then current on it."""
        if self._handle is None:
            return
        nat.check(self._lib.dcue_plan_sync(self._handle, self._stream if stream is None else stream),
                  "dcue_plan_sync")

    def set_next(self, item_track):
        """Announce the NEXT launch's item_track source (device [M] int32, unchanged until that
        launch): this step then also prepares that batch's bn0 statistics and conv-1 wgrad input
        beside itself, off the next step's critical path (include/dcue.h dcue_plan_set_next).
        The items must already be written in this stream's order. Returns False where the plan
        cannot look ahead (graph or BatchNorm-free plans)."""
        if self._handle is None:
            raise RuntimeError("TrainPlan was closed")
        st = self._lib.dcue_plan_set_next(self._handle, None if item_track is None else item_track.data_ptr())
        if st == nat.ERR_UNSUPPORTED:
            return False
        nat.check(st, "dcue_plan_set_next")
        self._hold.append((None, item_track))
        return True

    def set_comm(self, comm):
        """Data parallelism inside step(): with a distributed.NativeComm bound, each step() also
        all-reduces the dense gradient over RCCL between the backward and Adam (two buckets, the
        larger overlapping the conv-1 weight gradient) and Adam averages it -- one host call per
        step, as on one GPU. launch() -- and so step() with NativeSGD / NativeRanger, which run
        their own sweep after it -- makes the same exchange and leaves the mean over the ranks in
        the gradient. Build the plan with emb_grad_scale = 1/world. None unbinds."""
        if self._handle is None:
            raise RuntimeError("TrainPlan was closed")
        nat.check(self._lib.dcue_plan_set_comm(self._handle, None if comm is None else comm.handle),
                  "dcue_plan_set_comm")
        self._comm = comm  # keep the communicator alive while bound

    def set_sync_bn(self, on=True):
        """SyncBN over the bound communicator's ranks (dcue_plan_set_sync_bn): every train-mode
        BatchNorm of the item tower normalises over the global batch -- torch's
        convert_sync_batchnorm + DDP semantics. Bind the communicator first (set_comm)."""
        if self._handle is None:
            raise RuntimeError("TrainPlan was closed")
        nat.check(self._lib.dcue_plan_set_sync_bn(self._handle, 1 if on else 0), "dcue_plan_set_sync_bn")

    def wait_side(self, stream):
        """`stream` (a torch.cuda.Stream or raw handle) waits until the side-stream part of the last
        launched step is in: the flat gradient is then final past its first SEG_LATE segments
        (include/dcue.h dcue_plan_wait_side)."""
        if self._handle is None:
            raise RuntimeError("TrainPlan was closed")
        h = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
        nat.check(self._lib.dcue_plan_wait_side(self._handle, h), "dcue_plan_wait_side")

    def probe_report(self):
        """check="probe" plans: the probes that saw a non-finite output so far, earliest first
        (dcrecommend.check.ProbeCheck.report); [] otherwise."""
        return self._probes.report() if getattr(self, "_probes", None) is not None else []

    def close(self):
        if getattr(self, "_handle", None) is not None:
            self.sync()
            torch.cuda.synchronize()
            if getattr(self.net, "_pending_plan", None) is self:
                self.net._pending_plan = None
            self._lib.dcue_plan_destroy(self._handle)
            self._handle = None
            if getattr(self, "_probes", None) is not None:
                probes, self._probes = self._probes, None
                probes.close()
                probes.raise_if_any()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
