"""Cosine LR with warm restarts and weight-decay normalisation (AdamW paper, arXiv 1711.05101).

Host-side scalar schedule of the reference trainer, same constructor and stepping protocol as
dcrecommend/optim/cyclic_scheduler.py:49-215 (`step()` once per sub-epoch, `batch_step()` after
every optimizer step; StopIteration when more batches run than `epoch_size` announced). It edits
`param_groups[*]['lr']` and `['weight_decay']`, which NativeAdam passes to the HIP Adam sweep as
kernel arguments. Policies: cosine, arccosine, triangular, triangular2, exp_range.
"""
import math

import torch
from torch.optim import Optimizer


def _cosine(t_cur, period):
    return 0.5 * (1.0 + math.cos(math.pi * (t_cur / period)))


def _arccosine(t_cur, period):
    return math.acos(max(-1, min(1, 2 * t_cur / period - 1))) / math.pi


def _triangular(step):
    def f(t_cur, period):
        knee = step * period
        if t_cur < knee:
            return t_cur / knee
        return 1.0 - (t_cur - knee) / (period - knee)
    return f


class CyclicLRWithRestarts(object):
    """Per-batch cyclic schedule; see module docstring for the protocol."""

    def __init__(self, optimizer, batch_size, epoch_size, restart_period=100, t_mult=2,
                 last_epoch=-1, verbose=False, policy="cosine", policy_fn=None, min_lr=1e-7,
                 eta_on_restart_cb=None, eta_on_iteration_cb=None, gamma=1.0, triangular_step=0.5):
        if not isinstance(optimizer, Optimizer):
            raise TypeError("{} is not an Optimizer".format(type(optimizer).__name__))
        self.optimizer = optimizer
        for i, group in enumerate(optimizer.param_groups):
            if last_epoch == -1:
                group.setdefault("initial_lr", group["lr"])
                group.setdefault("minimum_lr", min_lr)
            elif "initial_lr" not in group:
                raise KeyError("param 'initial_lr' is not specified in param_groups[{}] when resuming "
                               "an optimizer".format(i))
        self.base_lrs = [g["initial_lr"] for g in optimizer.param_groups]
        self.min_lrs = [g["minimum_lr"] for g in optimizer.param_groups]
        self.base_weight_decays = [g["weight_decay"] for g in optimizer.param_groups]

        self.policy = policy
        self.eta_on_restart_cb = eta_on_restart_cb
        self.eta_on_iteration_cb = eta_on_iteration_cb
        if policy_fn is not None:
            self.policy_fn = policy_fn
        elif policy == "cosine":
            self.policy_fn = _cosine
        elif policy == "arccosine":
            self.policy_fn = _arccosine
        elif policy in ("triangular", "triangular2", "exp_range"):
            self.policy_fn = _triangular(triangular_step)
            if policy == "triangular2":
                self.eta_on_restart_cb = lambda lo, hi: (lo, hi * 0.5)
            elif policy == "exp_range":
                self.eta_on_iteration_cb = lambda lo, hi, it: (lo, hi * gamma ** it)

        self.last_epoch = last_epoch
        self.batch_size = batch_size
        self.epoch_size = epoch_size
        self.iteration = 0
        self.total_iterations = 0
        self.t_mult = t_mult
        self.verbose = verbose
        self.restart_period = math.ceil(restart_period)
        self.restarts = 0
        self.t_epoch = -1
        self.epoch = -1
        self.eta_min, self.eta_max = 0, 1
        self.end_of_period = False
        self.batch_increments = []
        self._reset_increments()

    def _reset_increments(self):
        full, rem = divmod(self.epoch_size, self.batch_size)
        # one increment per batch plus the closing one (and one more for a partial batch); the
        # reference builds these with torch.linspace in fp32, so the same call is used here
        n = full + (2 if rem > 0 else 1)
        self.iteration = 0
        self.batch_increments = torch.linspace(0, 1, n).tolist()

    def get_lr(self, t_cur):
        eta = self.eta_min + (self.eta_max - self.eta_min) * self.policy_fn(t_cur, self.restart_period)
        wd_norm = math.sqrt(self.batch_size / (self.epoch_size * self.restart_period))
        lrs = [lo + (hi - lo) * eta for hi, lo in zip(self.base_lrs, self.min_lrs)]
        wds = [w * eta * wd_norm for w in self.base_weight_decays]
        if (self.t_epoch + 1) % self.restart_period < self.t_epoch:
            self.end_of_period = True
        if self.t_epoch % self.restart_period < self.t_epoch:
            if self.verbose:
                print("Restart {} at epoch {}".format(self.restarts + 1, self.last_epoch))
            self.restart_period = math.ceil(self.restart_period * self.t_mult)
            self.restarts += 1
            self.t_epoch = 0
            if self.eta_on_restart_cb is not None:
                self.eta_min, self.eta_max = self.eta_on_restart_cb(self.eta_min, self.eta_max)
            self.end_of_period = False
        return zip(lrs, wds)

    def step(self):
        self.last_epoch += 1
        self.t_epoch += 1
        self._reset_increments()
        self.batch_step()

    def batch_step(self):
        if self.iteration >= len(self.batch_increments):
            raise StopIteration("Epoch size and batch size used in the training loop and while "
                                "initializing scheduler should be the same.")
        t_cur = self.t_epoch + self.batch_increments[self.iteration]
        if self.eta_on_iteration_cb is not None:
            self.eta_min, self.eta_max = self.eta_on_iteration_cb(self.eta_min, self.eta_max,
                                                                  self.total_iterations)
        self.iteration += 1
        self.total_iterations += 1
        for group, (lr, wd) in zip(self.optimizer.param_groups, self.get_lr(t_cur)):
            group["lr"] = lr
            group["weight_decay"] = wd

    def state_dict(self):
        return {k: v for k, v in self.__dict__.items() if k not in ("optimizer", "policy_fn",
                                                                      "eta_on_restart_cb",
                                                                      "eta_on_iteration_cb")}

    def load_state_dict(self, state_dict):
        self.__dict__.update(state_dict)
