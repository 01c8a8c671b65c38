"""Check mode: bounds and finiteness probes around training steps (the reference has
none). Probes run on the GPU (include/dcue.h dcue_check_*), OR a bit per finding into one device
word, and never fault on what they inspect; `raise_if_any` synchronises and raises naming what
failed. TrainPlan(check=True) -- or DCUE_CHECK=1 in the environment -- validates each step's user
and item ids before it is launched and its loss and dense parameters/gradients after it.
"""
import os

import torch

from dcrecommend import _native as nat


def enabled_by_env():
    return os.environ.get("DCUE_CHECK", "0") not in ("", "0")


class StepCheck:

    def __init__(self, device):
        self.flags = torch.zeros(1, dtype=torch.int32, device=device)
        self.names = []

    def _bit(self, what):
        if what not in self.names:
            if len(self.names) >= 31:
                raise RuntimeError("StepCheck: too many distinct probes")
            self.names.append(what)
        return 1 << self.names.index(what)

    def finite(self, t, what):
        """Flag `what` if the float32 tensor t holds a NaN or an infinity."""
        t = t.detach()
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError("finite(): contiguous float32 tensors only")
        nat.check(nat.lib().dcue_check_finite(nat.ptr(t), t.numel(), nat.ptr(self.flags), self._bit(what),
                                              nat.stream_handle(t.device)), "dcue_check_finite")

    def ids(self, t, limit, what):
        """Flag `what` if an id of the int32/int64 tensor t lies outside [0, limit)."""
        if t.dtype not in (torch.int32, torch.int64) or not t.is_contiguous():
            raise ValueError("ids(): contiguous int32/int64 tensors only")
        nat.check(nat.lib().dcue_check_ids(nat.ptr(t), t.element_size(), t.numel(), int(limit), nat.ptr(self.flags),
                                           self._bit(what), nat.stream_handle(t.device)), "dcue_check_ids")

    def failed(self):
        """Names of the probes that fired so far (synchronises)."""
        v = int(self.flags.item())
        return [n for i, n in enumerate(self.names) if v >> i & 1]

    def raise_if_any(self):
        bad = self.failed()
        if bad:
            self.flags.zero_()
            raise RuntimeError("DCUE check mode: " + ", ".join(bad))
