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
    """DCUE_CHECK=1: per-step checks (they synchronise each step); DCUE_CHECK=probe: the in-stream
    probes only (ProbeCheck), which keep the step's concurrency."""
    v = os.environ.get("DCUE_CHECK", "0")
    if v == "probe":
        return "probe"
    return v not in ("", "0")


class ProbeCheck:
    """In-stream output probes (include/dcue.h dcue_debug_probes). While bound, every step checks the
    output of each probed launch on that launch's own stream -- no extra order between streams, so a
    race still shows -- and report() names, by the device's wall clock, the first launch that wrote a
    non-finite value. One binding per process."""

    def __init__(self, device):
        n = nat.lib().dcue_debug_probe_count()
        self.names = [nat.lib().dcue_debug_probe_name(i).decode() for i in range(n)]
        # records {u32 nonfinite, u32 nonzero, u64 first_bad}
        self.buf = torch.zeros((n, 2), dtype=torch.int64, device=device)
        self.reset()
        nat.check(nat.lib().dcue_debug_probes(nat.ptr(self.buf)), "dcue_debug_probes")

    def reset(self):
        self.buf[:, 0] = 0
        self.buf[:, 1] = -1  # UINT64_MAX

    def report(self):
        """[(name, first_bad_tick)] of the probes that saw a non-finite value, earliest first
        (synchronises), and the names of the probes whose output was zero everywhere."""
        torch.cuda.synchronize(self.buf.device)
        rec = self.buf.cpu()
        flags = rec[:, 0]
        bad = [(self.names[i], int(rec[i, 1]) & (2 ** 64 - 1)) for i in range(len(self.names))
               if int(flags[i]) & 0xFFFFFFFF]
        bad.sort(key=lambda x: x[1])
        return bad

    def raise_if_any(self):
        bad = self.report()
        if bad:
            self.reset()
            raise RuntimeError("DCUE probes: first non-finite output from %s (then: %s)"
                               % (bad[0][0], ", ".join(b[0] for b in bad[1:]) or "none"))

    def close(self):
        nat.check(nat.lib().dcue_debug_probes(None), "dcue_debug_probes")


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
