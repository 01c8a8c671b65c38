"""The trainer's other optimizers executed by libdcue_hip (dcue_optimizer_step).

DCUE(optimize='sgd') builds torch.optim.SGD(params, lr, beta_one, weight_decay=wd, nesterov=True)
and optimize='ranger' the reference's Ranger(params, lr, alpha=0.5, k=6, N_sma_threshhold=5,
betas=(beta_one, beta_two), eps=1e-5, weight_decay=wd) (nn/dcue.py:148-157, optim/ranger.py:26-165).
NativeSGD / NativeRanger take the same arguments and are torch.optim.Optimizers, so
CyclicLRWithRestarts drives their param_group lr / weight_decay unchanged; step() is one HIP sweep
over the flat dense buffer and one over the user table (the dense embedding gradient: every row
steps every step, as the reference's torch optimizers do).
"""
import ctypes

import torch

from dcrecommend import _native as nat


class _NativeOptimizer(torch.optim.Optimizer):
    KIND = None
    BUFFERS = ()          # state buffers (dense, embedding) per letter
    COPY_PARAMS = ()      # buffers that start as copies of the parameters (lookahead weights)

    def __init__(self, params, defaults):
        params = list(params)
        super().__init__(params, defaults)
        owners = {}
        for p in params:
            ref = getattr(p, "_dcue_owner", None)
            if ref is not None and ref() is not None:
                owners[id(ref())] = ref()
        if len(owners) != 1:
            raise ValueError("%s steps the parameters of exactly one GPU-resident DCUENet (call model.cuda() "
                             "before building the optimizer)" % type(self).__name__)
        self.net = next(iter(owners.values()))
        if {id(p) for p in params} != {id(p) for p in self.net.parameters()}:
            raise ValueError("%s needs all of the model's parameters in its single group" % type(self).__name__)
        self.step_count = 0
        self._moments = None

    def _buffers(self):
        fl = self.net._flat
        if fl is None:
            self.net._require_device()
        emb = self.net.user_embd.embeddings.weight
        st = self._moments
        if st is None or st[self.BUFFERS[0]].device != fl["P"].device:
            st = {}
            for b in self.BUFFERS:
                src_d, src_e = fl["P"], emb.data
                st[b] = src_d.detach().clone() if b in self.COPY_PARAMS else torch.zeros_like(src_d)
                st["e" + b] = src_e.detach().clone() if b in self.COPY_PARAMS else torch.zeros_like(src_e)
            self._moments = st
        return st

    def _args(self, g):
        raise NotImplementedError

    def flush(self):  # API parity with NativeAdam (nothing is deferred here)
        return None

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if len(self.param_groups) != 1:
            raise ValueError("%s supports one parameter group (the reference uses one)" % type(self).__name__)
        st = self._buffers()
        self.step_count += 1
        fl = self.net._flat
        if fl["emb_grad"].numel() == 0:
            self.net._workspace(1, 0, 1)  # no backward yet: every row takes the zero-gradient step
        ptr = {b: st[b].data_ptr() for b in st}
        state = nat.OptState(*[ptr.get(k) for k in ("a", "b", "c", "ea", "eb", "ec")])
        args = self._args(self.param_groups[0])
        nat.check(nat.lib().dcue_optimizer_step(ctypes.byref(self.net._model_struct()), ctypes.byref(args),
                                                ctypes.byref(state), nat.stream_handle()), "dcue_optimizer_step")
        return loss

    def state_dict(self):
        sd = super().state_dict()
        sd["native"] = dict(step=self.step_count, moments=None if self._moments is None else dict(self._moments))
        return sd

    def load_state_dict(self, state_dict):
        native = state_dict.get("native")
        super().load_state_dict({k: v for k, v in state_dict.items() if k != "native"})
        if native is not None:
            self.step_count = native["step"]
            if native["moments"] is not None:
                st = self._buffers()
                for k, v in native["moments"].items():
                    st[k].copy_(v)


class NativeSGD(_NativeOptimizer):
    """torch.optim.SGD(params, lr, momentum, weight_decay=wd, nesterov=True) (nn/dcue.py:149-151)."""
    KIND = nat.OPT_SGD
    BUFFERS = ("a",)

    def __init__(self, params, lr, momentum=0, dampening=0, weight_decay=0, nesterov=False):
        if not nesterov or dampening != 0 or momentum <= 0:
            raise ValueError("NativeSGD implements the trainer's SGD: momentum > 0, dampening 0, nesterov=True")
        super().__init__(params, dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                                      nesterov=nesterov))

    def _args(self, g):
        return nat.OptArgs(nat.OPT_SGD, self.step_count, float(g["lr"]), float(g["momentum"]), 0.0, 0.0,
                           float(g["weight_decay"]), 0.0, 1, 0, 0.0, 0.0)


class NativeRanger(_NativeOptimizer):
    """The reference's Ranger (optim/ranger.py:26-165): RAdam + Lookahead, same arguments."""
    KIND = nat.OPT_RANGER
    BUFFERS = ("a", "b", "c")
    COPY_PARAMS = ("c",)

    def __init__(self, params, lr=1e-3, alpha=0.5, k=6, N_sma_threshhold=5, betas=(.95, 0.999), eps=1e-5,
                 weight_decay=0):
        # the reference's parameter checks (optim/ranger.py:30-37)
        if not 0.0 <= alpha <= 1.0:
            raise ValueError(f'Invalid slow update rate: {alpha}')
        if not 1 <= k:
            raise ValueError(f'Invalid lookahead steps: {k}')
        if not lr > 0:
            raise ValueError(f'Invalid Learning Rate: {lr}')
        if not eps > 0:
            raise ValueError(f'Invalid eps: {eps}')
        super().__init__(params, dict(lr=lr, alpha=alpha, k=k, step_counter=0, betas=betas,
                                      N_sma_threshhold=N_sma_threshhold, eps=eps, weight_decay=weight_decay))
        self.N_sma_threshhold = N_sma_threshhold
        self.alpha = alpha
        self.k = k

    def _args(self, g):
        b1, b2 = g["betas"]
        return nat.OptArgs(nat.OPT_RANGER, self.step_count, float(g["lr"]), float(b1), float(b2), float(g["eps"]),
                           float(g["weight_decay"]), float(self.alpha), int(g["k"]), 0, float(self.N_sma_threshhold),
                           0.0)
