"""torch.optim.Adam semantics executed by libdcue_hip (dcue_adam_step).

Drop-in for the optimizer the reference trainer builds (nn/dcue.py:143-147):
`NativeAdam(model.parameters(), lr, (beta_one, beta_two), eps, weight_decay)`. It is a
torch.optim.Optimizer (CyclicLRWithRestarts checks that and edits param_groups[*]['lr'] /
['weight_decay'] between steps, cyclic_scheduler.py:212-215), but `step()` is one HIP sweep over the
flat dense buffer plus one over the user table -- every user row moves every step, as the
reference's dense embedding gradient makes torch.optim.Adam do.
"""
import ctypes

import torch

from dcrecommend import _native as nat


class NativeAdam(torch.optim.Optimizer):

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0):
        params = list(params)
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        owners = {}
        for p in params:
            ref = getattr(p, "_dcue_owner", None)
            if ref is not None and ref() is not None:
                owners[id(ref())] = ref()
        if len(owners) != 1:
            raise ValueError("NativeAdam steps the parameters of exactly one GPU-resident DCUENet "
                             "(call model.cuda() before building the optimizer)")
        self.net = next(iter(owners.values()))
        names = {id(p) for p in self.net.parameters()}
        if {id(p) for p in params} != names:
            raise ValueError("NativeAdam needs all of the model's parameters in its single group")
        self.step_count = 0
        self._moments = None

    def _adam_state(self):
        fl = self.net._require_device()
        emb = self.net.user_embd.embeddings.weight
        st = self._moments
        if st is None or st["m"].numel() != fl["P"].numel() or st["m"].device != fl["P"].device:
            st = dict(m=torch.zeros_like(fl["P"]), v=torch.zeros_like(fl["P"]),
                      em=torch.zeros_like(emb.data), ev=torch.zeros_like(emb.data))
            self._moments = st
        return st

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if len(self.param_groups) != 1:
            raise ValueError("NativeAdam supports one parameter group (the reference uses one)")
        g = self.param_groups[0]
        st = self._adam_state()
        self.step_count += 1
        args = nat.AdamArgs(float(g["lr"]), float(g["betas"][0]), float(g["betas"][1]), float(g["eps"]),
                            float(g["weight_decay"]), self.step_count, 0)
        model = self.net._model_struct(st)
        if not model.emb_grad:
            # no backward ran yet (e.g. a resumed optimizer): every row takes the zero-gradient step
            self.net._workspace(1, 0, 1)
            model = self.net._model_struct(st)
        nat.check(nat.lib().dcue_adam_step(ctypes.byref(model), ctypes.byref(args), nat.stream_handle()),
                  "dcue_adam_step")
        return loss

    def state_dict(self):
        sd = super().state_dict()
        sd["native"] = dict(step=self.step_count, moments=self._moments)
        return sd

    def load_state_dict(self, state_dict):
        native = state_dict.get("native")
        base = {k: v for k, v in state_dict.items() if k != "native"}
        super().load_state_dict(base)
        if native is not None:
            self.step_count = native["step"]
            if native["moments"] is not None:
                st = self._adam_state()
                for k in st:
                    st[k].copy_(native["moments"][k])
