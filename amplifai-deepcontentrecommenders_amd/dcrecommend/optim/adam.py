"""torch.optim.Adam semantics executed by libdcue_hip (dcue_adam_step).

Drop-in for the optimizer the reference trainer builds (nn/dcue.py:143-147):
`NativeAdam(model.parameters(), lr, (beta_one, beta_two), eps, weight_decay)`. It is a
torch.optim.Optimizer (CyclicLRWithRestarts checks that and edits param_groups[*]['lr'] /
['weight_decay'] between steps, cyclic_scheduler.py:212-215), but `step()` is one HIP sweep over the
flat dense buffer plus one over the user table -- every user row moves every step, as the
reference's dense embedding gradient makes torch.optim.Adam do.

defer_embedding=True keeps those semantics bit for bit but performs the user table's zero-gradient
steps late (include/dcue.h, dcue_emb_log): the batch's rows step now, every other row replays its
missed steps right before a forward reads it and, for all rows, every `flush_every` steps and on
flush() / state_dict(). The table is then bit-identical to the dense sweep's; in between, read it
only through the model (forwards sync their users) or after model.sync_user_table().
"""
import ctypes
import weakref

import torch

from dcrecommend import _native as nat


class NativeAdam(torch.optim.Optimizer):

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0,
                 defer_embedding=False, flush_every=16):
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
        self.defer_embedding = bool(defer_embedding)
        if self.defer_embedding:
            if not 1 <= int(flush_every) <= nat.MAX_LOG_CAP:
                raise ValueError("flush_every must be in [1, %d]" % nat.MAX_LOG_CAP)
            self.flush_every = int(flush_every)
            self.net._deferred_opt = weakref.ref(self)

    def _adam_state(self):
        fl = self.net._flat
        if fl is None:
            self.net._require_device()  # raises: the model is not on the GPU
        emb = self.net.user_embd.embeddings.weight
        st = self._moments
        if st is None or st["m"].numel() != fl["P"].numel() or st["m"].device != fl["P"].device:
            st = dict(m=torch.zeros_like(fl["P"]), v=torch.zeros_like(fl["P"]),
                      em=torch.zeros_like(emb.data), ev=torch.zeros_like(emb.data),
                      emb_step=None, emb_log=None, cap=0)
            self._moments = st
            if self.defer_embedding:
                self._init_log(st)
        return st

    def _init_log(self, st):
        """Fresh deferred-Adam log: every row current at the present step count."""
        dev = st["m"].device
        # buffers are reused when present: plans (dcrecommend.dcue.plan) bind their addresses
        if st.get("emb_step") is None:
            st["emb_step"] = torch.zeros(max(self.net.user_count, 1), dtype=torch.int32, device=dev)
            st["emb_log"] = torch.zeros(nat.emb_log_bytes(self.flush_every), dtype=torch.uint8, device=dev)
        st["cap"] = self.flush_every
        nat.check(nat.lib().dcue_emb_log_init(ctypes.byref(self.net._model_struct(st)), self.flush_every,
                                              self.step_count, nat.stream_handle()), "dcue_emb_log_init")

    def flush(self):
        """Apply every deferred user-table step now (no-op in dense mode)."""
        if not self.defer_embedding or self._moments is None:
            return
        st = self._adam_state()
        nat.check(nat.lib().dcue_embedding_flush(ctypes.byref(self.net._model_struct(st)), nat.stream_handle()),
                  "dcue_embedding_flush")

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
        fl = self.net._flat
        if fl["emb_grad"].numel() == 0:
            # no backward ran yet (e.g. a resumed optimizer): every row takes the zero-gradient step
            self.net._workspace(1, 0, 1)
        # the ctypes model struct is rebuilt only when a bound buffer changed (host cost per step)
        key = (fl, fl["emb_grad"], st, self.net.user_embd.embeddings.weight.data_ptr())
        cache = getattr(self, "_model_cache", None)
        if cache is None or any(a is not b for a, b in zip(cache[0][:3], key[:3])) or cache[0][3] != key[3]:
            cache = (key, self.net._model_struct(st))
            self._model_cache = cache
        nat.check(nat.lib().dcue_adam_step(ctypes.byref(cache[1]), ctypes.byref(args), nat.stream_handle()),
                  "dcue_adam_step")
        return loss

    def state_dict(self):
        self.flush()
        sd = super().state_dict()
        moments = None
        if self._moments is not None:
            moments = {k: self._moments[k] for k in ("m", "v", "em", "ev")}
        sd["native"] = dict(step=self.step_count, moments=moments)
        return sd

    def load_state_dict(self, state_dict):
        native = state_dict.get("native")
        base = {k: v for k, v in state_dict.items() if k != "native"}
        super().load_state_dict(base)
        if native is not None:
            self.step_count = native["step"]
            if native["moments"] is not None:
                st = self._adam_state()
                for k in ("m", "v", "em", "ev"):
                    st[k].copy_(native["moments"][k])
            if self.defer_embedding and self._moments is not None:
                self._init_log(self._moments)  # the loaded table is current at the loaded step
