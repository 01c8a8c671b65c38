"""DCBR: the audio ConvNet regressing WRMF item factors (BASELINE config 5).

van den Oord, Dieleman, Schrauwen, "Deep content-based music recommendation" (NIPS 2013): latent
item factors from weighted matrix factorisation of the usage data (dcrecommend.dcbr.wrmf) are the
regression targets of a ConvNet over the item's mel-spectrogram, trained with the mean squared
error; at inference the ConvNet predicts factors for songs without usage data.

The ConvNet is this repository's DCUE item tower (any of the four wired model types, any width in
1..256) and the step is one C-ABI call, `dcue_dcbr_step` (capi.hip): the item tower's train
forward, the MSE head (tail.hip `k_mse_grad`) and the item tower's backward -- the same kernels as
the DCUE step, with the user tower and the scores left out. `NativeAdam` then steps the parameters.
The reference never published this path (`.gitignore:13`), so parity is unpinned against it; the
tests pin the step against the fp64 oracle item tower with an MSE head.
"""
import ctypes

import torch

from dcrecommend import _native as nat
from dcrecommend.dcue.dcue import DCUENet
from dcrecommend.optim.adam import NativeAdam


class DCBR:
    """Item-factor regression from audio. `step(tracks, item_track, target)` runs one Adam step on
    the batch's items (track ids into the HBM track table `tracks` [n, 131, 128] fp16/fp32) against
    `target` [M, feature_dim] factors and returns the batch loss (a device scalar)."""

    def __init__(self, feature_dim=128, conv_hidden=128, model_type="truedcuemel1dbn", lr=1e-3,
                 betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, device="cuda", comm=None):
        """comm (distributed.NativeComm / HostComm): data parallelism -- each rank steps its own item
        batches and the dense gradient is averaged over the ranks before Adam (DDP semantics,
        per-replica BatchNorm), so every rank keeps the same ConvNet."""
        self.comm = comm
        # the ConvNet is DCUENet's item tower; its user tower (one row) is carried but never used
        self.net = DCUENet({"feature_dim": feature_dim, "conv_hidden": conv_hidden, "user_embdim": 1,
                            "user_count": 1, "model_type": model_type}).to(device).train()
        self.opt = NativeAdam(self.net.parameters(), lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        self.feature_dim = feature_dim
        self._target = None

    def _padded_target(self, target, M):
        nat.require_gpu(target, "target")
        if target.dim() != 2 or tuple(target.shape) != (M, self.feature_dim):
            raise ValueError("target must be [%d, %d] (one row per item), got %s"
                             % (M, self.feature_dim, tuple(target.shape)))
        d = self.feature_dim
        ds = self.net._ds
        if self._target is None or self._target.shape[0] < M:
            self._target = torch.zeros((M, ds), dtype=torch.float32, device=target.device)
        t = self._target[:M]
        t[:, :d].copy_(target)
        return t

    def loss_and_grads(self, tracks, item_track, target):
        """Forward + MSE + backward (gradients in the model's .grad views); returns the loss."""
        net = self.net
        fl = net._require_device()
        nat.require_gpu(item_track, "item_track")
        item_track = item_track.to(torch.int32).contiguous()
        M = item_track.shape[0]
        tgt = self._padded_target(target.to(torch.float32), M)
        ws = net._workspace(M, 0, M)
        users = torch.zeros(M, dtype=torch.int64, device=item_track.device)
        batch = nat.Batch(M, 0, M, nat.LAYOUT_CATALOGUE, users.data_ptr(), item_track.data_ptr(), None)
        tr = nat.Tracks(tracks.data_ptr(), tracks.shape[0], 0 if tracks.dtype == torch.float16 else 1, 0)
        loss = torch.empty((), dtype=torch.float32, device=item_track.device)
        model = net._model_struct()
        nat.check(nat.lib().dcue_dcbr_step(ctypes.byref(model), ctypes.byref(batch), ctypes.byref(tr),
                                           nat.ptr(tgt), nat.ptr(loss), nat.ptr(ws), ws.numel(),
                                           nat.stream_handle()), "dcue_dcbr_step")
        net._expose_grads()
        del fl
        return loss

    def step(self, tracks, item_track, target):
        loss = self.loss_and_grads(tracks, item_track, target)
        if self.comm is not None and self.comm.world > 1:
            self.comm.allreduce_mean_(self.net._flat["G"])  # the DDP mean of the dense gradient
        self.opt.step()
        return loss

    @torch.no_grad()
    def predict(self, tracks, item_track):
        """Eval-mode item factors [M, feature_dim] (running BN statistics)."""
        nat.require_gpu(tracks, "tracks")
        nat.require_gpu(item_track, "item_track")
        self.net.eval()
        try:
            out = torch.empty((item_track.shape[0], self.net._ds), dtype=torch.float32, device=tracks.device)
            ws = self.net._workspace(1, 0, item_track.shape[0])
            tr = nat.Tracks(tracks.data_ptr(), tracks.shape[0], 0 if tracks.dtype == torch.float16 else 1, 0)
            it = item_track.to(torch.int32).contiguous()
            nat.check(nat.lib().dcue_item_tower_eval(ctypes.byref(self.net._model_struct()), ctypes.byref(tr),
                                                     nat.ptr(it), it.shape[0], nat.ptr(ws), ws.numel(),
                                                     nat.ptr(out), nat.stream_handle()), "dcue_item_tower_eval")
            return out[:, :self.feature_dim]
        finally:
            self.net.train()
