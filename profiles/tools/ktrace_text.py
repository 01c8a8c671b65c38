"""Per-workgroup phase timing of the config-4 text forward (k_text_fwd_full) at the bench's text shape
(diagnostic). DCUE_HIP_LIB=<ktrace build>/libdcue_hip.so python profiles/tools/ktrace_text.py
(after profiles/tools/build_ktrace.sh <dir>); DCUE_TEXT_FWD selects the shape as in the library."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "amplifai-deepcontentrecommenders_amd"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dcrecommend import _native as nat  # noqa: E402
from dcrecommend.dcue.dcue import DCUENet  # noqa: E402
from dcrecommend.dcue.plan import TrainPlan  # noqa: E402
from dcrecommend.optim import NativeAdam  # noqa: E402
from bench import synthetic_sentences  # noqa: E402

dev = "cuda:0"
B, N, n_users, n_tracks, T, V = 64, 20, 5000, 8000, 64, 20000
torch.manual_seed(0)
net = DCUENet({"feature_dim": 256, "conv_hidden": 128, "user_embdim": 300, "user_count": n_users,
               "model_type": "truedcuemel1dbntext", "text_dim": 256, "word_dim": 300, "text_len": T,
               "n_words": V, "pad_idx": 0}).to(dev).train()
gen = torch.Generator(device=dev).manual_seed(1)
with torch.no_grad():
    net.text.embeddings.weight.copy_(torch.randn(V, 300, generator=gen, device=dev) * 0.3)
opt = NativeAdam(net.parameters(), 1e-5, (0.9, 0.99), 1e-8, 0, defer_embedding=True, flush_every=12)
table = torch.randn(n_tracks, 131, 128, generator=gen, device=dev).half()
tokens = synthetic_sentences(n_tracks, T, V, dev, seed=77)
mt = torch.empty(nat.MT_STATE_BYTES, dtype=torch.uint8, device=dev)
nat.check(nat.lib().dcue_mt_seed(nat.ptr(mt), 7, nat.stream_handle()), "mt_seed")
plan = TrainPlan(net, table, B, N, mt_state=mt, optimizer=opt, tokens=tokens)
users = torch.randint(0, n_users, (40, B), generator=gen, device=dev)
items = torch.randint(0, n_tracks, (40, B), generator=gen, device=dev).to(torch.int32)
fn = nat.lib().dcue_ktrace_read_text
fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
buf = np.zeros((16, 512, 8), dtype=np.uint64)
labels = ["tokens", "sentence gather", "MFMA loop", "epilogue"]
for s_ in range(40):
    plan.set_next(items[(s_ + 1) % 40])
    plan.step(users[s_], items[s_])
    if s_ >= 36:
        torch.cuda.synchronize()
        assert fn(buf.ctypes.data, buf.nbytes) == 0
        t = buf[0].astype(np.int64)
        t = t[t[:, 6] > 0]
        t = t[t[:, 6] >= t[:, 6].max() - 100000]
        w = t[:, 7] - t[:, 6]
        ok = w > 0
        wall = w[ok] * 10 / 1000.0
        span = (t[ok, 7].max() - t[:, 6].min()) * 10 / 1000.0
        spread = (t[:, 6].max() - t[:, 6].min()) * 10 / 1000.0
        ph = np.diff(t[ok, :5], axis=1)
        cyc = np.median((t[ok, 4] - t[ok, 0]) / np.maximum(wall, 1e-3))
        print("step %d k_text_fwd_full WGs %4d span %5.1f us, WG wall med %5.1f max %5.1f, start spread %4.1f; %s"
              % (s_, len(t), span, np.median(wall), wall.max(), spread,
                 ", ".join("%s %.2f/%.2f" % (l, np.median(ph[:, i]) / cyc, ph[:, i].max() / cyc)
                           for i, l in enumerate(labels))), flush=True)
        # kernel 1: k_text_wgrad (slots by blockIdx.x only: one sample per o block)
        t = buf[1].astype(np.int64)
        t = t[t[:, 6] > 0]
        if len(t):
            t = t[t[:, 6] >= t[:, 6].max() - 100000]
            w = t[:, 7] - t[:, 6]
            ok = w > 0
            wall = w[ok] * 10 / 1000.0
            ph = np.diff(t[ok, :4], axis=1)
            cyc = np.median((t[ok, 3] - t[ok, 0]) / np.maximum(wall, 1e-3))
            print("step %d k_text_wgrad WGs(sampled) %4d WG wall med %5.1f max %5.1f; %s" % (
                s_, len(t), np.median(wall), wall.max(),
                ", ".join("%s %.2f/%.2f" % (l, np.median(ph[:, i]) / cyc, ph[:, i].max() / cyc) for i, l in
                          enumerate(["stage tokens + routing", "items (word loads + FMAs)", "stores"]))), flush=True)
plan.close()
