"""Per-workgroup phase timing of the score, item-gradient and conv row-GEMM kernels at the bench's in-batch
shape (diagnostic).
DCUE_HIP_LIB=scratch/ktrace/libdcue_hip.so python profiles/tools/ktrace.py (after profiles/tools/build_ktrace.sh)"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "amplifai-deepcontentrecommenders_amd"))
from dcrecommend import _native as nat  # noqa: E402
from dcrecommend.dcue.dcue import DCUENet  # noqa: E402
from dcrecommend.dcue.plan import TrainPlan  # noqa: E402
from dcrecommend.optim import NativeAdam  # noqa: E402

dev = "cuda:0"
B, N, n_tracks = 64, 20, 8000
n_users = int(os.environ.get("KT_USERS", "5000"))
n_steps = int(os.environ.get("KT_STEPS", "40"))  # (more steps: the user table's replays reach steady state)
torch.manual_seed(0)
net = DCUENet({"feature_dim": 128, "conv_hidden": 128, "user_embdim": 300, "user_count": n_users,
               "model_type": "truedcuemel1dbn"}).to(dev).train()
opt = NativeAdam(net.parameters(), 1e-4, (0.9, 0.99), 1e-8, 0, defer_embedding=True, flush_every=12)
gen = torch.Generator(device=dev).manual_seed(1)
table = torch.randn(n_tracks, 131, 128, generator=gen, device=dev).half()
mt = torch.empty(nat.MT_STATE_BYTES, dtype=torch.uint8, device=dev)
nat.check(nat.lib().dcue_mt_seed(nat.ptr(mt), 7, nat.stream_handle()), "mt_seed")
plan = TrainPlan(net, table, B, N, mt_state=mt, optimizer=opt)
users = torch.randint(0, n_users, (n_steps, B), generator=gen, device=dev)
items = torch.randint(0, n_tracks, (n_steps, B), generator=gen, device=dev).to(torch.int32)
lib = nat.lib()
KK, KB = 16, 512
readers = {}
for n in ("tail", "fwd", "dgrad", "wgrad", "adam"):
    fn = getattr(lib, "dcue_ktrace_read_" + n)
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    readers[n] = fn
bufs = {n: np.zeros((KK, KB, 8), dtype=np.uint64) for n in readers}
KERNELS = [("tail", 0, "k_score_fused", ["ids+f+u loads, |u|", "cosines", "sync+hinge", "backward", "dU"], [0, 2, 1, 3, 4, 5]),
           ("tail", 1, "k_item_grad_multi", ["W stage", "copy sums", "dfmax+sync+GEMV", "sync", "acc atomics"], [0, 1, 2, 3, 4, 5])]
for kid, nm in zip(range(2, 7), ["fwd L1", "fwd L2", "fwd L3", "fwd L4", "fwd L5"]):
    KERNELS.append(("fwd", kid, "k_conv_rows " + nm, ["chan+range setup", "slab stores", "barrier", "MFMA", "epilogue"], [0, 5, 1, 2, 3, 4]))
for kid, nm in zip(range(7, 12), ["dgrad in L1?", "dgrad l=2 (in 32)", "dgrad l=3 (in 8)", "dgrad l=4 (in 2)", "dgrad l=5 (in 1)"]):
    KERNELS.append(("dgrad", kid, "k_conv_rows " + nm, ["chan+range setup", "slab stores", "barrier", "MFMA", "epilogue"], [0, 5, 1, 2, 3, 4]))
KERNELS.append(("wgrad", 0, "k_conv_wgrad1k conv 1" if os.environ.get("DCUE_W1K", "0") == "1" else "k_conv_wgrad16t conv 1", ["prologue consts", "first stage fill", "stages (MFMA)", "partial stores"], [0, 1, 2, 3, 4]))
KERNELS.append(("adam", 0, "k_user_fwd", ["claims + history", "replay", "release + waits", "GEMM 1", "GEMM 2 + signal"], [0, 1, 2, 3, 4, 5]))
KERNELS.append(("wgrad", 1, "k_conv_wgrad16t layer 2", ["prologue consts", "first stage fill", "stages (MFMA)", "partial stores"], [0, 1, 2, 3, 4]))
for s_ in range(n_steps):
    plan.set_next(items[(s_ + 1) % n_steps])
    plan.step(users[s_], items[s_])
    if s_ >= n_steps - 3:
        torch.cuda.synchronize()
        for n, fn in readers.items():
            assert fn(bufs[n].ctypes.data, bufs[n].nbytes) == 0
        for src, kid, name, labels, order in KERNELS:
            t = bufs[src][kid].astype(np.int64)
            live = t[:, 6] > 0
            if not live.any():
                continue
            t = t[live]
            t = t[t[:, 6] >= t[:, 6].max() - 100000]  # this step's launch (within 1 ms)
            t = np.concatenate([t[:, order], t[:, 6:8]], axis=1)
            w = t[:, -1] - t[:, -2]
            ok = w > 0
            wall = w[ok] * 10 / 1000.0
            span = (t[ok, -1].max() - t[:, -2].min()) * 10 / 1000.0
            spread = (t[:, -2].max() - t[:, -2].min()) * 10 / 1000.0
            ph = np.diff(t[ok, :len(order)], axis=1)
            cyc = np.median((t[ok, len(order) - 1] - t[ok, 0]) / np.maximum(wall, 1e-3))
            print("step %d %-26s WGs %4d span %5.1f us, WG wall med %5.1f max %5.1f, start spread %4.1f; %s" % (
                s_, name, len(t), span, np.median(wall), wall.max(), spread,
                ", ".join("%s %.2f/%.2f" % (l, np.median(ph[:, i]) / cyc, ph[:, i].max() / cyc) for i, l in enumerate(labels))))
plan.close()
