"""Per-phase cycles of the fp64-MFMA WRMF solve (k_wrmf_solve_mfma) at the bench's DCBR shape
(diagnostic). DCUE_HIP_LIB=<ktrace build>/libdcue_hip.so python profiles/tools/ktrace_wrmf.py
(after profiles/tools/build_ktrace.sh <dir>); DCUE_WRMF_LOWRANK / DCUE_WRMF_PHASES select the variant as
in the library. Prints, per half-step and solve kernel (the Cholesky, k_wrmf_solve_mfma, and the
Woodbury path, k_wrmf_solve_lowrank), one thread of wave 0 and of wave 1: cycles per row in each
phase (a kernel's counters are left from its last launch: a half-step without rows for it repeats
the previous numbers)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "amplifai-deepcontentrecommenders_amd"))
from dcrecommend import _native as nat  # noqa: E402
from dcrecommend.dcbr import WRMF  # noqa: E402

dev = "cuda:0"
n_users, n_tracks, nnz, d = 100_000, 200_000, 5_000_000, 128
gen = torch.Generator(device=dev).manual_seed(100)
pu = torch.randint(0, n_users, (nnz,), generator=gen, device=dev)
pt = torch.randint(0, n_tracks, (nnz,), generator=gen, device=dev, dtype=torch.int64)
w = WRMF(factors=d, regularization=0.1, alpha=40.0, iterations=1, seed=0, device=dev)
w.fit(pu, pt, None, n_users=n_users, n_items=n_tracks)
fn = nat.lib().dcue_ktrace_read_wrmf
fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
buf = np.zeros((16, 512, 8), dtype=np.uint64)
labels = ["G", "accumulate", "diag", "barriers", "panel", "trailing", "backsub+store"]
low_labels = ["staging", "P", "b+S+Pb", "S store", "Gauss-Jordan", "x", "skipped rows"]
for name, args in (("users", (w.user_factors, w.item_factors, w.by_user)),
                   ("items", (w.item_factors, w.user_factors, w.by_item))):
    torch.cuda.synchronize()
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    w.half_step(*args)
    t1.record()
    torch.cuda.synchronize()
    assert fn(buf.ctypes.data, buf.nbytes) == 0
    for kern, base, labs in (("k_wrmf_solve_mfma", 0, labels), ("k_wrmf_solve_lowrank", 2, low_labels)):
        for wv in (0, 1):
            b = buf[base + wv].astype(np.float64)
            rows = max(1.0, b[:, 7].sum())
            tot = b[:, :7].sum()
            print("%s %.2f ms %s wave %d: %.0f rows over 512 traced blocks, %.0f cycles/row: %s" % (
                name, t0.elapsed_time(t1), kern, wv, rows, tot / rows,
                ", ".join("%s %.0f" % (l, b[:, i].sum() / rows) for i, l in enumerate(labs))), flush=True)
        buf[base:base + 2] = 0
