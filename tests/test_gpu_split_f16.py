"""Precision of the split-f16 conv forwards against the exact-f32 path.

The forward convs multiply f32 values as fp16 pairs (hi + lo) on f16 MFMA; DCUE_CONV_F16=0 selects
the f32-MFMA path of the same kernels. The switch is read once per process, so each path runs in
its own child process on the same seeded model and inputs: the catalogue layout at the bench shape
(B=64, N=20, M=1,344 distinct items, d=H=128), train mode (BatchNorm batch statistics) and eval mode
(running statistics). The two paths' scores, loss and item features must agree within 2e-5 of the
output's max magnitude -- five times inside north_star's 1e-4 -- with the observed gap printed. The
reference-parity tests (goldens, fp64 oracle at the bench shape) run on the split path already.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, numpy as np, torch
sys.path[:0] = [sys.argv[1], sys.argv[1] + "/amplifai-deepcontentrecommenders_amd"]
from dcrecommend import _native as nat
from dcrecommend.dcue.dcue import DCUENet
DEV = "cuda:0"
B, N, NU, NT = 64, 20, 500, 3000
torch.manual_seed(0)
net = DCUENet({"feature_dim": 128, "conv_hidden": 128, "user_embdim": 300, "user_count": NU,
               "model_type": "truedcuemel1dbn"}).to(DEV)
g = torch.Generator(device=DEV).manual_seed(3)
tracks = (torch.randn((NT, 131, 128), generator=g, device=DEV) * 2.0 - 1.0).half()
ids = torch.randperm(NT, generator=g, device=DEV)[:B * (1 + N)].to(torch.int32)
users = torch.randint(0, NU, (B,), generator=g, device=DEV)
out = {}
for train in (True, False):
    net.train(train)
    s, uf, f, loss = net.native_forward(users, tracks, ids, N, nat.LAYOUT_CATALOGUE, train=train)
    torch.cuda.synchronize()
    for k, v in (("scores", s), ("feat", f), ("loss", loss)):
        out["%s_%d" % (k, train)] = v.detach().double().cpu().numpy()
np.savez(sys.argv[2], **out)
"""


def _run(path, f16, tmp):
    env = dict(os.environ, DCUE_CONV_F16="1" if f16 else "0")
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT, path], env=env, capture_output=True, text=True,
                       timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    return np.load(path)


def test_split_f16_forward_matches_f32_path(tmp_path):
    a = _run(str(tmp_path / "f16.npz"), True, tmp_path)
    b = _run(str(tmp_path / "f32.npz"), False, tmp_path)
    gaps = {}
    for k in b.files:
        ref = b[k]
        scale = max(float(np.abs(ref).max()), 1e-30)
        gaps[k] = float(np.abs(a[k] - ref).max()) / scale
    print("split-f16 vs f32 (max |diff| / max |f32|):", json.dumps(gaps))
    for k, gap in gaps.items():
        assert gap <= 2e-5, "%s: split-f16 differs from the f32 path by %.3e of its max" % (k, gap)
    assert any(gap > 0 for gap in gaps.values()), "the two paths are identical: DCUE_CONV_F16 not honoured"
