"""CPU-side checks of the HIP library and the host mirror: the C ABI loads, exports every symbol
include/dcue.h declares, reports the reference layouts; DCUENet builds the reference's parameters."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "dcue.h")


def _declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|int64_t|const char\s*\*)\s*(dcue_\w+)\s*\(", src, flags=re.M)))


def test_library_exports_header_symbols():
    from dcrecommend import _native as nat
    lib = nat.lib()
    names = _declared()
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), n
    hdr = open(os.path.join(ROOT, "include", "dcue.h")).read()
    assert lib.dcue_abi_version() == int(re.search(r"#define DCUE_ABI_VERSION (\d+)", hdr).group(1))
    assert lib.dcue_abi_version() == nat.ABI_VERSION


def test_ctypes_structs_match_header(tmp_path):
    """sizeof/offsetof of every ABI struct, compiled from include/dcue.h, against the ctypes mirror."""
    import ctypes
    import subprocess
    from dcrecommend import _native as nat
    structs = {"dcue_dims": nat.Dims, "dcue_model": nat.Model, "dcue_batch": nat.Batch,
               "dcue_tracks": nat.Tracks, "dcue_adam_args": nat.AdamArgs, "dcue_opt_args": nat.OptArgs,
               "dcue_opt_state": nat.OptState}
    src = ["#include <stdio.h>", "#include <stddef.h>", '#include "dcue.h"', "int main(void) {"]
    for cname, py in structs.items():
        src.append('printf("%s %%zu\\n", sizeof(%s));' % (cname, cname))
        for fname, _ in py._fields_:
            src.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (cname, fname, cname, fname))
    src.append('printf("dcue_emb_log %zu\\n", sizeof(dcue_emb_log));')
    src.append('printf("dcue_mt_state %zu\\n", sizeof(dcue_mt_state));')
    src.append("return 0; }")
    (tmp_path / "probe.c").write_text("\n".join(src))
    subprocess.check_call(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), str(tmp_path / "probe.c"),
                           "-o", str(tmp_path / "probe")])
    got = dict(l.split() for l in subprocess.check_output([str(tmp_path / "probe")]).decode().splitlines())
    for cname, py in structs.items():
        assert int(got[cname]) == ctypes.sizeof(py), cname
        for fname, _ in py._fields_:
            assert int(got["%s.%s" % (cname, fname)]) == getattr(py, fname).offset, (cname, fname)
    assert int(got["dcue_mt_state"]) == nat.MT_STATE_BYTES
    assert int(got["dcue_emb_log"]) == 32


def test_binding_covers_header():
    from dcrecommend import _native as nat
    assert set(_declared()) == set(nat._SIGS), set(_declared()) ^ set(nat._SIGS)


def test_layouts_match_reference_shapes(golden):
    from dcrecommend import _native as nat
    g = golden("model_tiny.npz")
    H, d = int(g["H"]), int(g["d"])
    dims = nat.make_dims(H, d, 300, int(g["n_users"]))
    off = nat.param_layout(dims)
    for s, name in enumerate(nat.DENSE_NAMES):
        if name.startswith("text."):  # the text tower's segments: empty in the audio-only towers
            assert off[s + 1] == off[s], name
            continue
        n = g["init." + name].size
        assert off[s] % 4 == 0
        assert off[s + 1] - off[s] >= n, name
        assert off[s + 1] - off[s] < n + 4, name
    boff = nat.bn_layout(dims)
    assert boff[1] - boff[0] >= 128 and boff[-1] > 0
    # conv packs only: forward, dgrad (layers 2-5) and their split-f16 copies
    assert nat.wpack_floats(dims) == 2 * 128 * H * 4 + 4 * (2 * H * H * 4 + H * H * 2 + d * H)
    assert nat.workspace_bytes(dims, 4, 3, 16) > 0


@pytest.mark.parametrize("H,d,mt", [(128, 100, "truedcuemel1dbn"), (40, 24, "truedcuemel1dresbn"),
                                     (36, 20, "truedcuemel1d"), (200, 7, "truedcuemel1dres"),
                                     (1, 256, "truedcuemel1dbn")])
def test_any_width_accepted(H, d, mt):
    """Any conv_hidden / feature_dim in 1..256 (the reference's DCUENet takes any; its trainer's
    default is feature_dim = 100, nn/dcue.py:44). The library stores them at the width rounded up to
    32/64/128/256, and every reference-shaped parameter is the leading corner of its segment."""
    from dcrecommend import _native as nat
    from dcrecommend.dcue.dcue import DCUENet
    dims = nat.make_dims(H, d, 300, 10, mt)
    sd = nat.storage_dims(dims)
    for w, ws in ((H, sd.conv_hidden), (d, sd.feature_dim)):
        assert ws in (32, 64, 128, 256) and ws >= w and (ws == 32 or ws // 2 < w)
    off = nat.param_layout(dims)
    shapes = nat.segment_shapes(dims)
    torch.manual_seed(0)
    net = DCUENet({"feature_dim": d, "conv_hidden": H, "user_embdim": 300, "user_count": 10, "model_type": mt})
    named = dict(net.named_parameters())
    P = torch.zeros(off[-1])
    for s, name in enumerate(nat.DENSE_NAMES):
        seg = off[s + 1] - off[s]
        n = int(np.prod(shapes[s]))
        if name not in named:  # BN parameters of a tower without BN: empty segment
            assert seg == 0
            continue
        p = named[name]
        assert len(shapes[s]) == p.dim() and all(a >= b for a, b in zip(shapes[s], p.shape)), name
        assert n <= seg < n + 4, name
        nat.corner(P, off[s], shapes[s], p.shape).copy_(p.data)
    # the corners tile the buffer without overlap: every parameter's values appear exactly once
    total = sum(p.numel() for n, p in named.items() if n in nat.DENSE_NAMES)
    assert int((P != 0).sum()) <= total
    for s, name in enumerate(nat.DENSE_NAMES):
        if name in named:
            assert torch.equal(nat.corner(P, off[s], shapes[s], named[name].shape), named[name].data), name


def test_unsupported_dims_rejected():
    from dcrecommend import _native as nat
    for H, d in ((128, 257), (300, 128), (0, 128)):
        with pytest.raises(RuntimeError, match="UNSUPPORTED|INVALID"):
            nat.param_layout(nat.make_dims(H, d, 300, 10))


def test_dcuenet_init_matches_reference(golden):
    from dcrecommend.dcue.dcue import DCUENet
    g = golden("model_tiny.npz")
    torch.manual_seed(int(g["seed"]))
    net = DCUENet({"feature_dim": int(g["d"]), "conv_hidden": int(g["H"]), "user_embdim": 300,
                   "user_count": int(g["n_users"]), "model_type": "truedcuemel1dbn"})
    sd = net.state_dict()
    keys = [k[len("init."):] for k in g.files if k.startswith("init.")]
    assert set(sd) == set(keys)
    for k in keys:
        assert np.array_equal(sd[k].numpy(), g["init." + k]), k


def test_dcuenet_model_type_errors():
    from dcrecommend.dcue.dcue import DCUENet
    args = {"feature_dim": 32, "conv_hidden": 32, "user_embdim": 300, "user_count": 4}
    with pytest.raises(ValueError):
        DCUENet(dict(args, model_type="nope"))


@pytest.mark.parametrize("name", ["model_plain.npz", "model_res.npz", "model_resbn.npz"])
def test_dcuenet_towers_init_match_reference(golden, name):
    """truedcuemel1d / truedcuemel1dres / truedcuemel1dresbn: the reference's state_dict keys,
    shapes and init draws (checksums), and a flat layout whose BN segments are empty without BN."""
    from dcrecommend import _native as nat
    from dcrecommend.dcue.dcue import DCUENet
    g = golden(name)
    mt = str(g["model_type"])
    torch.manual_seed(int(g["seed"]))
    net = DCUENet({"feature_dim": int(g["d"]), "conv_hidden": int(g["H"]), "user_embdim": 300,
                   "user_count": int(g["n_users"]), "model_type": mt})
    sd = net.state_dict()
    keys = {k[len("initsum."):] for k in g.files if k.startswith("initsum.")}
    assert set(sd) == keys
    for k in keys:
        assert float(sd[k].double().sum()) == pytest.approx(float(g["initsum." + k]), rel=1e-12, abs=1e-9), k
    off = nat.param_layout(nat.make_dims(int(g["H"]), int(g["d"]), 300, int(g["n_users"]), mt))
    named = dict(net.named_parameters())
    for s_, n in enumerate(nat.DENSE_NAMES):
        size = named[n].numel() if n in named else 0
        assert size <= off[s_ + 1] - off[s_] < size + 4, n


def test_cpu_model_refuses_compute():
    from dcrecommend.dcue.dcue import DCUENet
    net = DCUENet({"feature_dim": 32, "conv_hidden": 32, "user_embdim": 300, "user_count": 4,
                   "model_type": "truedcuemel1dbn"})
    with pytest.raises(RuntimeError, match="GPU"):
        net(torch.zeros(2, dtype=torch.long), torch.zeros(2, 128, 131), torch.zeros(2, 1, 128, 131))


def test_check_mode_disabled_by_default(monkeypatch):
    """Check mode (dcrecommend.check) is opt-in: DCUE_CHECK unset or 0 leaves it off."""
    from dcrecommend import check
    monkeypatch.delenv("DCUE_CHECK", raising=False)
    assert not check.enabled_by_env()
    monkeypatch.setenv("DCUE_CHECK", "1")
    assert check.enabled_by_env()


@pytest.mark.parametrize("td,wd,t,d", [(256, 300, 64, 256), (100, 64, 20, 100), (40, 128, 128, 32)])
def test_text_tower_layout(td, wd, t, d):
    """The mixed audio + text tower (BASELINE config 4): its parameters -- the BN tower with
    fc(text_dim + d -> d), the text conv [text_dim][word_dim][3] -- are corners of the flat segments
    (text channels stored at 64 / 128 / 256), the frozen word vectors stay outside the flat buffer,
    and the split-f16 text weight pack is 3 x word_dim (rounded up to 32) x the storage channels."""
    from dcrecommend import _native as nat
    from dcrecommend.dcue.dcue import DCUENet
    args = {"feature_dim": d, "conv_hidden": 64, "user_embdim": 300, "user_count": 10,
            "model_type": "truedcuemel1dbntext", "text_dim": td, "word_dim": wd, "text_len": t,
            "n_words": 50, "pad_idx": 0}
    torch.manual_seed(0)
    net = DCUENet(args)
    dims = nat.make_dims(64, d, 300, 10, "truedcuemel1dbntext", (td, wd, t, 0))
    off, shapes = nat.param_layout(dims), nat.segment_shapes(dims)
    named = dict(net.named_parameters())
    assert named["conv.fc.weight"].shape == (d, td + d)
    assert named["text.conv.weight"].shape == (td, wd, 3)
    assert "text.embeddings.weight" not in nat.DENSE_NAMES
    for s, name in enumerate(nat.DENSE_NAMES):
        p = named[name]
        n = int(np.prod(shapes[s]))
        assert n <= off[s + 1] - off[s] < n + 4, name
        assert all(a >= b for a, b in zip(shapes[s], p.shape)), name
    cts = nat.text_storage(td)
    assert shapes[nat.DENSE_NAMES.index("text.conv.weight")] == (cts, wd, 3)
    plain = nat.wpack_floats(nat.make_dims(64, d, 300, 10, "truedcuemel1dbn"))
    assert nat.wpack_floats(dims) == plain + 3 * ((wd + 31) // 32 * 32) * cts


def test_text_tower_rejects_bad_dims():
    from dcrecommend import _native as nat
    for text, err in (((300, 300, 64, 0), "UNSUPPORTED"), ((256, 302, 64, 0), "UNSUPPORTED"),
                      ((256, 300, 129, 0), "UNSUPPORTED"), ((256, 300, 1, 0), "INVALID")):
        with pytest.raises(RuntimeError, match=err):
            nat.param_layout(nat.make_dims(64, 256, 300, 10, "truedcuemel1dbntext", text))


def test_text_oracle_contract():
    """oracle/text_oracle.py: token rows in the reference's shape (dcuelmitemset.py:40-56: BOS,
    sentence, EOS, PAD) and a forward whose PAD positions never win the max."""
    from oracle import text_oracle as TO
    gen = torch.Generator().manual_seed(0)
    tok = TO.sentences(gen, 50, 16, 30, pad_idx=0, min_len=0)
    assert tok.shape == (50, 16) and bool((tok[:, 0] == 1).all())
    for row in tok:
        L = int((row != 0).sum())
        assert int(row[L - 1]) == 2 and bool((row[L:] == 0).all()) and bool((row[1:L - 1] >= 3).all())
    torch.manual_seed(1)
    p, _ = TO.init_params(32, 32, 8, 4, 16, 12, 30)
    s = TO.text_features(p, tok, 0)
    assert s.shape == (50, 16) and bool((s >= 0).all())
    # PAD positions changed to anything: the features do not move unless a real neighbour reads them
    emb = p["text.embeddings.weight"].clone()
    p["text.embeddings.weight"][0] = 0.0
    s0 = TO.text_features(p, tok, 0)
    p["text.embeddings.weight"] = emb
    full = tok[:, -1] != 0  # no PAD at all: identical
    assert torch.equal(s0[full], s[full])
