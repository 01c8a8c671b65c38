"""DCUENet on MI355X: the reference module API (dcrecommend/dcue/dcue.py:21-108) over libdcue_hip.

Same constructor (`DCUENet(dict_args)`), attributes (`.conv`, `.user_embd`, `.sim`), forward
signature and return tuple, and the same state_dict keys -- so reference checkpoints and warm-start
audio models load unchanged. Parameters live in ONE flat fp32 device buffer (reference order and
layouts, views per nn.Parameter) so the optimizer step is one elementwise sweep; the user table is
its own buffer because it is sharded by user under data parallelism.

Every forward/backward runs through the HIP C ABI; there is no eager-PyTorch compute path.
"""
import ctypes
import weakref

import torch
from torch import nn

from dcrecommend import _native as nat

REFERENCE_TYPES = ("truedcuemel1d", "truedcuemel1dres", "truedcuemel1dbn", "truedcuemel1dresbn")
# BASELINE config 4: the mixed audio + text item encoder (no reference code: the reference's text item
# set imports a WordEmbeddings module it never published, datasets/dcuelmitemset.py:8)
TEXT_TYPE = nat.TEXT_TOWER
SUPPORTED_TYPES = REFERENCE_TYPES + (TEXT_TYPE,)
# the text tower's extra dict_args keys and their defaults (config 4: d = 256; 300-d word vectors;
# one sentence of at most 63 tokens + BOS/EOS per track, dcuelmitemset.py:40-56)
TEXT_DEFAULTS = {"text_dim": 256, "word_dim": 300, "text_len": 64, "n_words": 20000, "pad_idx": 0}

# conv stack shared by the towers, truedcuemel1dbn.py:25-61: (kernel, padding) per layer
_CONV = ((4, 2), (4, 2), (4, 2), (2, 1), (1, 0))


class _ItemTower(nn.Module):
    """Parameter container with the reference's names (conv.bn0..5, conv.layer1..5, conv.fc) for the
    four towers DCUENet wires (dcue/dcue.py:49-59): truedcuemel1dbn (default), truedcuemel1d (no
    BatchNorm), truedcuemel1dres / truedcuemel1dresbn (time-pooled skips into fc(4H + d -> d))."""

    def __init__(self, feature_dim, conv_hidden, model_type="truedcuemel1dbn", text_dim=0):
        super().__init__()
        bn = model_type in ("truedcuemel1dbn", "truedcuemel1dresbn", TEXT_TYPE)
        res = model_type in ("truedcuemel1dres", "truedcuemel1dresbn")
        chans = [nat.N_MELS] + [conv_hidden] * 4 + [feature_dim]
        # construction order = RNG consumption order of the reference constructors (BN draws nothing)
        for l in range(6):
            if bn:
                self.add_module("bn%d" % l, nn.BatchNorm1d(chans[l]))
            if l < 5:
                k, pad = _CONV[l]
                self.add_module("layer%d" % (l + 1), nn.Conv1d(chans[l], chans[l + 1], k, 1, pad, bias=True))
        # res towers: fc(4H + d -> d); the text tower: fc(text_dim + d -> d) over [text features ; audio]
        fi = 4 * conv_hidden + feature_dim if res else text_dim + feature_dim if model_type == TEXT_TYPE else feature_dim
        self.fc = nn.Linear(fi, feature_dim)
        for l in range(1, 6):
            nn.init.kaiming_uniform_(getattr(self, "layer%d" % l).weight, nonlinearity="relu")
        nn.init.xavier_uniform_(self.fc.weight)
        if model_type == "truedcuemel1dbn":
            self.outsize = [conv_hidden, 1]
        self._owner = None

    def forward(self, X):
        """DCUENet.conv(X): item features [M, d] for spectrograms X [M, 128, 131] (eval or train BN)."""
        net = self._owner() if self._owner is not None else None
        if net is None:
            raise RuntimeError("item tower is only callable through its DCUENet")
        return net.item_features(X)


class _TextTower(nn.Module):
    """The text branch of the mixed item tower (BASELINE config 4; csrc/text.hip): frozen word vectors
    `embeddings` [n_words, word_dim] -- the language-model-pretrained part, supplied by the caller
    through load_state_dict (never fetched; random N(0, 1) until then) -- and `conv`, a
    Conv1d(word_dim -> text_dim, kernel 3, padding 1) whose outputs are max-pooled over each sentence's
    non-PAD positions and passed through a ReLU."""

    def __init__(self, n_words, word_dim, text_dim):
        super().__init__()
        self.embeddings = nn.Embedding(n_words, word_dim)
        self.embeddings.weight.requires_grad_(False)
        self.conv = nn.Conv1d(word_dim, text_dim, 3, 1, 1, bias=True)
        nn.init.kaiming_uniform_(self.conv.weight, nonlinearity="relu")


class _UserTower(nn.Module):
    """userembedding.py:27-31 names: embeddings, linear1, linear2."""

    def __init__(self, user_count, user_embdim, feature_dim):
        super().__init__()
        self.user_embdim, self.user_count, self.feature_dim = user_embdim, user_count, feature_dim
        self.embeddings = nn.Embedding(user_count, user_embdim)
        self.linear1 = nn.Linear(user_embdim, user_embdim)
        self.linear2 = nn.Linear(user_embdim, feature_dim)
        self._owner = None

    def forward(self, user_idx):
        net = self._owner() if self._owner is not None else None
        if net is None:
            raise RuntimeError("user tower is only callable through its DCUENet")
        return net.user_features(user_idx)


class _StepFunction(torch.autograd.Function):
    """Train-mode forward through the C ABI; backward feeds dL/dscores to dcue_train_backward."""

    @staticmethod
    def forward(ctx, anchor, net, u, X, N, tokens=None):
        scores, uf, f, _ = net._native_forward(u, X, N, train=True, margin=0.0, tokens=tokens)
        ctx.net = net
        ctx.mark_non_differentiable(uf, f)
        return scores, uf, f

    @staticmethod
    def backward(ctx, dscores, duf, df):
        net = ctx.net
        if duf is not None and bool(torch.any(duf != 0)) or df is not None and bool(torch.any(df != 0)):
            raise RuntimeError("DCUENet backward supports gradients through the scores only")
        net._native_backward(dscores.contiguous().float())
        return None, None, None, None, None, None


class DCUENet(nn.Module):
    """PyTorch-facing DCUE model whose compute is libdcue_hip (dcue/dcue.py:21-108)."""

    def __init__(self, dict_args):
        super().__init__()
        self.feature_dim = dict_args["feature_dim"]
        self.conv_hidden = dict_args["conv_hidden"]
        self.user_embdim = dict_args["user_embdim"]
        self.user_count = dict_args["user_count"]
        self.model_type = dict_args["model_type"]
        if self.model_type not in SUPPORTED_TYPES:
            raise ValueError("{} is not a recognized model type!".format(self.model_type))
        self.is_text = self.model_type == TEXT_TYPE
        if self.is_text:
            for k, v in TEXT_DEFAULTS.items():
                setattr(self, k, int(dict_args.get(k, v)))
        self.conv = _ItemTower(self.feature_dim, self.conv_hidden, self.model_type,
                               self.text_dim if self.is_text else 0)
        self.user_embd = _UserTower(self.user_count, self.user_embdim, self.feature_dim)
        if self.is_text:
            self.text = _TextTower(self.n_words, self.word_dim, self.text_dim)
        self.sim = nn.CosineSimilarity(dim=1)
        self.conv._owner = weakref.ref(self)
        self.user_embd._owner = weakref.ref(self)
        self._anchor = torch.zeros((), requires_grad=True)
        self._flat = None  # device-side state, built by _apply when moved to the GPU
        self._pending_plan = None  # a TrainPlan whose last step left Adam work on a side stream
        self._ws = None
        self._ws_key = None

    # ------------------------------------------------------------------ device-resident layout
    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        p0 = self.conv.layer1.weight
        if p0.is_cuda:
            self._flatten(p0.device)
        else:
            self._flat = None
        return out

    def _flatten(self, device):
        """Move every dense parameter/buffer into the flat buffers the C ABI addresses."""
        dims = nat.make_dims(self.conv_hidden, self.feature_dim, self.user_embdim, self.user_count,
                             self.model_type, self._text_dims())
        poff = nat.param_layout(dims)
        boff = nat.bn_layout(dims)
        shapes = nat.segment_shapes(dims)
        named = dict(self.named_parameters())
        # zero-filled: the storage channels past the reference's H / d stay exactly zero (dcue.h)
        P = torch.zeros(poff[-1], dtype=torch.float32, device=device)
        G = torch.zeros_like(P)
        for s, name in enumerate(nat.DENSE_NAMES):
            if name not in named:  # BN parameters of a tower without BatchNorm: empty segment
                continue
            p = named[name]
            view = nat.corner(P, poff[s], shapes[s], p.shape)
            view.copy_(p.data)
            p.data = view
            p._dcue_owner = weakref.ref(self)
        stats = torch.zeros(boff[-1], dtype=torch.float32, device=device)
        nbt = torch.zeros(nat.N_BN, dtype=torch.int64, device=device)
        for l in range(nat.N_BN):
            bn = getattr(self.conv, "bn%d" % l, None)
            if bn is None:
                continue
            C = bn.num_features
            stats[boff[2 * l]:boff[2 * l] + C].copy_(bn.running_mean)
            stats[boff[2 * l + 1]:boff[2 * l + 1] + C].copy_(bn.running_var)
            nbt[l].copy_(bn.num_batches_tracked)
            bn.running_mean = stats[boff[2 * l]:boff[2 * l] + C]
            bn.running_var = stats[boff[2 * l + 1]:boff[2 * l + 1] + C]
            bn.num_batches_tracked = nbt[l]
        emb = self.user_embd.embeddings.weight
        emb._dcue_owner = weakref.ref(self)
        slot = torch.full((max(self.user_count, 1),), -1, dtype=torch.int32, device=device)
        # zero-filled once: the text weights' split-f16 pack has zero K padding past word_dim
        wpack = torch.zeros(nat.wpack_floats(dims), dtype=torch.float32, device=device)
        self._flat = dict(dims=dims, poff=poff, boff=boff, shapes=shapes, P=P, G=G, stats=stats, nbt=nbt, slot=slot,
                          wpack=wpack, emb_grad=torch.zeros(0, device=device),
                          emb_rows=torch.zeros(0, dtype=torch.int64, device=device), m=None, v=None,
                          em=None, ev=None)
        self._ws = None
        self._ds = nat.storage_dims(dims).feature_dim
        self._words_key = None
        self._repack()

    def _text_dims(self):
        return (self.text_dim, self.word_dim, self.text_len, self.pad_idx) if self.is_text else None

    def _words_exp(self):
        """dcue_model.words_exp of the (frozen) word vectors, recomputed when they are rewritten."""
        w = self.text.embeddings.weight
        key = (w.data_ptr(), w._version)
        if self._words_key != key:
            self._words_exp_v, self._words_key = nat.words_exponent(w), key
        return self._words_exp_v

    def _repack(self):
        """Refresh the MFMA-packed conv weights from the flat parameters."""
        nat.check(nat.lib().dcue_pack_weights(ctypes.byref(self._model_struct()), nat.stream_handle()),
                  "dcue_pack_weights")
        self._flat["packed_version"] = self._conv_versions()

    def _conv_versions(self):
        # each nn.Parameter keeps its own version counter (setting .data does not share P's), so the
        # conv weights' counters are what records a host-side write to them
        v = tuple(getattr(self.conv, "layer%d" % l).weight._version for l in range(1, 6))
        return v + ((self.text.conv.weight._version,) if self.is_text else ())

    def _sync_plan(self):
        """Order torch's current stream after the last plan step's side-stream Adam work
        (TrainPlan.sync): parameters read from torch are then current."""
        plan = getattr(self, "_pending_plan", None)
        if plan is not None:
            self._pending_plan = None
            plan.sync(nat.stream_handle())

    def _require_device(self):
        if self._flat is None:
            raise RuntimeError("DCUENet must be moved to the GPU (.cuda()) before use: its forward "
                               "and backward run only through libdcue_hip on the MI355X")
        self._sync_plan()
        if self.conv.layer1.weight.data_ptr() != self._flat["P"].data_ptr() + 4 * self._flat["poff"][2]:
            # parameters were re-assigned behind our back (load_state_dict copies in place, so this
            # only happens if a caller replaced .data): rebuild the flat view
            self._flatten(self._flat["P"].device)
        if self._conv_versions() != self._flat["packed_version"]:
            # a host-side write (load_state_dict, manual edits) changed the parameters; the native
            # optimizer repacks by itself and does not bump the version counter
            self._repack()
        return self._flat

    def _model_struct(self, adam_state=None):
        fl = self._flat
        m = nat.Model()
        m.dims = fl["dims"]
        m.params, m.grads = fl["P"].data_ptr(), fl["G"].data_ptr()
        m.emb = self.user_embd.embeddings.weight.data_ptr()
        m.emb_grad = fl["emb_grad"].data_ptr() if fl["emb_grad"].numel() else None
        m.emb_slot = fl["slot"].data_ptr()
        m.bn_stats, m.bn_batches, m.wpack = fl["stats"].data_ptr(), fl["nbt"].data_ptr(), fl["wpack"].data_ptr()
        m.emb_rows = fl["emb_rows"].data_ptr() if fl["emb_rows"].numel() else None
        if self.is_text:
            w = self.text.embeddings.weight
            nat.require_gpu(w, "text.embeddings.weight")
            m.words, m.n_words, m.words_exp = w.data_ptr(), w.shape[0], self._words_exp()
        opt = self._deferred_opt() if getattr(self, "_deferred_opt", None) is not None else None
        if opt is not None and adam_state is None:
            adam_state = opt._adam_state()  # the deferred user-table Adam replays inside forwards
        if adam_state is not None:
            m.exp_avg, m.exp_avg_sq = adam_state["m"].data_ptr(), adam_state["v"].data_ptr()
            m.emb_exp_avg, m.emb_exp_avg_sq = adam_state["em"].data_ptr(), adam_state["ev"].data_ptr()
            if adam_state.get("emb_step") is not None:
                m.emb_step, m.emb_log = adam_state["emb_step"].data_ptr(), adam_state["emb_log"].data_ptr()
                m.emb_log_cap = adam_state["cap"]
        return m

    def sync_user_table(self):
        """Bring every user row current under a deferred-embedding NativeAdam (no-op otherwise):
        afterwards the table and its moments equal the dense per-step sweep's bit for bit."""
        opt = self._deferred_opt() if getattr(self, "_deferred_opt", None) is not None else None
        if opt is not None:
            opt.flush()

    def state_dict(self, *args, **kwargs):
        if self._flat is not None:
            self._sync_plan()
            self.sync_user_table()
        return super().state_dict(*args, **kwargs)

    def load_state_dict(self, state_dict, strict=True, assign=False):
        if self._flat is not None:
            self._sync_plan()
            self.sync_user_table()  # pending deferred steps belong to the table being replaced
        return super().load_state_dict(state_dict, strict=strict, assign=assign)

    def _workspace(self, B, N, M):
        key = (B, N, M)
        if self._ws is None or self._ws_key is None or any(a < b for a, b in zip(self._ws_key, key)):
            grow = tuple(max(a, b) for a, b in zip(self._ws_key or key, key))
            nbytes = nat.workspace_bytes(self._flat["dims"], *grow)
            self._ws = torch.empty(nbytes, dtype=torch.uint8, device=self._flat["P"].device)
            if nat.poison_on():
                self._ws.fill_(255)
            self._ws_key = grow
        if self._flat["emb_grad"].numel() < B * self.user_embdim:
            self._flat["emb_grad"] = torch.zeros(B * self.user_embdim, dtype=torch.float32,
                                                 device=self._flat["P"].device)
            self._flat["emb_rows"] = torch.full((B,), -1, dtype=torch.int64, device=self._flat["P"].device)
        return self._ws

    # -------------------------------------------------------------------------- native calls
    def _spectro_table(self, X):
        """[M,128,131] fp32 spectrograms -> [M,131,128] track rows via the C ABI."""
        nat.require_gpu(X, "spectrograms")
        X = X.contiguous().float()
        M = X.shape[0]
        if X.shape[1:] != (nat.N_MELS, nat.N_FRAMES):
            raise ValueError("spectrograms must be [M, 128, 131], got %s" % (tuple(X.shape),))
        out = torch.empty((M, nat.N_FRAMES, nat.N_MELS), dtype=torch.float32, device=X.device)
        nat.check(nat.lib().dcue_transpose_spectrograms(nat.ptr(X), M, nat.ptr(out), nat.stream_handle()),
                  "dcue_transpose_spectrograms")
        return out

    def _tracks(self, tracks, tokens=None):
        """dcue_tracks of an HBM track table (+ the text tower's [n_tracks, text_len] token table)."""
        tr = nat.Tracks(tracks.data_ptr(), tracks.shape[0], 0 if tracks.dtype == torch.float16 else 1, 0)
        if self.is_text:
            if tokens is None:
                raise ValueError("the text tower needs each track's token ids (tokens [n_tracks, %d])" % self.text_len)
            nat.require_gpu(tokens, "tokens")
            if tokens.dtype != torch.int32 or tuple(tokens.shape) != (tracks.shape[0], self.text_len) \
                    or not tokens.is_contiguous():
                raise ValueError("tokens must be a contiguous int32 [%d, %d] tensor, got %s %s"
                                 % (tracks.shape[0], self.text_len, tokens.dtype, tuple(tokens.shape)))
            tr.tokens = tokens.data_ptr()
        return tr

    def native_forward(self, users, tracks, item_track, n_neg, layout, neg_item=None, train=True,
                       margin=0.2, copy_outputs=True, tokens=None):
        """Forward over an HBM-resident track table (text tower: and its token table). Returns
        (scores, user_feat, item_feat, loss).

        copy_outputs=False returns views into the workspace (no copy; overwritten by the next call)."""
        fl = self._require_device()
        B = users.shape[0]
        M = item_track.shape[0]
        ws = self._workspace(B, n_neg, M)
        batch = nat.Batch(B, n_neg, M, layout, users.data_ptr(), item_track.data_ptr(),
                          neg_item.data_ptr() if neg_item is not None else None)
        tr = self._tracks(tracks, tokens)
        model = self._model_struct()
        nat.check(nat.lib().dcue_forward(ctypes.byref(model), ctypes.byref(batch), ctypes.byref(tr),
                                         nat.ptr(ws), ws.numel(), int(bool(train)), float(margin),
                                         None, None, None, None, nat.stream_handle()), "dcue_forward")
        self._last = (users, tracks, item_track, n_neg, layout, neg_item, tokens)
        key = (B, n_neg, M)
        if fl.get("out_key") != key:
            fl["out_off"], fl["out_key"] = nat.workspace_outputs(fl["dims"], B, n_neg, M), key
        off = fl["out_off"]
        d, ds = self.feature_dim, self._ds  # feature rows are stored d_s wide, zero past d

        def view(o, n, shape):
            return ws[o:o + 4 * n].view(torch.float32).view(shape)
        outs = (view(off[0], B * n_neg, (B, n_neg)), view(off[1], B * ds, (B, ds))[:, :d],
                view(off[2], M * ds, (M, ds))[:, :d], view(off[3], 1, ()))
        return tuple(o.clone() for o in outs) if copy_outputs else outs

    def native_backward(self, dscores=None, emb_grad_scale=1.0):
        """Backward of the last train-mode native_forward: writes the flat grads + compact
        embedding rows (emb_grad/emb_slot)."""
        fl = self._require_device()
        users, tracks, item_track, n_neg, layout, neg_item, tokens = self._last
        B, M = users.shape[0], item_track.shape[0]
        ws = self._workspace(B, n_neg, M)
        batch = nat.Batch(B, n_neg, M, layout, users.data_ptr(), item_track.data_ptr(),
                          neg_item.data_ptr() if neg_item is not None else None)
        tr = self._tracks(tracks, tokens)
        model = self._model_struct()
        nat.check(nat.lib().dcue_train_backward(ctypes.byref(model), ctypes.byref(batch), ctypes.byref(tr),
                                                nat.ptr(ws), ws.numel(), nat.ptr(dscores),
                                                float(emb_grad_scale), nat.stream_handle()),
                  "dcue_train_backward")
        # expose reference-shaped .grad views of the flat gradient (the user table's gradient is
        # kept compact: embedding_grad_dense() materialises it on request)
        self._expose_grads()
        self.user_embd.embeddings.weight.grad = None
        self._grad_users = users

    def _expose_grads(self):
        fl = self._flat
        named = dict(self.named_parameters())
        for s, name in enumerate(nat.DENSE_NAMES):
            p = named.get(name)
            if p is not None:
                p.grad = nat.corner(fl["G"], fl["poff"][s], fl["shapes"][s], p.shape)

    def embedding_grad_dense(self):
        """Dense [n_users, E] view of the last backward's embedding gradient (for inspection)."""
        fl = self._require_device()
        dense = torch.zeros_like(self.user_embd.embeddings.weight)
        users = self._grad_users
        slots = fl["slot"][users.long()]
        rows = fl["emb_grad"][: users.shape[0] * self.user_embdim].view(-1, self.user_embdim)
        first = slots >= 0
        dense[users[first].long()] = rows[slots[first].long()]
        return dense

    def _token_table(self, tokens, M):
        if not self.is_text:
            return None
        if tokens is None:
            raise ValueError("the text tower's forward needs the items' token ids")
        nat.require_gpu(tokens, "tokens")
        t = tokens.reshape(M, -1).to(torch.int32).contiguous()
        if t.shape[1] != self.text_len:
            raise ValueError("token rows must hold text_len = %d ids, got %d" % (self.text_len, t.shape[1]))
        return t

    def _native_forward(self, u, X, N, train, margin, tokens=None):
        B = X.shape[0] // (1 + N)
        table = self._spectro_table(X)
        tok = self._token_table(tokens, X.shape[0])
        self._table_keepalive = (table, tok)
        item_track = torch.arange(X.shape[0], dtype=torch.int32, device=X.device)
        return self.native_forward(u.to(torch.int64).contiguous(), table, item_track, N,
                                   nat.LAYOUT_CATALOGUE, None, train=train, margin=margin, tokens=tok)

    def _native_backward(self, dscores):
        self.native_backward(dscores)

    # --------------------------------------------------------------------- reference API
    def item_features(self, X, tokens=None):
        fl = self._require_device()
        table = self._spectro_table(X)
        M = table.shape[0]
        out = torch.empty((M, self._ds), dtype=torch.float32, device=table.device)
        if self.training:
            raise NotImplementedError("DCUENet.conv(X) in train mode is only reachable through forward()")
        ws = self._workspace(1, 0, M)
        tr = self._tracks(table, self._token_table(tokens, M))
        item_track = torch.arange(M, dtype=torch.int32, device=table.device)
        nat.check(nat.lib().dcue_item_tower_eval(ctypes.byref(self._model_struct()), ctypes.byref(tr),
                                                 nat.ptr(item_track), M, nat.ptr(ws), ws.numel(),
                                                 nat.ptr(out), nat.stream_handle()), "dcue_item_tower_eval")
        return out[:, :self.feature_dim].squeeze()

    def user_features(self, user_idx):
        self._require_device()
        nat.require_gpu(user_idx, "user_idx")
        shape = tuple(user_idx.shape)
        u = user_idx.reshape(-1).to(torch.int64).contiguous()
        out = torch.empty((u.shape[0], self._ds), dtype=torch.float32, device=u.device)
        ws = self._workspace(u.shape[0], 0, 1)
        nat.check(nat.lib().dcue_user_tower(ctypes.byref(self._model_struct()), nat.ptr(u), u.shape[0],
                                            nat.ptr(ws), ws.numel(), nat.ptr(out), nat.stream_handle()),
                  "dcue_user_tower")
        return out[:, :self.feature_dim].reshape(*shape, self.feature_dim)

    def forward(self, u, pos, neg=None, pos_text=None, neg_text=None):
        """dcue/dcue.py:70-108 -> (scores [B,N], user feats [B,d], pos feats [B,d], neg feats [B,N,d]).
        The text tower (config 4) also takes the items' token ids: pos_text [B, T], neg_text [B, N, T]."""
        self._require_device()
        if neg is None:
            # reference quirk (dcue/dcue.py:101-108): neg_featvects is never bound on this path
            raise UnboundLocalError("local variable 'neg_featvects' referenced before assignment")
        B, N = neg.shape[0], neg.shape[1]
        X = torch.empty((B * (1 + N), nat.N_MELS, nat.N_FRAMES), dtype=torch.float32, device=pos.device)
        X[:B].copy_(pos)
        X[B:].copy_(neg.reshape(B * N, nat.N_MELS, nat.N_FRAMES))
        tok = None
        if self.is_text:
            if pos_text is None or neg_text is None:
                raise ValueError("the text tower's forward needs pos_text [B, T] and neg_text [B, N, T]")
            tok = torch.cat([pos_text.reshape(B, -1), neg_text.reshape(B * N, -1)], 0)
        if self.training and torch.is_grad_enabled():
            scores, uf, f = _StepFunction.apply(self._anchor, self, u, X, N, tok)
        else:
            scores, uf, f, _ = self._native_forward(u, X, N, train=self.training, margin=0.0, tokens=tok)
        return scores, uf, f[:B], f[B:].reshape(B, N, self.feature_dim)
