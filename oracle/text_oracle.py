"""ORACLE -- CPU restatement of the mixed audio + text item tower (BASELINE config 4).  TEST
INFRASTRUCTURE ONLY: imported by tests/ and bench.py's checks, never by the product path.

PARITY UNPINNED against the reference: the reference never published this path. Its text item set
(datasets/dcuelmitemset.py) imports `dcrecommend.dcue.embeddings.wordembedding.WordEmbeddings`, a
module that is not in the tree (:8), so there is no text encoder, no golden vector and nothing to
import. What the reference does pin is the data contract: one sentence of token ids per track,
[BOS] + sentence + [EOS], cut to max_sentence_length + 1 and right-padded with PAD_IDX
(dcuelmitemset.py:40-56). The encoder restated here is this build's choice:

    e  = words[tokens]                         frozen word vectors (LM-pretrained, caller supplied)
    z  = Conv1d(word_dim -> text_dim, k=3, pad=1)(e)
    s  = relu(max over the non-PAD positions of z)
    f  = fc(cat([s, bn5(audio)]))              Linear(text_dim + d -> d)

with the audio stack of the default tower truedcuemel1dbn (dcue_oracle.item_tower, reference
truedcuemel1dbn.py:77-99), the user tower, cosine scores and hinge loss of dcue_oracle. Float math is
torch-CPU (fp32, or fp64 for tolerance tests); the backward is autograd's.
"""
import math

import torch
import torch.nn.functional as F

from oracle import dcue_oracle as O

TEXT_TOWER = "truedcuemel1dbntext"


def init_params(feature_dim, conv_hidden, user_embdim, user_count, text_dim, word_dim, n_words):
    """DCUENet(model_type='truedcuemel1dbntext')'s parameters in its RNG order: the BN tower with
    fc(text_dim + d -> d), the user tower, then the text tower (Embedding N(0, 1), the conv's default
    reset, kaiming_uniform_(relu) on its weight)."""
    p, b = O.init_params(feature_dim, conv_hidden, user_embdim, user_count, "truedcuemel1dbn",
                         fc_in=text_dim + feature_dim)
    emb = torch.empty(n_words, word_dim)
    torch.nn.init.normal_(emb)
    w, bias = torch.empty(text_dim, word_dim, 3), torch.empty(text_dim)
    torch.nn.init.kaiming_uniform_(w, a=math.sqrt(5))
    bound = 1.0 / math.sqrt(word_dim * 3)
    torch.nn.init.uniform_(bias, -bound, bound)
    torch.nn.init.kaiming_uniform_(w, nonlinearity="relu")
    p["text.embeddings.weight"] = emb
    p["text.conv.weight"] = w
    p["text.conv.bias"] = bias
    return p, b


def text_features(p, tokens, pad_idx):
    """tokens [M, T] int -> s [M, text_dim]; positions holding PAD are left out of the max."""
    e = p["text.embeddings.weight"][tokens.long()]                      # [M, T, E]
    z = F.conv1d(e.permute(0, 2, 1), p["text.conv.weight"], p["text.conv.bias"], padding=1)  # [M, C, T]
    z = z.masked_fill((tokens == pad_idx).unsqueeze(1), float("-inf"))
    return F.relu(z.max(dim=2).values)


def item_tower(p, b, X, tokens, pad_idx, train=True, route=None):
    """X [M,128,131], tokens [M,T] -> [M,d]."""
    h = O._bn(X, p, b, 0, train)
    for l, (k, pad, pool) in enumerate(O.CONV_SPECS, start=1):
        h = F.conv1d(h, p["conv.layer%d.weight" % l], p["conv.layer%d.bias" % l], padding=pad)
        h = O._bn(O._pool_relu(h, pool, None if route is None else route[l]), p, b, l, train)
    s = text_features(p, tokens, pad_idx)
    x = torch.cat([s, h[:, :, 0]], dim=1)
    return F.linear(x, p["conv.fc.weight"], p["conv.fc.bias"])


def forward(p, b, u, pos, neg, pos_tok, neg_tok, pad_idx, train=True, route=None):
    B, N = neg.shape[0], neg.shape[1]
    uf = O.user_tower(p, u)
    X = torch.cat([pos, neg.reshape(B * N, O.N_MELS, -1)], 0)
    tok = torch.cat([pos_tok.reshape(B, -1), neg_tok.reshape(B * N, -1)], 0)
    feats = item_tower(p, b, X, tok, pad_idx, train, route)
    pf, nf = feats[:B], feats[B:].reshape(B, N, -1)
    pos_cos = F.cosine_similarity(uf, pf, dim=1)
    neg_cos = F.cosine_similarity(uf.unsqueeze(2), nf.permute(0, 2, 1), dim=1)
    return pos_cos[:, None] - neg_cos, uf, pf, nf


def loss_and_grads(p, b, u, pos, neg, pos_tok, neg_tok, pad_idx, margin=0.2, route=None):
    """Hinge loss and the gradient of every trainable parameter (the word vectors are frozen)."""
    leaves = {k: v.detach().clone().requires_grad_(k != "text.embeddings.weight") for k, v in p.items()}
    scores, uf, pf, nf = forward(leaves, b, u, pos, neg, pos_tok, neg_tok, pad_idx, train=True, route=route)
    loss = O.hinge_loss(scores, margin)
    loss.backward()
    grads = {k: v.grad.detach().clone() for k, v in leaves.items() if v.requires_grad}
    return loss.detach(), grads, (scores.detach(), uf.detach(), pf.detach(), nf.detach())


def sentences(gen, n, T, n_words, pad_idx=0, bos=1, eos=2, min_len=1):
    """Synthetic token rows in the reference's shape (dcuelmitemset.py:40-56): BOS, a sentence of
    random word ids (>= 3), EOS, PAD up to T; sentence lengths uniform in [min_len, T - 2]."""
    out = torch.full((n, T), pad_idx, dtype=torch.int32)
    lens = torch.randint(min_len, T - 1, (n,), generator=gen)
    for i in range(n):
        L = int(lens[i])
        out[i, 0] = bos
        out[i, 1:L + 1] = torch.randint(3, n_words, (L,), generator=gen, dtype=torch.int32)
        out[i, L + 1] = eos
    return out
