"""ORACLE -- CPU restatement of the reference DCUE training step.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and
only as the checker / the timed CPU baseline.  The product path (amplifai-deepcontentrecommenders_amd/)
never imports it and has no CPU fallback.

What it restates (reference = estebandito22/Amplifai-DeepContentRecommenders @ /root/reference):

* parameter construction order + init        dcue/audiomodels/truedcuemel1dbn.py:24-75,
                                              dcue/embeddings/userembedding.py:27-31, dcue/dcue.py:46-68
* item tower (bn0 -> 4x[conv,pool,relu,bn] -> conv,relu,bn -> fc)   truedcuemel1dbn.py:77-101
* user tower (gather, relu, linear, relu, linear)                   userembedding.py:33-44
* DCUENet.forward (concat pos+neg, one conv pass, cosine scores)    dcue/dcue.py:70-108
* hinge loss  mean_b sum_n max(0, margin - s)                       nn/dcue.py:167-170
* torch.optim.Adam (single-tensor CPU form, torch 2.10)             nn/dcue.py:143-147, 209
* in-batch sampler spec                                             nn/dcue.py:698-709
* catalogue negative sampler                                        datasets/dcuedataset.py:207-220

Float math is torch-CPU fp32 (functional ops, autograd for the backward); it is pinned against the
golden vectors under tests/golden/ produced by importing the reference (tests/golden/make_golden.py).
Integer RNG work is also restated in plain C (oracle/mt19937_oracle.c) and pinned the same way.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

N_MELS = 128
N_FRAMES = 131
BN_EPS = 1e-5
BN_MOMENTUM = 0.1

# (kernel, padding, maxpool) per conv layer: truedcuemel1dbn.py:25-61
CONV_SPECS = ((4, 2, 4), (4, 2, 4), (4, 2, 4), (2, 1, 2), (1, 0, 1))


TOWERS = ("truedcuemel1dbn", "truedcuemel1d", "truedcuemel1dres", "truedcuemel1dresbn")


def has_bn(model_type):
    return model_type in ("truedcuemel1dbn", "truedcuemel1dresbn")


def is_res(model_type):
    return model_type in ("truedcuemel1dres", "truedcuemel1dresbn")


def param_names(model_type="truedcuemel1dbn"):
    """Reference parameter order (DCUENet.named_parameters()) of each wired tower
    (dcue/dcue.py:49-59; audiomodels/truedcuemel1d*.py __init__ order)."""
    bn = has_bn(model_type)
    names = ["conv.bn0.weight", "conv.bn0.bias"] if bn else []
    for l in range(1, 6):
        names += ["conv.layer%d.weight" % l, "conv.layer%d.bias" % l]
        if bn:
            names += ["conv.bn%d.weight" % l, "conv.bn%d.bias" % l]
    names += ["conv.fc.weight", "conv.fc.bias", "user_embd.embeddings.weight",
              "user_embd.linear1.weight", "user_embd.linear1.bias",
              "user_embd.linear2.weight", "user_embd.linear2.bias"]
    return names


def init_params(feature_dim, conv_hidden, user_embdim, user_count, model_type="truedcuemel1dbn", fc_in=None):
    """Create parameters + BN buffers consuming torch's global CPU RNG in reference order.

    Order of RNG use in the reference constructors: each Conv1d/Linear default reset
    (kaiming_uniform a=sqrt(5) on the weight, U(+-1/sqrt(fan_in)) on the bias) as the modules are
    built (layer1..layer5, fc), then the explicit kaiming_uniform_(relu) on layer1..5 and
    xavier_uniform_ on fc, then Embedding N(0,1), linear1, linear2 defaults. BatchNorm layers draw
    nothing; the res towers' fc is Linear(4H + d, d) (truedcuemel1dres.py:63-64).
    """
    H, d, E = conv_hidden, feature_dim, user_embdim
    p, b = {}, {}

    def default_reset(w, bias):
        torch.nn.init.kaiming_uniform_(w, a=math.sqrt(5))
        fan_in = w.shape[1] * (w.shape[2] if w.dim() == 3 else 1)
        bound = 1.0 / math.sqrt(fan_in)
        torch.nn.init.uniform_(bias, -bound, bound)

    shapes = [(H, N_MELS, 4), (H, H, 4), (H, H, 4), (H, H, 2), (d, H, 1)]
    chans = [N_MELS, H, H, H, H, d]
    for l in range(6):
        if has_bn(model_type):
            p["conv.bn%d.weight" % l] = torch.ones(chans[l])
            p["conv.bn%d.bias" % l] = torch.zeros(chans[l])
            b["conv.bn%d.running_mean" % l] = torch.zeros(chans[l])
            b["conv.bn%d.running_var" % l] = torch.ones(chans[l])
            b["conv.bn%d.num_batches_tracked" % l] = torch.tensor(0, dtype=torch.long)
        if l < 5:
            w = torch.empty(shapes[l])
            bias = torch.empty(shapes[l][0])
            default_reset(w, bias)
            p["conv.layer%d.weight" % (l + 1)] = w
            p["conv.layer%d.bias" % (l + 1)] = bias
    fi = fc_in if fc_in is not None else 4 * H + d if is_res(model_type) else d
    fcw, fcb = torch.empty(d, fi), torch.empty(d)
    default_reset(fcw, fcb)
    for l in range(1, 6):
        torch.nn.init.kaiming_uniform_(p["conv.layer%d.weight" % l], nonlinearity="relu")
    torch.nn.init.xavier_uniform_(fcw)
    p["conv.fc.weight"], p["conv.fc.bias"] = fcw, fcb
    emb = torch.empty(user_count, E)
    torch.nn.init.normal_(emb)
    p["user_embd.embeddings.weight"] = emb
    for name, shp in (("linear1", (E, E)), ("linear2", (d, E))):
        w, bias = torch.empty(shp), torch.empty(shp[0])
        default_reset(w, bias)
        p["user_embd.%s.weight" % name] = w
        p["user_embd.%s.bias" % name] = bias
    return {k: p[k] for k in param_names(model_type)}, b


def _bn(x, p, b, l, train):
    if "conv.bn%d.weight" % l not in p:  # towers without BatchNorm (truedcuemel1d, ...res)
        return x
    out = F.batch_norm(x, b["conv.bn%d.running_mean" % l], b["conv.bn%d.running_var" % l],
                       p["conv.bn%d.weight" % l], p["conv.bn%d.bias" % l],
                       training=train, momentum=BN_MOMENTUM, eps=BN_EPS)
    if train:
        b["conv.bn%d.num_batches_tracked" % l].add_(1)
    return out


def _pool_relu(h, pool, route):
    """max_pool1d then relu (truedcuemel1dbn.py:80-82 order), or -- with route = (argmax [M,C,Lp],
    live [M,C,Lp]) -- the same pooling with the window argmax and the relu mask given (tests pass
    the GPU's own choices here, so the rest of the step is compared without max-pool near-ties,
    whose routing any 1-ulp difference can flip)."""
    if route is None:
        if pool > 1:
            h = F.max_pool1d(h, pool)
        return F.relu(h)
    idx, live = route
    if pool > 1:
        L = idx.shape[2] * pool
        h = h[:, :, :L].reshape(h.shape[0], h.shape[1], -1, pool).gather(3, idx.unsqueeze(3)).squeeze(3)
    return h * live.to(h.dtype)


def item_tower(p, b, X, train=True, route=None):
    """X [M,128,131] fp32 -> [M,d]: truedcuemel1dbn.py:77-101 (and, by the parameters present, the
    BN-free truedcuemel1d.py and the res towers' truedcuemel1dres(bn).py forward: each block's
    output time-averaged by AvgPool1d over its positions, concatenated with the last block before
    the fc). route: {layer: (argmax, live)}."""
    res = p["conv.fc.weight"].shape[1] != p["conv.fc.weight"].shape[0]  # fc(4H + d -> d)
    h = _bn(X, p, b, 0, train)
    pools = []
    for l, (k, pad, pool) in enumerate(CONV_SPECS, start=1):
        h = F.conv1d(h, p["conv.layer%d.weight" % l], p["conv.layer%d.bias" % l], padding=pad)
        h = _bn(_pool_relu(h, pool, None if route is None else route[l]), p, b, l, train)
        if res and l < 5:
            pools.append(F.avg_pool1d(h, kernel_size=h.shape[2]))
    if res:
        h = torch.cat(pools + [h], dim=1)
    return F.linear(h.permute(0, 2, 1), p["conv.fc.weight"], p["conv.fc.bias"]).squeeze()


def conv_trace(p, b, X):
    """Train-mode item tower returning each conv layer's pre-pool output [M,C,L] (BN running stats
    in `b` are left untouched): the inputs of the max-pool decisions."""
    b = {k: v.clone() for k, v in b.items()}
    out = []
    h = _bn(X, p, b, 0, True)
    for l, (k, pad, pool) in enumerate(CONV_SPECS, start=1):
        h = F.conv1d(h, p["conv.layer%d.weight" % l], p["conv.layer%d.bias" % l], padding=pad)
        out.append(h)
        h = _bn(_pool_relu(h, pool, None), p, b, l, True)
    return out


def user_tower(p, u):
    h = F.relu(p["user_embd.embeddings.weight"][u])
    h = F.relu(F.linear(h, p["user_embd.linear1.weight"], p["user_embd.linear1.bias"]))
    return F.linear(h, p["user_embd.linear2.weight"], p["user_embd.linear2.bias"])


def forward(p, b, u, pos, neg, train=True, route=None):
    """dcue/dcue.py:70-108: one conv pass over cat([pos, neg.view(B*N,...)])."""
    B, N = neg.shape[0], neg.shape[1]
    uf = user_tower(p, u)
    feats = item_tower(p, b, torch.cat([pos, neg.reshape(B * N, N_MELS, -1)], 0), train, route)
    pf, nf = feats[:B], feats[B:].reshape(B, N, -1)
    pos_cos = F.cosine_similarity(uf, pf, dim=1)
    neg_cos = F.cosine_similarity(uf.unsqueeze(2), nf.permute(0, 2, 1), dim=1)
    return pos_cos[:, None] - neg_cos, uf, pf, nf


def hinge_loss(scores, margin=0.2):
    return torch.maximum(torch.zeros_like(scores), margin - scores).sum(dim=1).mean()


def loss_and_grads(p, b, u, pos, neg, margin=0.2, route=None):
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in p.items()}
    scores, uf, pf, nf = forward(leaves, b, u, pos, neg, train=True, route=route)
    loss = hinge_loss(scores, margin)
    loss.backward()
    grads = {k: v.grad.detach().clone() for k, v in leaves.items()}
    return loss.detach(), grads, (scores.detach(), uf.detach(), pf.detach(), nf.detach())


class AdamState:
    """torch.optim.Adam single-tensor semantics (exp_avg lerp form), one param group."""

    def __init__(self, params, betas=(0.9, 0.99), eps=1e-8):
        self.betas, self.eps, self.step_count = betas, eps, 0
        self.m = {k: torch.zeros_like(v) for k, v in params.items()}
        self.v = {k: torch.zeros_like(v) for k, v in params.items()}

    def step(self, params, grads, lr, weight_decay=0.0):
        b1, b2 = self.betas
        self.step_count += 1
        t = self.step_count
        bc1 = 1 - b1 ** t
        bc2_sqrt = (1 - b2 ** t) ** 0.5
        step_size = lr / bc1
        for k, prm in params.items():
            g = grads[k]
            if weight_decay != 0:
                g = g.add(prm, alpha=weight_decay)
            self.m[k].lerp_(g, 1 - b1)
            self.v[k].mul_(b2).addcmul_(g, g, value=1 - b2)
            denom = (self.v[k].sqrt() / bc2_sqrt).add_(self.eps)
            prm.addcdiv_(self.m[k], denom, value=-step_size)


def train_step(p, b, adam, u, pos, neg, lr, weight_decay=0.0, margin=0.2):
    """One reference train step (nn/dcue.py:202-210): fwd, hinge, bwd, Adam."""
    loss, grads, _ = loss_and_grads(p, b, u, pos, neg, margin)
    adam.step(p, grads, lr, weight_decay)
    return loss


# ----------------------------------------------------------------------------------- samplers

def inbatch_negatives(rs, B, N):
    """nn/dcue.py:698-709 spec on a numpy RandomState: one choice() per (i, j), row-major."""
    r = np.empty((B, N), dtype=np.int64)
    for i in range(B):
        others = np.concatenate([np.arange(0, i), np.arange(i + 1, B)])
        for j in range(N):
            r[i, j] = rs.choice(others)
    return r


def user_nonitems(split_items, user_items):
    """datasets/dcuedataset.py:216-218: sorted split items the user never interacted with."""
    split_items = np.asarray(split_items)
    return split_items[~np.isin(split_items, user_items)]


def catalogue_negatives(rs, split_items, user_items_list, N, reseed=None):
    """datasets/dcuedataset.py:207-220; `reseed` mirrors random_seed (np.random.seed per sample)."""
    out = np.empty((len(user_items_list), N), dtype=np.int64)
    for i, items in enumerate(user_items_list):
        if reseed is not None:
            rs.seed(reseed)
        out[i] = rs.choice(user_nonitems(split_items, items), N)
    return out
