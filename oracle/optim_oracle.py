"""TEST INFRASTRUCTURE (oracle): the trainer's optimizers' per-element arithmetic, restated in numpy.

Adam (the default), Ranger and SGD + Nesterov (DCUE(optimize=...), nn/dcue.py:143-157).

The reference steps its model with torch.optim.Adam (nn/dcue.py:143-147, :209), i.e. torch 2.10's
`_single_tensor_adam` (torch/optim/adam.py) on CPU float32 tensors. Each tensor op there is a CPU
kernel with its own rounding; this module restates them one by one (fma = one rounding of a*b+c):

    grad.add(param, alpha=wd)                     g = fma(p, wd, g)
    exp_avg.lerp_(grad, 1-b1)                     m = fma(w, g - m, m)           (w < 0.5)
                                                  m = fma(w - 1, g - m, g)       (w >= 0.5)
    exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2)      v = fma((1-b2)*g, g, v*b2)
    (exp_avg_sq.sqrt() / bc2_sqrt).add_(eps)      d = sqrt(v) / bc2_sqrt + eps
    param.addcdiv_(exp_avg, denom, -step_size)    p = p + (-step_size * m) / d

with the Python-float scalars rounded once to float32 (step_size = lr / (1 - b1**t),
bc2_sqrt = (1 - b2**t) ** 0.5). `sqrt` is pluggable: torch's CPU sqrt is not correctly rounded
(its vectorised kernel is 1 ulp off on a fraction of a percent of inputs), the GPU's is.
tests/test_adam_cpu.py pins this restatement against torch.optim.Adam bit for bit (with torch's
sqrt); tests/test_gpu_adam_exact.py holds NativeAdam to it bit for bit (with the exact sqrt).
Only tests/ use this module.
"""
import math

import numpy as np

F32 = np.float32


def fma(a, b, c):
    """float32 fma via an 80-bit intermediate (the product is exact, the sum rounds once more; the
    double rounding this allows never showed on the test inputs)."""
    L = np.longdouble
    return (np.asarray(a, F32).astype(L) * np.asarray(b, F32).astype(L)
            + np.asarray(c, F32).astype(L)).astype(F32)


def exact_sqrt(x):
    return np.sqrt(np.asarray(x, F32))  # IEEE sqrtf: correctly rounded


def torch_cpu_sqrt(x):
    import torch
    return torch.from_numpy(np.ascontiguousarray(x, dtype=F32)).sqrt().numpy()


def scalars(lr, beta1, beta2, eps, wd, step):
    """The float32 constants torch's kernels receive at Adam step `step` (Python-float math)."""
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    w = 1 - beta1
    return dict(neg_step=F32(-(lr / bc1)), w=F32(w), b2=F32(beta2), one_m_b2=F32(1 - beta2),
                bc2_sqrt=F32(bc2 ** 0.5), eps=F32(eps), wd=F32(wd))


def adam_elementwise(p, g, m, v, lr, beta1, beta2, eps, wd, step, sqrt=exact_sqrt):
    """One Adam step of float32 arrays (copies returned: p, m, v)."""
    s = scalars(lr, beta1, beta2, eps, wd, step)
    p, g, m, v = (np.array(a, dtype=F32, copy=True) for a in (p, g, m, v))
    with np.errstate(all="ignore"):
        if wd != 0:
            g = fma(p, s["wd"], g)
        if s["w"] < 0.5:
            m = fma(s["w"], g - m, m)
        else:
            m = fma(s["w"] - F32(1), g - m, g)
        v = fma(s["one_m_b2"] * g, g, v * s["b2"])
        denom = sqrt(v) / s["bc2_sqrt"] + s["eps"]
        p = p + (s["neg_step"] * m) / denom
    return p, m, v


def ranger_scalars(lr, beta1, beta2, eps, wd, step, n_sma_threshold=5):
    """optim/ranger.py:132-154: the RAdam rectification of step `step` (Python-float math, in the
    reference's operation order), and the float32 constants the kernels receive."""
    beta2_t = beta2 ** step
    n_sma_max = 2 / (1 - beta2) - 1
    n_sma = n_sma_max - 2 * step * beta2_t / (1 - beta2_t)
    rect = n_sma > n_sma_threshold
    if rect:
        step_size = math.sqrt((1 - beta2_t) * (n_sma - 4) / (n_sma_max - 4) * (n_sma - 2) / n_sma * n_sma_max
                              / (n_sma_max - 2)) / (1 - beta1 ** step)
    else:
        step_size = 1.0 / (1 - beta1 ** step)
    return dict(rect=rect, b1=F32(beta1), one_m_b1=F32(1 - beta1), b2=F32(beta2), one_m_b2=F32(1 - beta2),
                neg_wd_lr=F32(-wd * lr), neg_step=F32(-step_size * lr), eps=F32(eps))


def ranger_elementwise(p, g, m, v, slow, lr, beta1, beta2, eps, wd, step, k=6, alpha=0.5, sqrt=exact_sqrt):
    """One Ranger step (optim/ranger.py:121-163) of float32 arrays; returns copies (p, m, v, slow).
    `slow` is the lookahead buffer (a copy of p before the first step, :113-114)."""
    s = ranger_scalars(lr, beta1, beta2, eps, wd, step)
    p, g, m, v, slow = (np.array(a, dtype=F32, copy=True) for a in (p, g, m, v, slow))
    with np.errstate(all="ignore"):
        v = fma(s["one_m_b2"] * g, g, v * s["b2"])         # exp_avg_sq.mul_(b2).addcmul_(1-b2, g, g)
        m = fma(g, s["one_m_b1"], m * s["b1"])             # exp_avg.mul_(b1).add_(1-b1, g)
        if wd != 0:
            p = fma(p, s["neg_wd_lr"], p)                  # p.add_(-wd*lr, p)
        if s["rect"]:
            p = p + (s["neg_step"] * m) / (sqrt(v) + s["eps"])   # addcdiv_(-step_size*lr, m, denom)
        else:
            p = fma(m, s["neg_step"], p)                   # p.add_(-step_size*lr, m)
        if step % k == 0:                                   # lookahead (:160-163)
            slow = fma(p - slow, F32(alpha), slow)
            p = slow.copy()
    return p, m, v, slow


def sgd_elementwise(p, g, buf, lr, momentum, wd, step):
    """torch.optim.SGD(momentum, nesterov=True, dampening=0) as nn/dcue.py:148-151 builds it
    (torch/optim/sgd.py _single_tensor_sgd); returns copies (p, buf)."""
    p, g, buf = (np.array(a, dtype=F32, copy=True) for a in (p, g, buf))
    with np.errstate(all="ignore"):
        if wd != 0:
            g = fma(p, F32(wd), g)                          # grad.add(param, alpha=wd)
        if step == 1:
            buf = g.copy()                                  # torch.clone(grad)
        else:
            buf = fma(g, F32(1.0), buf * F32(momentum))     # buf.mul_(m).add_(grad, alpha=1-dampening)
        g = fma(buf, F32(momentum), g)                      # nesterov: grad.add(buf, alpha=m)
        p = fma(g, F32(-lr), p)                             # param.add_(grad, alpha=-lr)
    return p, buf
