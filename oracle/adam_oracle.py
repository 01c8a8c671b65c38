"""TEST INFRASTRUCTURE (oracle): torch.optim.Adam's per-element arithmetic, restated in numpy.

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
