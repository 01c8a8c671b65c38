// torch.optim.Adam's element update and the deferred user-table replay, shared by the HIP kernels
// (adam.hip) and the host check of the replay shortcut (tests/native/adam_replay_check.cpp).
// The includer defines DCUE_RHD (function qualifiers) and the correctly rounded primitives
// rn_fma, rn_mul, rn_add, rn_sub, rn_div, rn_sqrt (float, round-to-nearest-even, no contraction).
//
// Reference: optim.Adam as built at nn/dcue.py:143-147 and stepped at :209, CPU single-tensor path
// (torch/optim/adam.py _single_tensor_adam; each form below was matched bit for bit against torch
// 2.10's CPU kernels on random inputs, tests/test_adam_cpu.py):
//   g = fma(p, wd, g)                      grad.add(param, alpha=wd)
//   m = fma(c, g - m, base)                exp_avg.lerp_(grad, 1-b1): c = w, base = m (w < 0.5),
//                                          else c = w - 1, base = g (the vectorised lerp)
//   v = fma((1-b2)*g, g, v*b2)             exp_avg_sq.mul_(b2).addcmul_(grad, grad, value=1-b2)
//   d = sqrt(v) / bc2_sqrt + eps           (exp_avg_sq.sqrt() / bias_correction2_sqrt).add_(eps)
//   p = p + (step * m) / d                 param.addcdiv_(exp_avg, denom, value=-step_size)
// The one place this cannot be bit-identical is sqrt: the CPU kernel's vectorised sqrt is not
// correctly rounded (1 ulp off on ~0.6% of inputs, tests/test_adam_cpu.py); here it is.
#pragma once

namespace dcue {

struct AdamScalars {
  float neg_step, lerp_c, b2, one_m_b2, bc2_sqrt, eps, wd;  // neg_step = -(lr / bc1)
  float inv_bc2_sqrt;  // RN(1 / bc2_sqrt): Markstein division by the per-step constant
};
static_assert(sizeof(AdamScalars) == 32, "history entry is [8] floats");

// The lerp's blend base is carried by lerp_c's SIGN BIT: lerp_c = w (base m) for a weight w < 0.5
// (beta1 > 0.5), else lerp_c = -(1 - w) (base g) -- a negative zero when w = 1 (beta1 = 0), where the
// lerp returns g itself. launch_adam forms it as -(1 - (float)w), never (float)w - 1, which would
// give +0 at w = 1 and lose the branch.
DCUE_RHD bool lerp_base_g(const AdamScalars& s) { return __builtin_signbit(s.lerp_c); }

DCUE_RHD void adam_elem(float& p, float g, float& m, float& v, const AdamScalars& s) {
  if (s.wd != 0.f) g = rn_fma(p, s.wd, g);
  m = rn_fma(s.lerp_c, rn_sub(g, m), lerp_base_g(s) ? g : m);
  v = rn_fma(rn_mul(s.one_m_b2, g), g, rn_mul(v, s.b2));
  const float denom = rn_add(rn_div(rn_sqrt(v), s.bc2_sqrt), s.eps);
  p = rn_add(p, rn_div(rn_mul(s.neg_step, m), denom));
}

// The zero-gradient step (a row outside the batch, wd == 0, lerp base m: weight < 0.5), bit-identical to
// adam_elem(p, +0, m, v, s): fma((1-b2)*0, 0, v*b2) == v*b2 (v >= 0), and sqrt(v)/bc2_sqrt by
// Markstein's correction with r = RN(1/bc2_sqrt): q = RN(a r), q' = RN(q + RN?(a - q bc2)*r) is the
// correctly rounded quotient for a >= 2^-100 (below it the plain division runs).
DCUE_RHD void adam_zero_elem(float& p, float& m, float& v, const AdamScalars& s) {
  m = rn_fma(s.lerp_c, rn_sub(0.f, m), m);
  v = rn_mul(v, s.b2);
  const float sq = rn_sqrt(v);
  float t;
  if (sq >= 0x1p-100f) {
    const float q = rn_mul(sq, s.inv_bc2_sqrt);
    const float r = rn_fma(-q, s.bc2_sqrt, sq);
    t = rn_fma(r, s.inv_bc2_sqrt, q);
  } else {
    t = rn_div(sq, s.bc2_sqrt);
  }
  const float denom = rn_add(t, s.eps);
  p = rn_add(p, rn_div(rn_mul(s.neg_step, m), denom));
}

// replay of a zero-gradient step: the fast form when no weight decay touches g
DCUE_RHD void adam_replay(float& p, float& m, float& v, const AdamScalars& s, float gz) {
  if (s.wd == 0.f && !lerp_base_g(s) && s.lerp_c < 0.5f)
    adam_zero_elem(p, m, v, s);
  else
    adam_elem(p, gz, m, v, s);
}

// ------------------------------------------------------------------ the long-idle shortcut
// A user row outside the batch for many steps keeps taking zero-gradient steps whose parameter
// update x = RN(RN(neg_step m) / d) shrinks geometrically (m decays by beta1 per step, d does not
// fall below eps), while p stays put: RN(p + x) == p exactly once |x| is below half the smaller
// spacing of floats around p, 2^(e-25) for 2^e <= |p|. Past that point the step changes only m and
// v, whose updates never read p or the per-step lr -- so the replay of the remaining steps is the
// two-operation recurrence m = fma(c, -m, m), v = v * b2, bit for bit what the full step computes.
//
// Sufficient condition, checked before step j of a window whose steps all satisfy `ok` below:
//   S |m_j| <= LB |p| 2^-27
// with S = max |neg_step| over the window, LB = max(eps_min, sqrt(v_j * vdec)) a lower bound of every
// later denominator (d_k >= eps and d_k >= RN(sqrt v_k) since bc2_sqrt <= 1; v_k >= v_j * vdec with
// vdec <= prod b2 (1 - 2^-24)), and |m_k| <= |m_j| for k >= j (lerp weight < 0.5 shrinks m). Then
// |x_k| <= S |m_j| (1 + 2^-24)^2 / LB <= |p| 2^-27 (1 + 2^-21) < |p| 2^-26 < 2^(e-25). The float
// evaluation of the two sides errs by a few 2^-24 relative, well inside the factor-2 margin; |p| is
// kept in [2^-60, 2^100] (normal products, no p = +-0 sign cases, no infinities) and m finite.
struct ReplayBound {
  float S;      // max |neg_step|
  float b2min;  // min b2
  float eps;    // min eps
  float vdec;   // lower bound of v_end / v_start over the window (finalize)
  int ok;       // every step: wd == 0, lerp base m (+0 <= lerp_c < 0.5), eps > 0, 0 <= b2 < 1,
                // 0 < bc2_sqrt <= 1
  int nd;       // every step free of weight decay (and the replayed gradient is +0)
};

DCUE_RHD ReplayBound bound_init(float gz) {
  ReplayBound b;
  b.S = 0.f;
  b.b2min = 1.f;
  b.eps = 0x1p127f;
  b.vdec = 0.f;
  b.ok = gz == 0.f;
  b.nd = gz == 0.f;
  return b;
}

DCUE_RHD void bound_fold(ReplayBound& b, const AdamScalars& s) {
  const float a = s.neg_step < 0.f ? -s.neg_step : s.neg_step;
  b.S = a > b.S ? a : b.S;
  b.b2min = s.b2 < b.b2min ? s.b2 : b.b2min;
  b.eps = s.eps < b.eps ? s.eps : b.eps;
  const int nd = s.wd == 0.f;
  b.nd &= nd;
  b.ok &= nd & !lerp_base_g(s) & (s.lerp_c < 0.5f) & (s.eps > 0.f) & (s.b2 >= 0.f) & (s.b2 < 1.f) &
          (s.bc2_sqrt > 0.f) & (s.bc2_sqrt <= 1.f) & (a <= 0x1p60f);
}

// n = steps in the window: vdec = b2min^n (square-and-multiply, <= 16 roundings of 2^-24 each)
// times 1 - 2^-12, below prod (b2 (1 - 2^-24)) for n <= 4096
DCUE_RHD void bound_finalize(ReplayBound& b, int n) {
  if (n > 4096) b.ok = 0;
  float pw = 1.f, base = b.b2min;
  for (int k = n; k > 0; k >>= 1) {
    if (k & 1) pw *= base;
    base *= base;
  }
  b.vdec = pw * (1.f - 0x1p-12f);
}

DCUE_RHD bool replay_deep(float p, float m, float v, const ReplayBound& b) {
  const float ap = p < 0.f ? -p : p, am = m < 0.f ? -m : m;
  const float vlb = v * b.vdec;
  float lb = b.eps;
  if (vlb > 1e-16f) {
    const float s = rn_sqrt(vlb) * 0.99999f;
    lb = s > lb ? s : lb;
  }
  return (ap >= 0x1p-60f) & (ap <= 0x1p100f) & (am <= 0x1p100f) & (v <= 0x1p126f) &
         (b.S * am <= lb * ap * 0x1p-27f);
}

// Replay the zero-gradient steps j0..j1 (history slots j % cap) of W elements in lockstep; b is the
// bound of a window containing [j0, j1]. Long-idle elements switch to the m/v recurrence (checked
// every fourth step, for all W elements at once).
template <int W>
DCUE_RHD void replay_run(float (&p)[W], float (&m)[W], float (&v)[W], const AdamScalars* hs, int j0, int j1,
                         int cap, const ReplayBound& b, float gz) {
  int j = j0, slot = j0 % cap;  // slot == j % cap throughout (no division in the loops)
  if (b.ok) {
    for (; j <= j1; ++j, slot = slot + 1 == cap ? 0 : slot + 1) {
      if (((j - j0) & 3) == 0) {
        bool deep = true;
#pragma unroll
        for (int w = 0; w < W; ++w) deep &= replay_deep(p[w], m[w], v[w], b);
        if (deep) break;
      }
      const AdamScalars s = hs[slot];
#pragma unroll
      for (int w = 0; w < W; ++w) adam_zero_elem(p[w], m[w], v[w], s);
    }
    for (; j <= j1; ++j, slot = slot + 1 == cap ? 0 : slot + 1) {
      const float lc = hs[slot].lerp_c, b2 = hs[slot].b2;
#pragma unroll
      for (int w = 0; w < W; ++w) {
        m[w] = rn_fma(lc, rn_sub(0.f, m[w]), m[w]);
        v[w] = rn_mul(v[w], b2);
      }
    }
  } else {
    for (; j <= j1; ++j, slot = slot + 1 == cap ? 0 : slot + 1) {
      const AdamScalars s = hs[slot];
#pragma unroll
      for (int w = 0; w < W; ++w) adam_replay(p[w], m[w], v[w], s, gz);
    }
  }
}

// ------------------------------------------------------------------ frozen rows (round 6)
// A row whose every element is long idle for EVERY future step, not only over the current history
// window, needs no history at all: its remaining zero-gradient steps are the m / v recurrence with
// the optimizer's constant (lerp_c, b2), p bit-identical. Such a row is "frozen": bit 30 of its clock
// (emb_step) is set, the rolling slices skip it (no p / m / v traffic) or only refresh its m / v
// with the recurrence now and then, and whoever next reads it replays the recurrence from its clock.
// The future is bounded by an epoch the host keeps (adam.hip frz_before_record): every step of the
// epoch has wd = 0, lerp base m with the epoch's lerp_c < 0.5, the epoch's b2, |neg_step| <= S and
// eps >= eps_min; a step outside it first thaws every frozen row (k_emb_thaw: replayed to the last
// step, the bit cleared). Then the long-idle bound of above holds for any later step k with
// LB = eps_min (d_k >= eps_k >= eps_min): S |m| <= eps_min |p| 2^-27 at freezing time suffices.
constexpr int kFrozenBit = 0x40000000;
DCUE_RHD int clock_of(int e) { return e < 0 ? e : (e & ~kFrozenBit); }
DCUE_RHD bool is_frozen(int e) { return e >= 0 && (e & kFrozenBit) != 0; }

// (m, v) = (+0, +0) (idle: a fixed point), or long idle under every step of the epoch
DCUE_RHD bool frz_elem_ok(float p, float m, float v, float S, float eps_min) {
  if ((__builtin_bit_cast(unsigned, m) | __builtin_bit_cast(unsigned, v)) == 0u) return true;
  const float ap = p < 0.f ? -p : p, am = m < 0.f ? -m : m;
  return (ap >= 0x1p-60f) & (ap <= 0x1p100f) & (am <= 0x1p100f) & (v >= 0.f) & (v <= 0x1p126f) &
         (S * am <= eps_min * ap * 0x1p-27f);
}

// n zero-gradient steps of a frozen element: m = fma(c, -m, m), v = v b2 (replay_run's long-idle
// loop with the epoch's constants)
DCUE_RHD void frz_replay(float& m, float& v, float lc, float b2, int n) {
  for (int k = 0; k < n; ++k) {
    m = rn_fma(lc, rn_sub(0.f, m), m);
    v = rn_mul(v, b2);
  }
}
// the same for W elements in lockstep (independent chains interleaved)
template <int W>
DCUE_RHD void frz_replay_n(float (&m)[W], float (&v)[W], float lc, float b2, int n) {
  for (int k = 0; k < n; ++k) {
#pragma unroll
    for (int w = 0; w < W; ++w) {
      m[w] = rn_fma(lc, rn_sub(0.f, m[w]), m[w]);
      v[w] = rn_mul(v[w], b2);
    }
  }
}

}  // namespace dcue
