// Host check of the deferred user-table Adam replay (csrc/adam_replay.h): replay_run -- with its
// long-idle shortcut -- against the plain step-by-step zero-gradient replay, bit for bit, on random
// and adversarial (p, m, v) states and Adam schedules. Built and run by tests/test_adam_replay_cpu.py
// with g++ -O2 -ffp-contract=off (every float op rounded on its own, as in adam.hip).
//
// Also measures the margin the shortcut leaves: for every element that took it, the largest
// |x_k| / 2^(e-25) over the steps it skipped (x_k the update the full step would have added to p,
// 2^e <= |p|); it must stay below 1 (the proof in adam_replay.h bounds it by 1/2 + 2^-22).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#define DCUE_RHD static inline
namespace dcue {
DCUE_RHD float rn_fma(float a, float b, float c) { return std::fma(a, b, c); }
DCUE_RHD float rn_mul(float a, float b) { return a * b; }
DCUE_RHD float rn_add(float a, float b) { return a + b; }
DCUE_RHD float rn_sub(float a, float b) { return a - b; }
DCUE_RHD float rn_div(float a, float b) { return a / b; }
DCUE_RHD float rn_sqrt(float a) { return std::sqrt(a); }
}  // namespace dcue
#include "dcue.h"
#include "adam_replay.h"

using namespace dcue;

static uint32_t bits(float x) {
  uint32_t u;
  std::memcpy(&u, &x, 4);
  return u;
}

// the scalars launch_adam (adam.hip) forms for step t
static AdamScalars scalars(double lr, double b1, double b2, double eps, int t) {
  const double bc1 = 1.0 - std::pow(b1, (double)t), bc2 = 1.0 - std::pow(b2, (double)t);
  const double w = 1.0 - b1;
  AdamScalars s;
  s.neg_step = (float)(-(lr / bc1));
  s.lerp_c = w < 0.5 ? (float)w : -(1.0f - (float)w);  // as launch_adam (sign bit = base g)
  s.b2 = (float)b2;
  s.one_m_b2 = (float)(1.0 - b2);
  s.bc2_sqrt = (float)std::pow(bc2, 0.5);
  s.eps = (float)eps;
  s.wd = 0.f;
  s.inv_bc2_sqrt = 1.0f / s.bc2_sqrt;
  return s;
}

int main(int argc, char** argv) {
  const long cases = argc > 1 ? std::atol(argv[1]) : 100000;
  const unsigned seed = argc > 2 ? (unsigned)std::atol(argv[2]) : 1u;
  std::mt19937_64 rng(seed);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  auto pick = [&](int n) { return (int)(rng() % (unsigned)n); };
  auto logu = [&](double lo, double hi) { return std::pow(10.0, lo + (hi - lo) * U(rng)); };
  auto sgn = [&]() { return (rng() & 1) ? 1.0 : -1.0; };

  AdamScalars hs[DCUE_MAX_LOG_CAP];
  long deep_elems = 0, elems = 0, steps_total = 0, steps_short = 0, mismatches = 0;
  double worst = 0.0;
  for (long c = 0; c < cases; ++c) {
    const int cap = 1 + pick(DCUE_MAX_LOG_CAP);
    // beta1 <= 0.5 (lerp weight >= 0.5, base g; 0 -> weight 1) as well as the usual > 0.5
    const double b1s[4] = {0.0, 0.3, 0.5, 0.5 + 0.49 * U(rng)};
    const double b1 = pick(3) ? 0.9 : b1s[pick(4)];
    const double b2 = pick(3) ? (pick(2) ? 0.99 : 0.999) : 0.9 + 0.0999 * U(rng);
    const double eps = pick(4) ? 1e-8 : logu(-12, -4);
    const double lr_hi = logu(-5, -1);
    const int t0 = pick(2) ? 1 + pick(300) : 1 + pick(200000);
    // window [lo, T] (absolute steps), history slots j % cap
    const int n = 1 + pick(cap);
    const int lo = t0, T = t0 + n - 1;
    for (int j = lo; j <= T; ++j) {
      const double ph = std::cos(3.14159 * (j % 97) / 97.0);
      hs[j % cap] = scalars(lr_hi * (0.5 + 0.5 * ph) + 1e-7, b1, b2, eps, j);
    }
    ReplayBound b = bound_init(0.f);
    for (int j = lo; j <= T; ++j) bound_fold(b, hs[j % cap]);
    bound_finalize(b, n);
    const int j0 = lo + pick(n);

    float p[4], m[4], v[4];
    const int mode = pick(6);
    for (int w = 0; w < 4; ++w) {
      double pv = sgn() * logu(-3, 1), g = sgn() * logu(-9, 2);
      double mv = g * (1.0 - b1) * logu(-1, 1), vv = g * g * (1.0 - b2) * logu(-2, 2);
      switch (mode) {
        case 0: break;
        case 1:  // long-idle states: m decayed far below sqrt(v)
          mv *= std::pow(b1, 50 + pick(800));
          vv *= std::pow(b2, pick(800));
          break;
        case 2: {  // p at a binade edge, m around the shortcut's threshold
          pv = sgn() * std::ldexp(1.0, -20 + pick(24));
          const double lb = std::fmax(eps, std::sqrt(vv * b.vdec));
          mv = sgn() * lb * std::fabs(pv) * std::ldexp(1.0, -27) / b.S * (0.25 + 4.0 * U(rng));
          break;
        }
        case 3:  // tiny / zero / subnormal p and moments
          pv = pick(3) == 0 ? 0.0 : sgn() * std::ldexp(1.0, -55 - pick(95));
          mv = pick(2) ? 0.0 : sgn() * std::ldexp(1.0, -120 - pick(29));
          vv = pick(2) ? 0.0 : std::ldexp(1.0, -125 - pick(24));
          break;
        case 4:  // large magnitudes
          pv = sgn() * logu(10, 30);
          mv = sgn() * logu(-30, 20);
          vv = logu(-40, 36);
          break;
        default:  // the same element state across the lanes
          break;
      }
      p[w] = (float)pv;
      m[w] = (float)mv;
      v[w] = (float)vv;
      if (mode == 5 && w > 0) { p[w] = p[0]; m[w] = m[0]; v[w] = v[0]; }
    }
    // reference: every step in full
    float rp[4], rm[4], rv[4];
    for (int w = 0; w < 4; ++w) {
      rp[w] = p[w]; rm[w] = m[w]; rv[w] = v[w];
      // the full Adam step with g = +0 -- what the dense sweep computes for a row outside the batch
      for (int j = j0; j <= T; ++j) adam_elem(rp[w], 0.f, rm[w], rv[w], hs[j % cap]);
    }
    // margin: where replay_run switches, the largest skipped update relative to 2^(e-25)
    if (b.ok) {
      float qp[4], qm[4], qv[4];
      std::memcpy(qp, p, sizeof p); std::memcpy(qm, m, sizeof m); std::memcpy(qv, v, sizeof v);
      int j = j0;
      for (; j <= T; ++j) {
        if (((j - j0) & 3) == 0) {
          bool deep = true;
          for (int w = 0; w < 4; ++w) deep &= replay_deep(qp[w], qm[w], qv[w], b);
          if (deep) break;
        }
        for (int w = 0; w < 4; ++w) adam_zero_elem(qp[w], qm[w], qv[w], hs[j % cap]);
      }
      if (j <= T) {
        deep_elems += 4;
        steps_short += 4L * (T - j + 1);
        for (int w = 0; w < 4; ++w) {
          int e;
          std::frexp(qp[w], &e);  // |p| in [2^(e-1), 2^e)
          const double half = std::ldexp(1.0, e - 1 - 25);
          float pp = qp[w], mm = qm[w], vv = qv[w];
          for (int k = j; k <= T; ++k) {
            const AdamScalars& s = hs[k % cap];
            mm = rn_fma(s.lerp_c, rn_sub(0.f, mm), mm);
            vv = rn_mul(vv, s.b2);
            const float sq = rn_sqrt(vv);
            const float t = sq >= 0x1p-100f ? rn_fma(rn_fma(-rn_mul(sq, s.inv_bc2_sqrt), s.bc2_sqrt, sq),
                                                     s.inv_bc2_sqrt, rn_mul(sq, s.inv_bc2_sqrt))
                                            : rn_div(sq, s.bc2_sqrt);
            const float x = rn_div(rn_mul(s.neg_step, mm), rn_add(t, s.eps));
            const double r = std::fabs((double)x) / half;
            if (r > worst) worst = r;
            if (rn_add(pp, x) != pp) {
              std::printf("shortcut skipped a step that moves p: case %ld lane %d p=%a x=%a\n", c, w, pp, x);
              ++mismatches;
            }
          }
        }
      }
    }
    // product path
    replay_run<4>(p, m, v, hs, j0, T, cap, b, 0.f);
    elems += 4;
    steps_total += 4L * (T - j0 + 1);
    for (int w = 0; w < 4; ++w) {
      if (bits(p[w]) != bits(rp[w]) || bits(m[w]) != bits(rm[w]) || bits(v[w]) != bits(rv[w])) {
        if (mismatches < 10)
          std::printf("MISMATCH case %ld mode %d lane %d: p %a vs %a, m %a vs %a, v %a vs %a\n", c, mode, w,
                      p[w], rp[w], m[w], rm[w], v[w], rv[w]);
        ++mismatches;
      }
    }
  }
  // Frozen rows (adam_replay.h, round 6): an element that passes frz_elem_ok under an epoch (S bounds
  // every later |neg_step|, eps_min every later eps, lerp_c / b2 fixed) takes any number of later
  // zero-gradient steps of that epoch -- lr, eps and bc2 varying within it -- with p unchanged and
  // m / v exactly frz_replay's recurrence. Reference: adam_elem step by step.
  long frz_elems = 0, frz_steps = 0, frz_mism = 0;
  for (long c = 0; c < cases; ++c) {
    const double b1 = pick(4) ? 0.9 : 0.5 + 0.49 * U(rng);
    const double b2 = pick(3) ? (pick(2) ? 0.99 : 0.999) : 0.9 + 0.0999 * U(rng);
    const double eps_min = pick(4) ? 1e-8 : logu(-12, -4);
    const double lr_hi = logu(-5, -1);
    const AdamScalars s1 = scalars(lr_hi, b1, b2, eps_min, 1);
    const float S = std::fabs(s1.neg_step), lc = s1.lerp_c, fb2 = s1.b2;
    float p = (float)(sgn() * logu(-3, 1)), m, v;
    const double g = logu(-9, 1);
    v = (float)(g * g * (1.0 - b2) * logu(-3, 2));
    switch (pick(4)) {
      case 0:  // just inside the freeze threshold
        m = (float)(sgn() * (double)eps_min * std::fabs((double)p) * std::ldexp(1.0, -27) / S * (0.5 + 0.5 * U(rng)));
        break;
      case 1:  // far below it
        m = (float)(sgn() * (double)eps_min * std::fabs((double)p) * std::ldexp(1.0, -27) / S * logu(-6, -1));
        break;
      case 2:  // binade-edge p, at the threshold
        p = (float)(sgn() * std::ldexp(1.0, -20 + pick(24)));
        m = (float)(sgn() * (double)eps_min * std::fabs((double)p) * std::ldexp(1.0, -27) / S);
        break;
      default:  // subnormal moments
        m = (float)(sgn() * std::ldexp(1.0, -130 - pick(19)));
        v = pick(2) ? 0.f : (float)std::ldexp(1.0, -128 - pick(20));
        break;
    }
    if (!frz_elem_ok(p, m, v, S, (float)eps_min)) continue;
    ++frz_elems;
    const int t0 = 1 + pick(5000), n = 1 + pick(pick(8) ? 300 : 4000);
    float rp = p, rm = m, rv = v;
    for (int k = 0; k < n; ++k) {  // the epoch's steps: lr <= lr_hi, eps >= eps_min, the same betas
      const double lr = lr_hi * U(rng) + 1e-12;
      const double eps = eps_min * (pick(3) ? 1.0 : 1.0 + 9.0 * U(rng));
      adam_elem(rp, 0.f, rm, rv, scalars(lr, b1, b2, eps, t0 + k));
    }
    float fm = m, fv = v;
    frz_replay(fm, fv, lc, fb2, n);
    frz_steps += n;
    if (bits(rp) != bits(p) || bits(rm) != bits(fm) || bits(rv) != bits(fv)) {
      if (frz_mism < 10)
        std::printf("FROZEN MISMATCH case %ld: p %a -> %a, m %a vs %a, v %a vs %a\n", c, p, rp, rm, fm, rv, fv);
      ++frz_mism;
    }
  }
  std::printf("cases %ld elements %ld element-steps %ld shortcut-elements %ld shortcut-steps %ld "
              "worst-margin %.6f mismatches %ld frozen-elements %ld frozen-steps %ld frozen-mismatches %ld\n",
              cases, elems, steps_total, deep_elems, steps_short, worst, mismatches, frz_elems, frz_steps, frz_mism);
  return mismatches == 0 && frz_mism == 0 && worst < 1.0 ? 0 : 1;
}
