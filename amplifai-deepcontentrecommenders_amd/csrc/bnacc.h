// Exact, order-independent BatchNorm sums accumulated by the kernels that produce the data.
//
// Train-mode BatchNorm needs per-channel sums over the whole batch (forward: Σc·y, Σc·y²; backward:
// Σg, Σg·x̂) before anything downstream can run. Rather than a partials pass + finalize launch per
// layer, the producing kernel (conv epilogue, input-stats, dgrad epilogue, fc backward) adds its
// per-workgroup fp32 partial sums into fixed-point accumulators of resolution 2^-64 (two int64
// words, see acc128_add) with two non-returning integer atomics. Integer addition is associative,
// so the totals -- and everything computed from them -- are bit-identical run to run whatever
// order the workgroups finish in. Every fp32 value of magnitude >= 2^-40 converts exactly; smaller
// ones are floored at 2^-64. Consumers finalize a channel on the fly from the two accumulators with one
// shared formula (bn_chan_train), so every kernel sees the same mean / invstd bits.
#pragma once

#include "dcue_common.h"

namespace dcue {

// One accumulator = two int64 words. A value v is the integer X = v * 2^64 (exact for |v| >= 2^-40,
// floor at 2^-64 below), split as X = hi * 2^40 + lo with 0 <= lo < 2^40: lo goes to a[0], hi to
// a[1]. Neither word can carry into the other (a[0] stays below 2^40 x the number of adds), so the
// two atomics are independent and non-returning. Total range |sum| < 2^39.
__device__ __forceinline__ void acc128_add(unsigned long long* a, float v) {
  if (v == 0.f) return;
  int e;
  const float fr = frexpf(v, &e);                  // v = fr * 2^e, 0.5 <= |fr| < 1
  const long long m = (long long)ldexpf(fr, 24);  // exact signed 24-bit mantissa
  const int sh = e + 40;                           // X = v * 2^64 = m * 2^sh
  long long hi, lo;
  if (sh >= 40) {
    hi = m << (sh - 40);
    lo = 0;
  } else {
    const long long x = sh >= 0 ? (m << sh) : (sh > -63 ? (m >> -sh) : (m < 0 ? -1ll : 0ll));
    hi = x >> 40;                                  // floor
    lo = x - (hi << 40);                           // 0 <= lo < 2^40
  }
  if (lo) atomicAdd(a, (unsigned long long)lo);
  if (hi) atomicAdd(a + 1, (unsigned long long)hi);
}

__device__ __forceinline__ double acc128_words(unsigned long long lo, unsigned long long hi) {
  return (double)(long long)hi * 0x1p-24 + (double)lo * 0x1p-64;
}
__device__ __forceinline__ double acc128_value(const unsigned long long* a) { return acc128_words(a[0], a[1]); }

// Accumulator block of one BN layer: [2 sums][C channels][2 words].
__device__ __forceinline__ unsigned long long* acc_at(unsigned long long* acc, int C, int which, int c) {
  return acc + ((size_t)which * C + c) * 2;
}
__device__ __forceinline__ double acc_sum(const unsigned long long* acc, int C, int which, int c) {
  return acc128_value(acc + ((size_t)which * C + c) * 2);
}

// Train-mode statistics of channel c (torch BatchNorm1d: biased variance normalises).
struct BnChan {
  float mean, invstd, var;
  double var_unbiased;
};
// ... from the channel's two sums (s = sum x, ss = sum x^2)
__device__ __forceinline__ BnChan bn_chan_sums(double s, double ss, double count, double inv_count) {
  const double m = s * inv_count;
  double v = ss * inv_count - m * m;
  if (v < 0.0) v = 0.0;
  BnChan r;
  r.mean = (float)m;
  r.var = (float)v;
  r.invstd = 1.f / sqrtf(r.var + 1e-5f);
  r.var_unbiased = count > 1.0 ? v * count / (count - 1.0) : v;
  return r;
}
__device__ __forceinline__ BnChan bn_chan_train(const unsigned long long* acc, int C, int c, double count,
                                                double inv_count) {
  return bn_chan_sums(acc_sum(acc, C, 0, c), acc_sum(acc, C, 1, c), count, inv_count);
}

// Where a forward consumer publishes a finalized BN layer (its block 0 does it once per step):
// mean / invstd / gamma*invstd for the backward, and the running-statistics update.
struct BnPublish {
  const unsigned long long* acc;  // null: the consumer reads `mean/invstd/a` (eval or finalized)
  double count;                   // copies x positions
  double inv_count;               // 1 / count (host-rounded; every consumer multiplies by it)
  const float* gamma;
  const float* beta;              // nullable (0)
  float *mean, *invstd, *a;       // published buffers
  float *rmean, *rvar;            // running statistics
  int64_t* nbt;                   // num_batches_tracked
  int C;
  float* beta_out;                // nullable: the step's beta, snapshotted for the backward (a split
                                  // plan's Adam may update the parameter while side streams still read it)
};

__device__ __forceinline__ void bn_publish(const BnPublish& p, int tid) {
  if (!p.acc || tid >= p.C) return;
  const BnChan s = bn_chan_train(p.acc, p.C, tid, p.count, p.inv_count);
  p.mean[tid] = s.mean;
  p.invstd[tid] = s.invstd;
  if (p.beta_out) p.beta_out[tid] = p.beta ? p.beta[tid] : 0.f;
  p.a[tid] = p.gamma[tid] * s.invstd;
  const float momentum = 0.1f;
  p.rmean[tid] = (1.f - momentum) * p.rmean[tid] + momentum * s.mean;
  p.rvar[tid] = (1.f - momentum) * p.rvar[tid] + momentum * (float)s.var_unbiased;
  if (tid == 0) p.nbt[0] += 1;
}

}  // namespace dcue
