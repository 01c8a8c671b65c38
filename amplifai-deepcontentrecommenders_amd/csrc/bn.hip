// BatchNorm1d: bn0's batch statistics over the gathered spectrograms, and the eval-mode constants --
// gfx950. The other layers' sums are accumulated by the kernels that produce them (bnacc.h).
// Reference: the six nn.BatchNorm1d of truedcuemel1dbn.py:24-61 (torch BN semantics: biased variance
// to normalise, unbiased variance into running_var, momentum 0.1, eps 1e-5).
#include "dcue_internal.h"

namespace dcue {

// --------------------------------------------------------------------------- BN statistics
// bn0 input statistics over the gathered spectrograms, weighted by item copy counts (acc; nullable)
// and the per-mel range of the raw input (range; nullable: [0][c] max ord(x), [1][c] max ord(-x),
// ordered keys, kRngC apart) -- what layer 1's split-f16 forward scales its operand by (conv.hip).
template <int SRC>
__global__ __launch_bounds__(256) void k_input_stats(const void* tracks, const int32_t* item_track,
                                                     const float* counts, int M, int rows_per_blk,
                                                     unsigned long long* acc, unsigned* range) {
  critical_path_priority();
  __shared__ float red[8][2][kMels];
  __shared__ float rmx[8][2][kMels];
  const int q = threadIdx.x & 31, slot = threadIdx.x >> 5;
  const long rows = (long)M * kFrames;
  const long r0 = (long)blockIdx.x * rows_per_blk;
  const long r1 = min(r0 + rows_per_blk, rows);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f), ss = s;
  float4 hi = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY), nlo = hi;  // max x, max -x
  constexpr int FB = 4;  // rows in flight per thread
  for (long rb = r0 + slot; rb < r1; rb += 8 * FB) {
    long trk[FB];
    int pp[FB];
    float w[FB];
    uint2 raw16[FB];
    float4 raw32[FB];
#pragma unroll
    for (int j = 0; j < FB; ++j) {
      const long r = rb + 8 * j;
      const long i = r / kFrames;
      pp[j] = (int)(r - i * kFrames);
      trk[j] = r < r1 ? item_track[i] : -1;
      w[j] = r < r1 ? (counts ? counts[i] : 1.f) : 0.f;
    }
#pragma unroll
    for (int j = 0; j < FB; ++j) {
      if (trk[j] < 0) continue;
      const long off = (trk[j] * kFrames + pp[j]) * kMels + 4 * q;
      if constexpr (SRC == SRC_TRACK_F16)
        raw16[j] = *reinterpret_cast<const uint2*>(reinterpret_cast<const __half*>(tracks) + off);
      else
        raw32[j] = ld4(reinterpret_cast<const float*>(tracks) + off);
    }
#pragma unroll
    for (int j = 0; j < FB; ++j) {
      if (trk[j] < 0) continue;
      float x[4];
      if constexpr (SRC == SRC_TRACK_F16) {
        const __half2 h0 = *reinterpret_cast<const __half2*>(&raw16[j].x);
        const __half2 h1 = *reinterpret_cast<const __half2*>(&raw16[j].y);
        x[0] = __low2float(h0); x[1] = __high2float(h0); x[2] = __low2float(h1); x[3] = __high2float(h1);
      } else {
        x[0] = raw32[j].x; x[1] = raw32[j].y; x[2] = raw32[j].z; x[3] = raw32[j].w;
      }
      const float ww = w[j];
      s.x += ww * x[0]; s.y += ww * x[1]; s.z += ww * x[2]; s.w += ww * x[3];
      ss.x += ww * x[0] * x[0]; ss.y += ww * x[1] * x[1]; ss.z += ww * x[2] * x[2]; ss.w += ww * x[3] * x[3];
      hi.x = fmaxf(hi.x, x[0]); hi.y = fmaxf(hi.y, x[1]); hi.z = fmaxf(hi.z, x[2]); hi.w = fmaxf(hi.w, x[3]);
      nlo.x = fmaxf(nlo.x, -x[0]); nlo.y = fmaxf(nlo.y, -x[1]); nlo.z = fmaxf(nlo.z, -x[2]); nlo.w = fmaxf(nlo.w, -x[3]);
    }
  }
  st4(&red[slot][0][4 * q], s);
  st4(&red[slot][1][4 * q], ss);
  st4(&rmx[slot][0][4 * q], hi);
  st4(&rmx[slot][1][4 * q], nlo);
  __syncthreads();
  {
    const int c = threadIdx.x & 127, which = threadIdx.x >> 7;
    float v = 0.f, m = -INFINITY;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      v += red[k][which][c];
      m = fmaxf(m, rmx[k][which][c]);
    }
    if (acc) acc128_add(acc_at(acc, kMels, which, c), v);
    if (range && m > -INFINITY) atomicMax(range + which * kRngC + c, ord_key(m));
  }
}

int launch_input_stats(int src, const void* tracks, const int32_t* item_track, const float* counts,
                       int M, unsigned long long* acc, unsigned* range, hipStream_t s) {
  const long rows = (long)M * kFrames;
  int nb = (int)((rows + 31) / 32);  // short per-block row loops: the gather is latency-bound
  if (nb > 256) nb = 256;
  const int rpb = (int)((rows + nb - 1) / nb);
  nb = (int)((rows + rpb - 1) / rpb);
  if (src == SRC_TRACK_F16)
    DCUE_LAUNCH(k_input_stats<SRC_TRACK_F16>, dim3(nb), dim3(256), 0, s, tracks, item_track,
                       counts, M, rpb, acc, range);
  else
    DCUE_LAUNCH(k_input_stats<SRC_TRACK_F32>, dim3(nb), dim3(256), 0, s, tracks, item_track,
                       counts, M, rpb, acc, range);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

// eval mode (model.eval()): the running statistics normalise
__global__ void k_bn_eval(int C, const float* gamma, const float* rmean, const float* rvar, float* mean,
                          float* invstd, float* a) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float is = 1.f / sqrtf(rvar[c] + 1e-5f);
  mean[c] = rmean[c];
  invstd[c] = is;
  a[c] = gamma[c] * is;
}

int launch_bn_eval(int C, const float* gamma, const float* rmean, const float* rvar, float* mean,
                   float* invstd, float* a, hipStream_t s) {
  DCUE_LAUNCH(k_bn_eval, dim3((C + 255) / 256), dim3(256), 0, s, C, gamma, rmean, rvar, mean, invstd, a);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

// ----------------------------------------------------------------- tower variants (dcue_dims.tower)
struct BnIdentity {
  float* mean[6];
  float* invstd[6];
  float* a[6];
  float *ones, *zeros;
  int C[6];
  int cmax;
};

// truedcuemel1d / truedcuemel1dres have no BatchNorm: every kernel that normalises reads mean 0 and
// a = invstd = 1 (x = (y - 0) * 1 + 0), and gamma / beta operands read ones / zeros
__global__ void k_bn_identity(BnIdentity b) {
  for (int c = threadIdx.x; c < b.cmax; c += blockDim.x) {
    b.ones[c] = 1.f;
    b.zeros[c] = 0.f;
  }
  for (int l = 0; l < 6; ++l)
    for (int c = threadIdx.x; c < b.C[l]; c += blockDim.x) {
      b.mean[l][c] = 0.f;
      b.invstd[l][c] = 1.f;
      b.a[l][c] = 1.f;
    }
}

int launch_bn_identity(float* const* mean, float* const* invstd, float* const* a, float* ones, float* zeros,
                       int cmax, int H, int D, hipStream_t s) {
  BnIdentity b = {};
  for (int l = 0; l < 6; ++l) {
    b.mean[l] = mean[l];
    b.invstd[l] = invstd[l];
    b.a[l] = a[l];
    b.C[l] = l == 0 ? kMels : l == 5 ? D : H;
  }
  b.ones = ones;
  b.zeros = zeros;
  b.cmax = cmax;
  DCUE_LAUNCH(k_bn_identity, dim3(1), dim3(256), 0, s, b);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

struct TimepoolArgs {
  const float* y[6];
  const float* mean[6];
  const float* a[6];
  const float* beta[6];  // nullable (0)
  BnPublish p5;          // train + BN: BN_5 from its accumulators (this kernel is its first consumer)
  int M, H, HL, D;       // y_l channel stride H (storage); xfc block width HL (the reference's H)
  int off5, ld;          // bn5(y5)'s first column and the row stride of xfc
  float* xfc;
};

// The res towers' fc input, one workgroup per item (truedcuemel1dres.py:86-97, ...resbn.py:82-107):
// tp_l = AvgPool1d(Lp_l)(bn_l(y_l)) for blocks 1-4 -- each position normalised, then the mean over
// the block's Lp positions (sum in position order / Lp) -- then bn_5(y_5).
__global__ __launch_bounds__(256) void k_timepool(TimepoolArgs t) {
  __shared__ float m5[256], a5[256];
  const int i = blockIdx.x, H = t.H, HL = t.HL, D = t.D;
  for (int c = threadIdx.x; c < D; c += blockDim.x) {
    if (t.p5.acc) {
      const BnChan st = bn_chan_train(t.p5.acc, D, c, t.p5.count, t.p5.inv_count);
      m5[c] = st.mean;
      a5[c] = t.p5.gamma[c] * st.invstd;
    } else {
      m5[c] = t.mean[5][c];
      a5[c] = t.a[5][c];
    }
  }
  if (i == 0) bn_publish(t.p5, threadIdx.x);
  __syncthreads();
  for (int cc = threadIdx.x; cc < 4 * HL + D; cc += blockDim.x) {
    const int col = cc < 4 * HL ? cc : t.off5 + (cc - 4 * HL);
    float v;
    if (cc < 4 * HL) {
      const int l = col / HL + 1, c = col - (l - 1) * HL;
      const int lp = layer_geom(l).lp;
      const float mu = t.mean[l][c], sc = t.a[l][c], be = t.beta[l] ? t.beta[l][c] : 0.f;
      const float* yl = t.y[l] + (long)i * lp * H + c;
      float acc = 0.f;
      for (int q = 0; q < lp; ++q) acc += (yl[(long)q * H] - mu) * sc + be;
      v = acc / (float)lp;
    } else {
      const int c = cc - 4 * HL;
      v = (t.y[5][(long)i * D + c] - m5[c]) * a5[c] + (t.beta[5] ? t.beta[5][c] : 0.f);
    }
    t.xfc[(long)i * t.ld + col] = v;
  }
}

int launch_timepool(float* const* y, float* const* mean, float* const* a, const float* beta1, const float* beta2,
                    const float* beta3, const float* beta4, const float* beta5, const BnPublish& p5, int M, int H,
                    int HL, int D, int off5, int ld, float* xfc, hipStream_t s) {
  if (D > 256) return DCUE_ERR_UNSUPPORTED;
  TimepoolArgs t = {};
  for (int l = 1; l <= 5; ++l) {
    t.y[l] = y[l];
    t.mean[l] = mean[l];
    t.a[l] = a[l];
  }
  t.beta[1] = beta1; t.beta[2] = beta2; t.beta[3] = beta3; t.beta[4] = beta4; t.beta[5] = beta5;
  t.p5 = p5;
  t.M = M; t.H = H; t.HL = HL; t.D = D;
  t.off5 = off5; t.ld = ld;
  t.xfc = xfc;
  DCUE_LAUNCH(k_timepool, dim3((unsigned)M), dim3(256), 0, s, t);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

}  // namespace dcue
