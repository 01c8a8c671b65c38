// BatchNorm1d statistics (train: batch stats weighted by copies + running-stat update; eval:
// running stats) and the backward reductions -- gfx950.
// Reference: the six nn.BatchNorm1d of truedcuemel1dbn.py:24-61 (torch BN semantics: biased variance
// to normalise, unbiased variance into running_var, momentum 0.1, eps 1e-5).
#include "dcue_internal.h"

namespace dcue {

// --------------------------------------------------------------------------- BN statistics
// bn0 input statistics over the gathered spectrograms, weighted by item copy counts.
template <int SRC>
__global__ __launch_bounds__(256) void k_input_stats(const void* tracks, const int32_t* item_track,
                                                     const float* counts, int M, int rows_per_blk,
                                                     float* partials) {
  __shared__ float red[8][2][kMels];
  const int q = threadIdx.x & 31, slot = threadIdx.x >> 5;
  const long rows = (long)M * kFrames;
  const long r0 = (long)blockIdx.x * rows_per_blk;
  const long r1 = min(r0 + rows_per_blk, rows);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f), ss = s;
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
    }
  }
  st4(&red[slot][0][4 * q], s);
  st4(&red[slot][1][4 * q], ss);
  __syncthreads();
  {
    const int c = threadIdx.x & 127, which = threadIdx.x >> 7;
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) v += red[k][which][c];
    partials[((long)blockIdx.x * 2 + which) * kMels + c] = v;
  }
}

int launch_input_stats(int src, const void* tracks, const int32_t* item_track, const float* counts,
                       int M, float* partials, int* nparts, hipStream_t s) {
  const long rows = (long)M * kFrames;
  int nb = (int)((rows + 31) / 32);  // short per-block row loops: the gather is latency-bound
  if (nb > 256) nb = 256;
  const int rpb = (int)((rows + nb - 1) / nb);
  nb = (int)((rows + rpb - 1) / rpb);
  *nparts = nb;
  if (src == SRC_TRACK_F16)
    hipLaunchKernelGGL(k_input_stats<SRC_TRACK_F16>, dim3(nb), dim3(256), 0, s, tracks, item_track,
                       counts, M, rpb, partials);
  else
    hipLaunchKernelGGL(k_input_stats<SRC_TRACK_F32>, dim3(nb), dim3(256), 0, s, tracks, item_track,
                       counts, M, rpb, partials);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

// partials [nparts][2][C] -> mean, invstd, a = gamma*invstd; train mode also updates running stats
// (momentum 0.1, unbiased running variance) and num_batches_tracked, as torch BatchNorm1d does.
// Eval mode (train == 0) takes mean/var from the running stats. Sums are combined in fp64.
// 32 slices x 32 channels per workgroup: short per-thread loops over the partials (latency-bound).
__global__ __launch_bounds__(1024) void k_bn_finalize(const float* __restrict__ partials, int nparts,
                                                      int C, double count, const float* gamma,
                                                      float* rmean, float* rvar, int64_t* nbt,
                                                      int train, float* mean, float* invstd,
                                                      float* a) {
  __shared__ double red[32][2][33];
  const int cl = threadIdx.x & 31, sl = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  double s = 0.0, ss = 0.0;
  if (train && c < C)
    for (int p = sl; p < nparts; p += 32) {
      s += (double)partials[((long)p * 2 + 0) * C + c];
      ss += (double)partials[((long)p * 2 + 1) * C + c];
    }
  red[sl][0][cl] = s;
  red[sl][1][cl] = ss;
  __syncthreads();
  if (sl == 0 && c < C) {
    const float eps = 1e-5f, momentum = 0.1f;
    float mu, var;
    if (train) {
      s = 0.0;
      ss = 0.0;
      for (int k = 0; k < 32; ++k) {
        s += red[k][0][cl];
        ss += red[k][1][cl];
      }
      const double m = s / count;
      double v = ss / count - m * m;
      if (v < 0.0) v = 0.0;
      mu = (float)m;
      var = (float)v;
      const double unbiased = count > 1.0 ? v * count / (count - 1.0) : v;
      rmean[c] = (1.f - momentum) * rmean[c] + momentum * mu;
      rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)unbiased;
      if (c == 0) nbt[0] += 1;
    } else {
      mu = rmean[c];
      var = rvar[c];
    }
    const float is = 1.f / sqrtf(var + eps);
    mean[c] = mu;
    invstd[c] = is;
    a[c] = gamma[c] * is;
  }
}

int launch_bn_finalize(const float* partials, int nparts, int C, double count, const float* gamma,
                       float* rmean, float* rvar, int64_t* nbt, int train, float* mean,
                       float* invstd, float* a, hipStream_t s) {
  hipLaunchKernelGGL(k_bn_finalize, dim3((C + 31) / 32), dim3(1024), 0, s, partials, nparts, C, count,
                     gamma, rmean, rvar, nbt, train, mean, invstd, a);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

// backward partial sums over rows of g and g*xhat (xhat from the stored pre-BN activation).
__global__ __launch_bounds__(256) void k_bwd_partials(const float* __restrict__ g,
                                                      const float* __restrict__ y,
                                                      const float* mean, const float* invstd,
                                                      long rows, int C, int rows_per_blk,
                                                      float* partials) {
  extern __shared__ __attribute__((aligned(16))) float red[];  // [slots][2][C]
  const int quads = C / 4;
  const int nslots = 256 / quads;
  const int q = threadIdx.x % quads, slot = threadIdx.x / quads;
  const long r0 = (long)blockIdx.x * rows_per_blk;
  const long r1 = min(r0 + rows_per_blk, rows);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f), sx = s;
  if (slot < nslots) {
    const float4 mu = ld4(mean + 4 * q), is = ld4(invstd + 4 * q);
    for (long r = r0 + slot; r < r1; r += nslots) {
      const float4 gv = ld4(g + r * C + 4 * q), yv = ld4(y + r * C + 4 * q);
      s.x += gv.x; s.y += gv.y; s.z += gv.z; s.w += gv.w;
      sx.x += gv.x * ((yv.x - mu.x) * is.x);
      sx.y += gv.y * ((yv.y - mu.y) * is.y);
      sx.z += gv.z * ((yv.z - mu.z) * is.z);
      sx.w += gv.w * ((yv.w - mu.w) * is.w);
    }
    st4(&red[(slot * 2 + 0) * C + 4 * q], s);
    st4(&red[(slot * 2 + 1) * C + 4 * q], sx);
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 2 * C; e += 256) {
    const int which = e / C, c = e - which * C;
    float v = 0.f;
    for (int k = 0; k < nslots; ++k) v += red[(k * 2 + which) * C + c];
    partials[((long)blockIdx.x * 2 + which) * C + c] = v;
  }
}

int launch_bwd_partials(const float* g, const float* y, const float* mean, const float* invstd,
                        long rows, int C, float* partials, int* nparts, hipStream_t s) {
  int nb = (int)((rows + 63) / 64);
  if (nb > 512) nb = 512;
  if (nb < 1) nb = 1;
  const int rpb = (int)((rows + nb - 1) / nb);
  nb = (int)((rows + rpb - 1) / rpb);
  if (nb < 1) nb = 1;
  *nparts = nb;
  const int nslots = 256 / (C / 4);
  const size_t lds = (size_t)nslots * 2 * C * sizeof(float);
  hipLaunchKernelGGL(k_bwd_partials, dim3(nb), dim3(256), lds, s, g, y, mean, invstd, rows, C, rpb,
                     partials);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

__global__ __launch_bounds__(1024) void k_bwd_finalize(const float* __restrict__ partials, int nparts,
                                                       int C, float* sD, float* sDx, float* dgamma,
                                                       float* dbeta) {
  __shared__ double red[32][2][33];
  const int cl = threadIdx.x & 31, sl = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  double s = 0.0, sx = 0.0;
  if (c < C)
    for (int p = sl; p < nparts; p += 32) {
      s += (double)partials[((long)p * 2 + 0) * C + c];
      sx += (double)partials[((long)p * 2 + 1) * C + c];
    }
  red[sl][0][cl] = s;
  red[sl][1][cl] = sx;
  __syncthreads();
  if (sl == 0 && c < C) {
    s = 0.0;
    sx = 0.0;
    for (int k = 0; k < 32; ++k) {
      s += red[k][0][cl];
      sx += red[k][1][cl];
    }
    sD[c] = (float)s;
    sDx[c] = (float)sx;
    dbeta[c] = (float)s;   // BN output = gamma*xhat + beta
    dgamma[c] = (float)sx;
  }
}

int launch_bwd_finalize(const float* partials, int nparts, int C, float* sD, float* sDx,
                        float* dgamma, float* dbeta, hipStream_t s) {
  hipLaunchKernelGGL(k_bwd_finalize, dim3((C + 31) / 32), dim3(1024), 0, s, partials, nparts, C, sD,
                     sDx, dgamma, dbeta);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

}  // namespace dcue
